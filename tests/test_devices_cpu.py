"""Multi-GPU self-tests that need no GPU: device distinctness (a job claiming N GPUs must not put two
ranks on one device) and the fence policy of the peer-mapped row barriers (always on across devices)."""
import pytest

from rag_llm_k8s_amd.parallel import dist as D
from rag_llm_k8s_amd.parallel.ipc_allreduce import fences_for


def test_distinct_devices_pass():
    ids = ["h/pci:0000:%02x:00" % i for i in range(8)]
    assert D.check_distinct_devices(ids) == []


def test_shared_device_is_refused_unless_allowed():
    ids = ["h/pci:0000:0a:00", "h/pci:0000:0b:00", "h/pci:0000:0a:00", "h/pci:0000:0c:00"]
    with pytest.raises(RuntimeError, match=r"ranks \[\[0, 2\]\] share a GPU"):
        D.check_distinct_devices(ids)
    assert D.check_distinct_devices(ids, allow_shared=True) == [[0, 2]]


def test_same_bus_id_on_two_hosts_is_distinct():
    assert D.check_distinct_devices(["a/pci:0000:0a:00", "b/pci:0000:0a:00"]) == []


def test_cpu_ranks_may_share_the_host():
    assert D.check_distinct_devices(["h/cpu"] * 4) == []


def test_device_identity_cpu():
    assert D.device_identity("cpu").endswith("/cpu")


def test_fence_policy():
    assert fences_for(True, env="") and fences_for(True, env="0") and fences_for(True, env="1")
    assert not fences_for(False, env="") and not fences_for(False, env="0") and fences_for(False, env="1")
