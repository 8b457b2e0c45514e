"""T3 comm tier on one GPU: the peer-mapped all-reduce (csrc/comm/allreduce.hip) with two ranks.

Both ranks live on the same MI355X (the gpurun box has one GPU); the mechanism is the one the
8-GPU node uses -- each rank maps the other's uncached staging region through a hipIpc handle
exchanged over gloo -- only the xGMI hop is replaced by local HBM. Oracle: fp32 sum of both
ranks' bf16 inputs, rounded once (what the kernel computes, in rank order).
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
WORLD = 2
SIZES = [4096, 8 * 4096, 32 * 4096, 1000 * 8, 1 << 20]  # 8 KB .. 2 MB (one-shot and two-shot)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(rank, n, it):
    g = torch.Generator().manual_seed(1000 * rank + 17 * it + n)
    return torch.randn(n, generator=g).bfloat16()


def _worker(rank, port, d):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    torch.cuda.set_device(0)
    from rag_llm_k8s_amd.parallel.ipc_allreduce import IPCAllReduce

    ar = IPCAllReduce(None, None, WORLD, rank, "cuda:0", max_bytes=4 << 20, blocks=32)
    res = {}
    try:
        for n in SIZES:
            for mode in (0, 1):
                outs = []
                for it in range(6):  # several epochs: exercises the double-buffered halves
                    x = _inputs(rank, n, it).cuda()
                    y = torch.empty_like(x)
                    ar.all_reduce(x, out=y, mode=mode)
                    outs.append(y.cpu())
                res[(n, mode)] = outs
        # in place, default mode choice, inside a captured graph
        x = _inputs(rank, 8 * 4096, 99).cuda()
        ar.all_reduce(x)
        res["inplace"] = x.cpu()
        xs = torch.empty(8 * 4096, dtype=torch.bfloat16, device="cuda")
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                ar.all_reduce(xs)
        torch.cuda.current_stream().wait_stream(s)
        graph_out = []
        for it in range(3):
            xs.copy_(_inputs(rank, 8 * 4096, 200 + it).cuda())
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            graph_out.append(xs.cpu().clone())
        res["graph"] = graph_out
        res["error"] = ar.error()
    finally:
        torch.cuda.synchronize()
        dist.barrier()
        ar.close()
        torch.save(res, os.path.join(d, "r%d.pt" % rank))
        dist.destroy_process_group()


def test_ipc_allreduce_two_ranks(native):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker, args=(r, port, d)) for r in range(WORLD)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join()
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        out = [torch.load(os.path.join(d, "r%d.pt" % r), weights_only=False) for r in range(WORLD)]

    def ref(n, it):
        return sum(_inputs(r, n, it).float() for r in range(WORLD)).bfloat16()

    for n in SIZES:
        for mode in (0, 1):
            for it in range(6):
                want = ref(n, it)
                for r in range(WORLD):
                    got = out[r][(n, mode)][it]
                    assert torch.equal(got, want), (n, mode, it, r, (got.float() - want.float()).abs().max())
    for r in range(WORLD):
        assert torch.equal(out[r]["inplace"], ref(8 * 4096, 99))
        for it in range(3):
            assert torch.equal(out[r]["graph"][it], ref(8 * 4096, 200 + it))
        assert out[r]["error"] is False
