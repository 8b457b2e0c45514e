"""T3 comm tier on one GPU: the peer-mapped all-reduce / all-gather and the fused decode reduction
(csrc/comm/allreduce.hip) with 2, 4 and 8 ranks.

All ranks live on the same MI355X (the gpurun box has one GPU); the mechanism is the one the
8-GPU node uses -- each rank maps every other rank's uncached staging region through a hipIpc
handle exchanged over gloo -- only the xGMI hop is replaced by local HBM. Oracle: fp32 sum of the
ranks' inputs in rank order, rounded once (what the kernels compute).
"""
import os
import sys
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


def _worker(rank, port, d, WORLD=WORLD):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    torch.cuda.set_device(0)
    from rag_llm_k8s_amd.parallel.ipc_allreduce import IPCAllReduce

    ar = IPCAllReduce(None, None, WORLD, rank, "cuda:0", max_bytes=4 << 20, blocks=32, fused_rows=64, fused_h=4096)
    res = {}
    try:
        mine = torch.arange(40, dtype=torch.int32, device="cuda") + 1000 * rank  # all-gather
        res["gather"] = ar.all_gather(mine).cpu()
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


def _spawn(target, world, d, port):
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=target, args=(r, port, d, world)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [torch.load(os.path.join(d, "r%d.pt" % r), weights_only=False) for r in range(world)]


@pytest.mark.parametrize("WORLD", [2, 4, 8])
def test_ipc_allreduce_ranks(native, WORLD):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker, args=(r, port, d, WORLD)) for r in range(WORLD)]
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
        acc = torch.zeros(n)
        for r in range(WORLD):  # rank order, fp32
            acc = acc + _inputs(r, n, it).float()
        return acc.bfloat16()

    for n in SIZES:
        for mode in (0, 1):
            for it in range(6):
                want = ref(n, it)
                for r in range(WORLD):
                    got = out[r][(n, mode)][it]
                    assert torch.equal(got, want), (n, mode, it, r, (got.float() - want.float()).abs().max())
    for r in range(WORLD):
        assert torch.equal(out[r]["gather"], torch.cat([torch.arange(40, dtype=torch.int32) + 1000 * p
                                                        for p in range(WORLD)]))
        assert torch.equal(out[r]["inplace"], ref(8 * 4096, 99))
        for it in range(3):
            assert torch.equal(out[r]["graph"][it], ref(8 * 4096, 200 + it))
        assert out[r]["error"] is False


# ---------------------------------------------------------------- fused decode reduction
H_F = int(os.environ.get("RAGK_TEST_FUSED_H", "4096"))  # set per case by the test before spawning
FUSED_CASES = [(1, 1), (3, 2), (32, 1), (5, 4), (1, 3), (17, 1)]  # (M rows, S slabs): varying grids


def _partials(rank, M, S, it):
    g = torch.Generator().manual_seed(7919 * rank + 131 * M + 17 * S + it)
    return torch.randn(S, M, H_F, generator=g) * 0.05


def _fused_worker(rank, port, d, WORLD):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    torch.cuda.set_device(0)
    from rag_llm_k8s_amd.parallel.ipc_allreduce import IPCAllReduce

    ar = IPCAllReduce(None, None, WORLD, rank, "cuda:0", max_bytes=1 << 20, blocks=16, fused_rows=64, fused_h=H_F)
    ar.set_fences(os.environ.get("RAGK_TEST_FENCES", "0") == "1")  # the cross-device (xGMI) setting
    res = {"fences": ar.fences}
    g = torch.Generator().manual_seed(5)
    w = (1 + 0.1 * torch.randn(H_F, generator=g)).bfloat16().cuda()
    try:
        for mode in (0, 1):
            for it, (M, S) in enumerate(FUSED_CASES):
                h = (torch.randn(M, H_F, generator=torch.Generator().manual_seed(M + it))).bfloat16().cuda()
                P = _partials(rank, M, S, it).cuda()
                out = torch.empty_like(h)
                ar.add_rmsnorm(P, h, w, 1e-5, out, mode=mode)
                res[(mode, it)] = (h.cpu(), out.cpu())
        # captured in a graph, replayed with new partials (row epochs advance inside the graph)
        M, S = 4, 2
        P = torch.zeros(S, M, H_F, device="cuda")
        h = torch.zeros(M, H_F, dtype=torch.bfloat16, device="cuda")
        out = torch.empty_like(h)
        gr = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            with torch.cuda.graph(gr, stream=st):
                ar.add_rmsnorm(P, h, w, 1e-5, out)
        torch.cuda.current_stream().wait_stream(st)
        gl = []
        for it in range(3):
            P.copy_(_partials(rank, M, S, 100 + it).cuda())
            h.copy_(torch.ones(M, H_F).bfloat16())
            dist.barrier()
            gr.replay()
            torch.cuda.synchronize()
            gl.append((h.cpu().clone(), out.cpu().clone()))
        res["graph"] = gl
        res["error"] = ar.error()
    finally:
        torch.cuda.synchronize()
        dist.barrier()
        ar.close()
        torch.save(res, os.path.join(d, "r%d.pt" % rank))
        dist.destroy_process_group()


@pytest.mark.parametrize("WORLD,H,fences", [(2, 4096, 0), (4, 4096, 0), (8, 4096, 0), (8, 8192, 0), (4, 8192, 1),
                                             (8, 4096, 1)])
def test_fused_allreduce_add_rmsnorm(native, WORLD, H, fences, monkeypatch):
    """h <- bf16(h + bf16(sum over ranks (rank order) of sum over slabs (slab order) of P)), out = rmsnorm(h):
    the residual stream is exact vs an fp32 oracle, identical on every rank (bit for bit) in both the
    one-shot and the two-shot mode, for varying row counts, and inside a replayed graph. H = 8192 is the
    70B hidden size; fences = 1 runs the system-scope release / acquire barriers that peers on other GPUs
    get by default (parallel/ipc_allreduce.fences_for)."""
    from rag_llm_k8s_amd.ops import reference as R

    global H_F
    monkeypatch.setenv("RAGK_TEST_FUSED_H", str(H))
    monkeypatch.setenv("RAGK_TEST_FENCES", str(fences))
    monkeypatch.setattr(sys.modules[__name__], "H_F", H)
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        out = _spawn(_fused_worker, WORLD, d, port)
    assert all(out[r]["fences"] == bool(fences) for r in range(WORLD))
    w = (1 + 0.1 * torch.randn(H_F, generator=torch.Generator().manual_seed(5))).bfloat16()

    def ref(M, S, it, h0):
        tot = torch.zeros(M, H_F)
        for r in range(WORLD):
            P = _partials(r, M, S, it)
            a = torch.zeros(M, H_F)
            for s in range(S):
                a = a + P[s]
            tot = tot + a
        return (h0.float() + tot.bfloat16().float()).bfloat16()

    for mode in (0, 1):
        for it, (M, S) in enumerate(FUSED_CASES):
            h0 = torch.randn(M, H_F, generator=torch.Generator().manual_seed(M + it)).bfloat16()
            want = ref(M, S, it, h0)
            for r in range(WORLD):
                h, o = out[r][(mode, it)]
                assert torch.equal(h, want), (mode, it, r)
                assert torch.equal(o, out[0][(mode, it)][1])
                ro = R.rmsnorm(want, w, 1e-5)
                assert ((o.float() - ro.float()).abs().max() <= 0.02 * ro.float().abs().max()), (mode, it)
    for mode_it in [(0, i) for i in range(len(FUSED_CASES))]:  # one-shot == two-shot, bit for bit
        assert torch.equal(out[0][mode_it][1], out[0][(1, mode_it[1])][1])
    for it in range(3):
        want = ref(4, 2, 100 + it, torch.ones(4, H_F).bfloat16())
        for r in range(WORLD):
            assert torch.equal(out[r]["graph"][it][0], want)
    assert all(out[r]["error"] is False for r in range(WORLD))


# ---------------------------------------------------------------- watchdog error record
def _timeout_worker(rank, port, d, WORLD=2):
    """Rank 1 skips the collectives: rank 0's bounded peer waits give up and record which one."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    torch.cuda.set_device(0)
    from rag_llm_k8s_amd.parallel.ipc_allreduce import IPCAllReduce, describe_error

    ar = IPCAllReduce(None, None, WORLD, rank, "cuda:0", max_bytes=1 << 20, blocks=8, fused_rows=8, fused_h=512,
                      spin_limit=200000)  # 0.2 s per peer wait
    res = {}
    try:
        if rank == 0:
            x = torch.ones(8 * 512, dtype=torch.bfloat16, device="cuda")
            ar.all_reduce(x, mode=0)  # call 1 of every block: peer 1 never arrives
            torch.cuda.synchronize()
            res["rec"] = ar.error_record()
            res["text"] = describe_error(res["rec"])
    finally:
        torch.cuda.synchronize()
        dist.barrier()
        ar.close()
        torch.save(res, os.path.join(d, "r%d.pt" % rank))
        dist.destroy_process_group()


def test_ipc_timeout_error_record(native):
    """A peer that never arrives: the waiting rank's error word names the collective (start barrier of the
    all-reduce), the peer (rank 1), the block and the call index -- what CommError reports."""
    with tempfile.TemporaryDirectory() as d:
        out = _spawn(_timeout_worker, 2, d, _free_port())
    rec = out[0]["rec"]
    assert rec & 1, rec
    assert (rec >> 1) & 7 == 1 and (rec >> 4) & 7 == 1 and (rec >> 7) & 255 < 8 and (rec >> 15) & 0xFFFF == 1, rec
    assert "peer rank 1 never arrived" in out[0]["text"] and "all-reduce (start barrier)" in out[0]["text"]
