"""Pure HBM read roofline on one MI355X: the prefetch kernel (csrc/kernels/prefetch.hip, 16-B loads,
8 in flight per lane, result discarded) over buffers of 16 MB .. 1 GB, cold (rotating over >= 2 GB of
buffers, so nothing is served from the 256 MB MALL), captured in a hipGraph (no launch overhead).
The bound a decode GEMM of that many weight bytes can reach."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402


def main():
    res = []
    for mb in (16, 32, 48, 112, 224, 1024):
        n = max(2, (2048 + mb - 1) // mb)
        bufs = [torch.empty(mb << 20, dtype=torch.uint8, device="cuda") for _ in range(n)]
        for blocks in (256, 512, 1024, 2048):
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for b in bufs:
                    N.prefetch(b, None, blocks)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for b in bufs:
                    N.prefetch(b, None, blocks)
            g.replay()
            torch.cuda.synchronize()
            a, e = torch.cuda.Event(True), torch.cuda.Event(True)
            a.record()
            for _ in range(3):
                g.replay()
            e.record()
            e.synchronize()
            us = a.elapsed_time(e) * 1e3 / (3 * n)
            row = dict(MB=mb, blocks=blocks, us=round(us, 1), TBps=round((mb << 20) / us / 1e6, 2))
            res.append(row)
            print(json.dumps(row), flush=True)
        del bufs
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/read_roofline.json", "w"), indent=1)


if __name__ == "__main__":
    main()
