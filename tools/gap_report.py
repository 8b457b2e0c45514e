"""Idle gaps between kernels in a rocprofv3 --kernel-trace run (kernel_trace.csv): where the GPU waits on
the host. Busy time is the union of kernel intervals (side streams may overlap); a gap is attributed to the
kernels on either side of it, classified as prefill (large-M GEMM / prefill attention), decode (split-K /
stream GEMMs, decode attention, norms) or other.

  python tools/gap_report.py gpurun_out/prof/run_kernel_trace.csv [max_gap_ms]

Gaps longer than max_gap_ms (default 20) are treated as phase boundaries (setup, host-side pauses) and
only counted, not attributed.
"""
import csv
import sys
from collections import defaultdict


def _base(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def kind(name):
    n = _base(name)
    if "gemm_w4" in n or "gemm_pp" in n or "attn_prefill" in n:
        return "prefill"
    if any(k in n for k in ("gemm_part", "gemm_stream", "gemm_skinny", "gemm_dec", "attn_decode", "add_partials",
                            "attn_oproj", "sample", "topk")):
        return "decode"
    return "other"


def short(name):
    return _base(name)[:60]


def main(path, max_gap_ms=20.0):
    rows = list(csv.DictReader(open(path)))
    cols = list(rows[0].keys()) if rows else []
    col = lambda want: next(c for c in cols if want in c.lower())  # noqa: E731  (column names vary by version)
    cs, ce, cn = col("start"), col("end"), col("kernel_name") if any("kernel_name" in c.lower() for c in cols) else col("name")
    ks = sorted((int(r[cs]), int(r[ce]), r[cn]) for r in rows)
    if not ks:
        print("no kernels")
        return
    # the serving window: from the first prefill kernel on (weight init / ingest before it are setup)
    first = next((i for i, k in enumerate(ks) if kind(k[2]) == "prefill"), 0)
    if "--all" not in sys.argv:
        ks = ks[first:]
    busy = 0
    cur_s, cur_e, cur_n = ks[0]
    gaps = []
    for s, e, n in ks[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_n, n))
            cur_s, cur_e, cur_n = s, e, n
        elif e > cur_e:
            cur_e, cur_n = e, n
    busy += cur_e - cur_s
    span = ks[-1][1] - ks[0][0]
    big = [g for g in gaps if g[0] > max_gap_ms * 1e6]
    small = [g for g in gaps if g[0] <= max_gap_ms * 1e6]
    print("# %s: %d kernels, span %.1f ms, busy %.1f ms (%.1f %%)" % (path, len(ks), span / 1e6, busy / 1e6,
                                                                  100.0 * busy / span))
    print("# %d gaps > %.0f ms (phase boundaries): %.1f ms" % (len(big), max_gap_ms, sum(g[0] for g in big) / 1e6))
    print("# %d gaps <= %.0f ms: %.1f ms" % (len(small), max_gap_ms, sum(g[0] for g in small) / 1e6))
    by = defaultdict(lambda: [0, 0])
    for g, a, b in small:
        k = "%s -> %s" % (kind(a), kind(b))
        by[k][0] += 1
        by[k][1] += g
    print("# by neighbour class (count, ms, mean us):")
    for k, (c, t) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print("%-22s %7d %9.2f %9.1f" % (k, c, t / 1e6, t / c / 1e3))
    hist = defaultdict(lambda: [0, 0])
    for g, _, _ in small:
        b = "<2us" if g < 2e3 else "<10us" if g < 1e4 else "<100us" if g < 1e5 else "<1ms" if g < 1e6 else ">=1ms"
        hist[b][0] += 1
        hist[b][1] += g
    print("# gap sizes (count, ms):")
    for b in ("<2us", "<10us", "<100us", "<1ms", ">=1ms"):
        if b in hist:
            print("%-8s %7d %9.2f" % (b, hist[b][0], hist[b][1] / 1e6))
    print("# largest attributed gaps:")
    for g, a, b in sorted(small, key=lambda x: -x[0])[:20]:
        print("%9.1f us  %s -> %s" % (g / 1e3, short(a), short(b)))


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--all"]
    main(args[0], float(args[1]) if len(args) > 1 else 20.0)
