"""Per-kernel mean durations in two phases of one rocprofv3 kernel trace (kernel_trace.csv), split at the
start of the N-th last dispatch of an anchor kernel -- e.g. the in-situ decode steps of
tools/decode_anatomy.py vs its back-to-back graph replays at the end (21 replays x 32 layers):

  python tools/phase_kernel_stats.py gpurun_out/pdb32/run_kernel_trace.csv attn_decode 672 [first_anchor_skip]

first_anchor_skip: anchor dispatches at the start to leave out of phase A (warm-up / capture runs).
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:70]


def main(path, anchor, last, skip=0):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    split = int(rows[idx[-last]]["Start_Timestamp"])
    begin = int(rows[idx[skip]]["Start_Timestamp"]) if skip else 0
    acc = defaultdict(lambda: [[0, 0.0], [0, 0.0]])
    span = [[None, None], [None, None]]
    for r in rows:
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 < begin:
            continue
        ph = 1 if t0 >= split else 0
        a = acc[short(r["Kernel_Name"])][ph]
        a[0] += 1
        a[1] += (t1 - t0) / 1e3
        s = span[ph]
        s[0] = t0 if s[0] is None else min(s[0], t0)
        s[1] = t1 if s[1] is None else max(s[1], t1)
    print("# phase A: %.2f ms span, phase B: %.2f ms span" % tuple(
        ((s[1] - s[0]) / 1e6 if s[0] is not None else 0.0) for s in span))
    print("# %-70s %8s %10s %8s %10s" % ("kernel", "n A", "mean us A", "n B", "mean us B"))
    for k, (a, b) in sorted(acc.items(), key=lambda kv: -(kv[1][0][1] + kv[1][1][1])):
        print("%-72s %8d %10.2f %8d %10.2f" % (k, a[0], a[1] / max(a[0], 1), b[0], b[1] / max(b[0], 1)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 0)
