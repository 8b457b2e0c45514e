"""Cross-rank view of a rocprofv3 kernel trace of N TP ranks sharing one GPU (tools/gpu_tp8_trace.sh).

For every peer-mapped collective kernel (csrc/comm/allreduce.hip: allreduce / allgather / ar_add_rmsnorm)
the k-th dispatch of each process is matched with the k-th of every other process (all ranks issue the
same collective sequence). Per call index: the start skew across ranks, and whether some rank's kernel
ENDED before another rank's matching kernel STARTED -- the waiting rank gave up (bounded spin) while its
peer was not yet running: the peer was never co-resident, a scheduling stall rather than a protocol one
(a protocol error would show every peer kernel running and still a timeout).

  python tools/tp_trace_report.py gpurun_out/tp8trace
"""
import collections
import csv
import glob
import os
import sys

KEYS = ("allreduce_kernel", "allgather_kernel", "ar_add_rmsnorm_kernel")


def load(root):
    per = collections.defaultdict(list)  # pid -> [(start, end, name)]
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if any(k in name for k in KEYS):
                pid = r.get("Process_Id") or os.path.basename(f).split("_")[0]
                per[pid].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                 next(k for k in KEYS if k in name)))
    for v in per.values():
        v.sort()
    return per


def main():
    root = sys.argv[1]
    per = load(root)
    pids = sorted(per, key=lambda p: per[p][0][0] if per[p] else 0)
    print("processes with collective kernels: %d; dispatches per process: %s" % (
        len(pids), [len(per[p]) for p in pids]))
    if len(pids) < 2:
        return
    n = min(len(per[p]) for p in pids)
    worst, stalls = [], []
    for k in range(n):
        calls = [per[p][k] for p in pids]
        starts = [c[0] for c in calls]
        ends = [c[1] for c in calls]
        skew = (max(starts) - min(starts)) / 1e6
        durs = [(c[1] - c[0]) / 1e6 for c in calls]
        worst.append((skew, k, calls[0][2], max(durs)))
        if min(ends) < max(starts):  # someone gave up before a peer began
            early = pids[ends.index(min(ends))]
            late = pids[starts.index(max(starts))]
            stalls.append((k, calls[0][2], early, late, (max(starts) - min(ends)) / 1e6, max(durs)))
    worst.sort(reverse=True)
    print("matched calls: %d; median start skew %.3f ms" % (n, sorted(w[0] for w in worst)[n // 2]))
    print("largest start skews (ms, call, kernel, longest duration ms):")
    for w in worst[:10]:
        print("  %.3f  #%d  %s  %.3f" % w)
    print("calls where a rank's kernel ENDED before a peer's matching kernel STARTED: %d" % len(stalls))
    for s in stalls[:20]:
        print("  #%d %s: pid %s ended %.3f ms before pid %s started (longest run %.3f ms)" % (
            s[0], s[1], s[2], s[4], s[3], s[5]))
    if len(per[pids[0]]) != len(per[pids[-1]]):
        print("dispatch counts differ across processes (a rank stopped early):",
              {p: len(per[p]) for p in pids})


if __name__ == "__main__":
    main()
