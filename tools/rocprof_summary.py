"""Summarize a rocprofv3 --kernel-trace --stats run (kernel_stats.csv) into a ranked table."""
import csv
import sys


def main(path, top=40):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("# %s: %d kernels, %.1f ms total GPU time" % (path, len(rows), tot / 1e6))
    print("# %9s %7s %7s %10s  %s" % ("ms", "%", "calls", "avg us", "kernel"))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print("%11.1f %6.2f%% %7s %10.1f  %s" % (float(r["TotalDurationNs"]) / 1e6, 100 * float(r["TotalDurationNs"]) / tot,
                                              r["Calls"], float(r["AverageNs"]) / 1e3, r["Name"][:110]))
    cijk = [r for r in rows if "Cijk" in r["Name"]]
    print("# hipBLASLt (Cijk) kernels: %d" % len(cijk))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
