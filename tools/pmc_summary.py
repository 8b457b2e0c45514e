"""Per-dispatch summary of a rocprofv3 --pmc run (counter_collection.csv): wall time, effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / wall), MFMA-pipe utilisation (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x
clock cycles) and the SQ wait/active split. python tools/pmc_summary.py gpurun_out/pmc [filter]"""
import collections
import csv
import glob
import os
import sys


def short(name):
    for key in ("gemm_w4_kernel", "gemm_pp_kernel", "attn_prefill_v3_kernel", "attn_prefill_kernel",
                "attn_decode_kernel", "Cijk"):
        if key in name:
            i = name.find("<")
            return key + (name[i:i + 12] if i >= 0 and key != "Cijk" else "")
    return name[:40]


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        print("==", f)
        disp = collections.OrderedDict()
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if filt and filt not in name:
                continue
            d = disp.setdefault(r["Dispatch_Id"], {"name": short(name), "grid": int(r["Grid_Size"]),
                                                   "wg": int(r["Workgroup_Size"]),
                                                   "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                   "c": collections.defaultdict(float)})
            d["c"][r["Counter_Name"]] += float(r["Counter_Value"])
        for did, d in disp.items():
            c, ns = d["c"], max(1, d["ns"])
            gui = c.get("GRBM_GUI_ACTIVE", 0) / 8
            out = ["%6s %-34s wg=%6d %9.1fus" % (did, d["name"], d["grid"] // max(1, d["wg"]), ns / 1e3)]
            if gui:
                out.append("clk=%.2fGHz" % (gui / ns))
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c and gui:
                out.append("mfma=%.1f%%" % (100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * gui)))
            wc = c.get("SQ_WAVE_CYCLES", 0)
            if wc:
                for k, lab in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "winst"), ("SQ_ACTIVE_INST_ANY", "act"),
                               ("SQ_WAIT_INST_LDS", "wlds")):
                    if k in c:
                        out.append("%s=%.1f%%" % (lab, 100 * c[k] / wc))
            if "SQ_LDS_IDX_ACTIVE" in c:
                out.append("ldsconf=%.3f" % (c.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, c["SQ_LDS_IDX_ACTIVE"])))
            waves = max(1, d["grid"] // 64)
            ins = ["%s=%.0f" % (k[9:].lower(), c[k] / waves) for k in sorted(c) if k.startswith("SQ_INSTS_")]
            if ins:
                out.append("per-wave " + " ".join(ins))
            if "TCC_HIT_sum" in c:
                out.append("l2hit=%.1f%%" % (100 * c["TCC_HIT_sum"] / max(1, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])))
            print("  ".join(out))


if __name__ == "__main__":
    main()
