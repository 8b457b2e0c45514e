"""CPU tests for the profile post-processing tools (tools/gap_report.py, rocprof_summary.py, pmc_summary.py)
on small synthetic rocprofv3 CSVs of the same column layout the GPU runs write."""
import csv
import os
import sys

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gap_report  # noqa: E402
import pmc_summary  # noqa: E402
import rocprof_summary  # noqa: E402


def _write(path, cols, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(cols)
        w.writerows(rows)


def test_gap_report_kind_strips_namespace():
    assert gap_report.kind("void (anonymous namespace)::gemm_part_kernel<4>(float*, int)") == "decode"
    assert gap_report.kind("void (anonymous namespace)::attn_prefill_kernel<8, false>(...)") == "prefill"
    assert gap_report.kind("Cijk_Alik_Bljk_BBS_BH") == "other"


def test_gap_report_gaps(tmp_path, capsys):
    us = 1000  # ns
    rows = [
        (0, 10 * us, "void (anonymous namespace)::embed_kernel()"),          # setup, dropped (before prefill)
        (20 * us, 120 * us, "void (anonymous namespace)::gemm_w4_kernel<1>(x)"),
        (125 * us, 130 * us, "void (anonymous namespace)::gemm_part_kernel<2>(x)"),   # 5 us gap prefill->decode
        (128 * us, 140 * us, "void (anonymous namespace)::attn_decode_kernel<128>(x)"),  # overlaps, no gap
        (141 * us, 150 * us, "void (anonymous namespace)::add_partials_rmsnorm(x)"),  # 1 us decode->decode
        (150 * us + 50_000 * us, 150 * us + 50_010 * us, "void (anonymous namespace)::gemm_part_kernel<2>(x)"),
    ]
    p = tmp_path / "run_kernel_trace.csv"
    _write(p, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], [(n, s, e) for s, e, n in rows])
    gap_report.main(str(p), 20.0)
    out = capsys.readouterr().out
    assert "5 kernels" in out                      # embed dropped: window starts at the first prefill kernel
    assert "1 gaps > 20 ms" in out                 # the 50 ms pause is a phase boundary
    assert "2 gaps <= 20 ms: 0.0 ms" in out        # 5 us + 1 us
    lines = {ln.split()[0] + ln.split()[1] + ln.split()[2]: ln for ln in out.splitlines() if "->" in ln and "us " not in ln}
    assert "prefill->decode" in lines and "decode->decode" in lines
    assert int(lines["prefill->decode"].split()[3]) == 1


def test_rocprof_summary(tmp_path, capsys):
    p = tmp_path / "kernel_stats.csv"
    _write(p, ["Name", "Calls", "TotalDurationNs", "AverageNs"],
           [("gemm_part_kernel", 10, 3_000_000, 300_000), ("Cijk_Alik_Bljk", 2, 1_000_000, 500_000)])
    rocprof_summary.main(str(p))
    out = capsys.readouterr().out
    assert "4.0 ms total" in out
    assert "75.00%" in out and "hipBLASLt (Cijk) kernels: 1" in out


def test_pmc_summary(tmp_path, capsys, monkeypatch):
    d = tmp_path / "pmc" / "host0"
    d.mkdir(parents=True)
    cols = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Workgroup_Size", "Start_Timestamp", "End_Timestamp",
            "Counter_Name", "Counter_Value"]
    base = ["7", "void gemm_w4_kernel<1, 2>(x)", "65536", "256", "0", "10000"]
    _write(d / "run_counter_collection.csv", cols, [
        base + ["GRBM_GUI_ACTIVE", str(8 * 24000)],           # 24000 cycles over 10 us -> 2.40 GHz
        base + ["SQ_VALU_MFMA_BUSY_CYCLES", str(1024 * 12000)],  # half the MFMA pipe-cycles busy
    ])
    monkeypatch.setattr(sys, "argv", ["pmc_summary.py", str(tmp_path / "pmc")])
    pmc_summary.main()
    out = capsys.readouterr().out
    assert "wg=   256" in out and "clk=2.40GHz" in out and "mfma=50.0%" in out


def test_isa_lds_hazard_model():
    """The asm-wait checker: a register of an LDS read touched before its lgkmcnt retires it is a
    hazard (the spill gemm_w4's GELU epilogues produced); counted waits retire the oldest reads."""
    import isa_lds_hazard as H

    spill = [(0, "ds_read_b128 v[0:3], v112"), (8, "scratch_store_dwordx4 off, v[0:3], off")]
    assert [h[0] for h in H.check_kernel(0, spill)] == [8]
    counted = [(0, "ds_read_b128 v[0:3], v9"), (8, "ds_read_b128 v[4:7], v9 offset:2048"),
               (16, "s_waitcnt lgkmcnt(1)"), (24, "v_mfma_f32_16x16x32_bf16 a[0:3], v[0:3], v[0:3], a[0:3]"),
               (32, "v_mfma_f32_16x16x32_bf16 a[0:3], v[4:7], v[0:3], a[0:3]")]
    assert [h[0] for h in H.check_kernel(0, counted)] == [32]
    # loop back edge: reads issued at the bottom are pending at the top until the wait there
    loop = [(0, "v_mfma_f32_16x16x32_bf16 a[0:3], v[0:3], v[0:3], a[0:3]"), (8, "ds_read_b128 v[0:3], v9"),
            (16, "s_cbranch_scc1 -3 <k+0x0>")]
    assert [h[0] for h in H.check_kernel(0, loop)] == [0]
    # forward branch: the taken path reaches its target with the read pending, the fall-through waits first
    fwd = [(0, "ds_read_b128 v[0:3], v9"), (8, "s_cbranch_scc1 2 <k+0x18>"), (16, "s_waitcnt lgkmcnt(0)"),
           (24, "v_add_f32 v4, v0, v5")]
    assert [h[0] for h in H.check_kernel(0, fwd)] == [24]
    fwd_ok = fwd[:1] + [(4, "s_waitcnt lgkmcnt(0)")] + fwd[1:]
    assert H.check_kernel(0, fwd_ok) == []
    waited = [(0, "s_waitcnt lgkmcnt(0)")] + [(a + 8, i) for a, i in loop]
    assert H.check_kernel(0, waited) == []


def test_isa_lds_hazard_kernels_clean():
    """Every built kernel object passes the checker (the hand-placed waits of gemm_w4 included)."""
    import glob

    import isa_lds_hazard as H

    objs = sorted(glob.glob(os.path.join(ROOT, "build", "obj", "*.hip.o")))
    if not objs or not os.path.exists(os.path.join(H.LLVM, "llvm-objdump")):
        pytest.skip("kernel objects not built here")
    for obj in objs:
        assert H.check_object(obj) == [], obj
