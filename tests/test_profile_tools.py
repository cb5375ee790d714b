"""CPU tests of the profile-analysis scripts that turn rocprofv3 CSVs into the committed evidence
(scripts/pmc_summary.py, scripts/streamk_cap_trace.py --summarize, scripts/step_sequence.py), on
small synthetic traces with the rocprofv3 column layout."""

import csv
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def _run(*args):
    r = subprocess.run([sys.executable, *args], capture_output=True, text=True, cwd=REPO, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_pmc_summary_medians_and_ratios(tmp_path):
    hdr = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]
    rows = []
    for d, (mfma, valu, wc, wait, gui, busy) in enumerate([(100, 900, 1000, 300, 8000, 3200), (100, 1100, 1000, 500, 8000, 3200),
                                                        (100, 1000, 1000, 400, 8000, 3200)]):
        for name, v in (("SQ_INSTS_MFMA", mfma), ("SQ_INSTS_VALU", valu), ("SQ_WAVE_CYCLES", wc), ("SQ_WAIT_ANY", wait),
                        ("GRBM_GUI_ACTIVE", gui), ("SQ_VALU_MFMA_BUSY_CYCLES", busy)):
            rows.append([d, "void fa_fwd_kernel<x>", name, v])
            rows.append([d, "other_kernel", name, 7 * v])
    _write(str(tmp_path / "p1" / "run_counter_collection.csv"), hdr, rows)
    kt = ["Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    _write(str(tmp_path / "kt" / "run_kernel_trace.csv"), kt,
           [["void fa_fwd_kernel<x>", 0, 1000], ["void fa_fwd_kernel<x>", 5000, 7000], ["void fa_fwd_kernel<x>", 9000, 10500]])
    out = _run("scripts/pmc_summary.py", str(tmp_path), "fa_fwd_kernel")
    vals = dict(line.split(None, 1) for line in out.strip().splitlines())
    assert float(vals["us"]) == 1.5  # median of 1.0, 2.0, 1.5 us
    assert float(vals["valu_per_mfma"]) == 10.0  # median VALU 1000 / median MFMA 100
    assert float(vals["SQ_WAIT_ANY/WAVE_CYCLES"]) == 0.4
    # 3200 busy cycles over (8000 / 8) kernel cycles x 1024 SIMDs
    assert abs(float(vals["mfma_busy_per_simd_cycle"]) - round(3200 / (1000 * 1024), 3)) < 1e-9


def test_streamk_summary_counts_workgroups(tmp_path):
    hdr = ["Kernel_Name", "Workgroup_Size_X", "Grid_Size_X"]
    name = "Cijk_Ailk_Bljk_BBS_BH_Bias_HA_S_SAV_UserArgs_MT256x256x64_MI16x16x1_SK3"
    _write(str(tmp_path / "cap" / "run_kernel_trace.csv"), hdr,
           [[name, 256, 256 * 224], [name, 256, 256 * 240], ["void at::native::foo", 256, 1024]])
    out = _run("scripts/streamk_cap_trace.py", "--summarize", str(tmp_path / "cap"))
    assert "[224, 240]" in out and "at::native" not in out


def test_step_sequence_anchors_on_hs_kernel(tmp_path):
    hdr = ["Start_Timestamp", "End_Timestamp", "Kernel_Name", "Stream_Id"]
    t, rows = 0, []

    def k(name, dur=10):
        nonlocal t
        rows.append([t, t + dur, name, 0])
        t += dur + 1

    for _step in range(2):  # two steps, each opened by the embedding gather
        k("vectorized_gather_kernel")
        for _layer in range(3):
            k("fa_fwd_kernel<...>")
            k("gemm8_kernel<...>")
        for _layer in range(3):
            k("fa_bwd_hs_kernel<...>")
            k("rope_kernel")
            k("gemm8_kernel<...>")
        k("adamw_t_kernel")
    k("vectorized_gather_kernel")
    _write(str(tmp_path / "trace.csv"), hdr, rows)
    out = _run("scripts/step_sequence.py", str(tmp_path / "trace.csv"), "--layer", "1")
    assert "== backward, between FA bwd of layer 1 and the next" in out
    assert "fa_bwd_hs_kernel" in out and "adamw_t_kernel" in out
