"""scripts/pmc_summary.py ``--cycle`` labelling (CPU only, synthetic counter files).

An fp8 profile also holds the quantize kernels (abs, max-reduce, fp8 copy)
between the GEMMs. Round 6 found them counted into the arm cycle, which rotated
every label by one (session r8zl); the cycle now counts GEMM dispatches only.
"""
import csv
import importlib.util
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SPEC = importlib.util.spec_from_file_location("pmc_summary", os.path.join(HERE, "..", "scripts", "pmc_summary.py"))
pmc_summary = importlib.util.module_from_spec(SPEC)
SPEC.loader.exec_module(pmc_summary)

FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]


def _write(tmp_path):
    d = tmp_path / "pmc" / "p1"
    d.mkdir(parents=True)
    rows, did, t = [], 0, 0
    arms = [("void pdmb::k8::gemm_fp8_w4s<true, false>(pdmb::GemmArgs)", 80),
            ("void pdmb::k8::gemm_fp8_w4s<true, false>(pdmb::GemmArgs)", 75),
            ("Custom_Cijk_Alik_Bljk_F8BS_SK3_MT256x256x128_MI16x16x1_gfx950", 70)]
    for _ in range(4):
        for extra in ("void at::native::reduce_kernel<512, 1>(int)", "void at::native::float8_copy(int)"):
            did += 1
            rows.append([did, extra, "GRBM_GUI_ACTIVE", 1000, t, t + 20_000])
            t += 30_000
        for name, us in arms:
            did += 1
            rows.append([did, name, "GRBM_GUI_ACTIVE", us * 2000 * 8, t, t + us * 1000])
            t += us * 1000 + 10_000
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(FIELDS)
        w.writerows(rows)
    return tmp_path / "pmc"


def test_cycle_labels_count_only_gemm_dispatches(tmp_path, capsys):
    pmc_summary.main(str(_write(tmp_path)), ["fp8_w4s", "x_fp8_w4s_thin", "torch"])
    out = capsys.readouterr().out
    by = {ln.split("|")[1].strip(" `"): int(ln.split("|")[2]) for ln in out.splitlines()
          if ln.startswith("| `")}
    assert by == {"fp8_w4s": 80, "x_fp8_w4s_thin": 75, "torch": 70}


def test_without_cycle_labels_by_kernel_name(tmp_path, capsys):
    pmc_summary.main(str(_write(tmp_path)))
    out = capsys.readouterr().out
    assert "hipBLASLt 256x256x128" in out
    assert "at::native::reduce_kernel<512, 1>" in out
