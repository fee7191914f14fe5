"""Per-kernel SQ counter report from tools/pmc_session.sh output.
    python tools/pmc_report.py gpurun_out/pmc_<tag>

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles): the busy counter is
summed over every SIMD of the chip (it equals 32 cycles x the number of
v_mfma_f32_16x16x4_f32 and 16 x the number of v_mfma_f32_16x16x32_f16, the instructions'
issue cycles on one SIMD), and the kernel's cycles are GRBM_GUI_ACTIVE / 8 (rocprofv3 sums
GRBM_GUI_ACTIVE over the 8 XCDs; MI355X_MICROARCH.md, DVFS).  It is the fraction of the MFMA
peak at the clock the kernel ran at.  SQ_BUSY_CYCLES is summed over the 32 shader engines,
so mfma_busy / (32 x SQ_BUSY_CYCLES) is printed beside it as a cross-check."""
import csv
import glob
import os
import sys
from collections import defaultdict

N_SIMD = 256 * 4  # MI355X: 256 CUs x 4 SIMDs
N_XCD = 8
N_SE = 32
d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("nc::", "")
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(vals.items()):
    m = {n: sum(v) / len(v) for n, v in c.items()}
    g = lambda n: m.get(n, float("nan"))
    wc = g("SQ_WAVE_CYCLES")
    print(f"== {k}")
    print(f"   waves {g('SQ_WAVES'):.0f}  busy_cycles {g('SQ_BUSY_CYCLES'):.3g}  wave_cycles {wc:.3g}")
    print(f"   wait_any {g('SQ_WAIT_ANY') / wc:.2f}  wait_inst_any {g('SQ_WAIT_INST_ANY') / wc:.2f}  "
          f"active_inst_any {g('SQ_ACTIVE_INST_ANY') / wc:.2f}  wait_inst_lds {g('SQ_WAIT_INST_LDS') / wc:.2f}")
    mf32 = g("SQ_INSTS_VALU_MFMA_F32")
    mf16 = m.get("SQ_INSTS_VALU_MFMA_F16", 0.0)
    mf = (mf32 if mf32 == mf32 else 0.0) + mf16
    print(f"   insts: valu {g('SQ_INSTS_VALU'):.3g} (per mfma {g('SQ_INSTS_VALU') / max(mf, 1):.2f})  mfma_f32 {mf32:.3g}  "
          f"mfma_f16 {mf16:.3g}  lds {g('SQ_INSTS_LDS'):.3g} (per mfma {g('SQ_INSTS_LDS') / max(mf, 1):.2f})  "
          f"salu {g('SQ_INSTS_SALU'):.3g}  vmem {g('SQ_INSTS_VMEM'):.3g}")
    busy = g("SQ_VALU_MFMA_BUSY_CYCLES")
    kcyc = g("GRBM_GUI_ACTIVE") / N_XCD
    print(f"   mfma_util {busy / (N_SIMD * kcyc) if kcyc > 0 else float('nan'):.3f} (busy / (SIMDs x GRBM_GUI_ACTIVE/8))  "
          f"cross-check {busy / (N_SE * max(g('SQ_BUSY_CYCLES'), 1)):.3f} (busy / (32 x SQ_BUSY_CYCLES))  "
          f"busy per mfma {busy / max(mf, 1):.1f} cyc")
    print(f"   lds_bank_conflict/active_lds {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_ACTIVE_INST_LDS'), 1):.3f}  "
          f"active_valu/wave_cycles {g('SQ_ACTIVE_INST_VALU') / wc:.2f}")
    if g('SQ_LDS_IDX_ACTIVE') > 0:
        print(f"   lds_bank_conflict {g('SQ_LDS_BANK_CONFLICT'):.3e} of lds_idx_active {g('SQ_LDS_IDX_ACTIVE'):.3e} "
              f"({g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f})")
