"""Per-kernel SQ counter report from tools/pmc_session.sh output.
    python tools/pmc_report.py gpurun_out/pmc_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict

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
    mf = g("SQ_INSTS_VALU_MFMA_F32")
    print(f"   insts: valu {g('SQ_INSTS_VALU'):.3g} (per mfma {g('SQ_INSTS_VALU') / max(mf, 1):.2f})  mfma_f32 {mf:.3g}  "
          f"lds {g('SQ_INSTS_LDS'):.3g} (per mfma {g('SQ_INSTS_LDS') / max(mf, 1):.2f})  salu {g('SQ_INSTS_SALU'):.3g}  vmem {g('SQ_INSTS_VMEM'):.3g}")
    print(f"   mfma_busy/busy {g('SQ_VALU_MFMA_BUSY_CYCLES') / max(g('SQ_BUSY_CYCLES'), 1):.3f}  "
          f"lds_bank_conflict/active_lds {g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_ACTIVE_INST_LDS'), 1):.3f}  "
          f"active_valu/wave_cycles {g('SQ_ACTIVE_INST_VALU') / wc:.2f}")
