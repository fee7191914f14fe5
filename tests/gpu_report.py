"""Print the scale-aware error of every output / gradient of every golden case on
the HIP core (diagnostic companion of test_gpu_parity.py; run on the GPU box)."""
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import conftest  # noqa: E402,F401  (import paths)
from conftest import CASE_NAMES  # noqa: E402
from parity_common import compare, run_case  # noqa: E402

if __name__ == "__main__":
    worst = 0.0
    for cl in (False, True):
        for case in CASE_NAMES:
            try:
                rec, got = run_case(case, channels_last=cl)
            except Exception:
                print(f"== {case} channels_last={cl}: EXCEPTION")
                traceback.print_exc()
                continue
            errs = compare(rec, got)
            missing = [k for k in rec if k.startswith("grad/") and k not in got]
            print(f"== {case} channels_last={cl} missing={missing}")
            for k, e in sorted(errs.items(), key=lambda kv: -kv[1]):
                flag = "" if k in rec else "  (ref has no grad: abs max)"
                print(f"   {e:10.3e}  {k}{flag}")
                worst = max(worst, e)
    print("WORST", worst)
