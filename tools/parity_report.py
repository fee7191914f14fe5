"""Print the scale-aware errors of every golden case (both grid layouts) against the
reference's golden vectors, without asserting (GPU box; NICECORE_LIB selects a build).
    python tools/parity_report.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "nice-slam-annotation_amd")):
    sys.path.insert(0, p)
from conftest import CASE_NAMES  # noqa: E402
from parity_common import compare, run_case  # noqa: E402

worst = {}
for cl in (False, True):
    for case in CASE_NAMES:
        rec, got = run_case(case, channels_last=cl)
        errs = compare(rec, got)
        top = sorted(errs.items(), key=lambda kv: -kv[1])[:4]
        print(f"{case:16s} cl={int(cl)} " + "  ".join(f"{k} {v:.2e}" for k, v in top), flush=True)
        for k, v in errs.items():
            kk = k.split("/")[0] + ("/" + k.split("/")[1] if "/" in k else "")
            worst[kk] = max(worst.get(kk, 0.0), v)
print("worst:", {k: f"{v:.2e}" for k, v in sorted(worst.items())})
