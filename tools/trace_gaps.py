"""Summarise a rocprofv3 --kernel-trace CSV: GPU busy time vs wall per step and
the largest idle gaps (host/launch-bound diagnosis).
    python tools/trace_gaps.py <kernel_trace.csv> [steps]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# take the last `steps` worth of kernels: find the period by k_ray_setup launches
marks = [i for i, e in enumerate(ev) if "k_ray_setup" in e[2]]
if steps and len(marks) > steps:
    ev = ev[marks[-steps - 1]:marks[-1]]
t0, t1 = ev[0][0], ev[-1][0]
busy, last_end = 0, t0
gaps = defaultdict(int)
per = defaultdict(int)
for s, e, n in ev:
    s2 = max(s, last_end)
    if e > s2:
        busy += e - s2
    if s > last_end:
        gaps[n.split("(")[0][:60]] += s - last_end
    last_end = max(last_end, e)
    per[n.split("(")[0][:60]] += e - s
nst = max(len([1 for e in ev if "k_ray_setup" in e[2]]), 1)
print(f"steps {nst}: wall/step {(t1 - t0) / nst / 1e3:.1f} us, GPU busy/step {busy / nst / 1e3:.1f} us, "
      f"kernels/step {len(ev) / nst:.1f}")
print("idle time before kernel (us/step):")
for n, g in sorted(gaps.items(), key=lambda kv: -kv[1])[:15]:
    print(f"  {g / nst / 1e3:8.1f}  {n}")
print("busy per kernel (us/step):")
for n, g in sorted(per.items(), key=lambda kv: -kv[1])[:25]:
    print(f"  {g / nst / 1e3:8.1f}  {n}")
