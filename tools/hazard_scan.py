"""Scan hipcc assembly for VALU/VMEM reads of a v_mfma_f32_16x16x32_{f16,bf16} result
closer than 8 wait states (the measured gfx950 requirement for the last result
register, tools/mfma_hazard.hip).  Straight-line distance within a basic block;
s_nop N counts N + 1 states, every other instruction 1.   python tools/hazard_scan.py file.s"""
import re
import sys

NEED = 8
lines = open(sys.argv[1]).read().split("\n")
reg_re = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in reg_re.finditer(text):
        if m.group(1):
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


func = None
pending = {}  # reg -> states since the MFMA that wrote it
hits = 0
for ln, raw in enumerate(lines, 1):
    s = raw.split(";")[0].strip()
    if not s:
        continue
    if s.endswith(":") and not s.startswith("."):
        if not s.startswith(".L"):
            func = s[:-1]
        pending = {}  # new basic block: be conservative only within blocks
        continue
    if s.startswith("."):
        continue
    op = s.split()[0]
    args = s[len(op):]
    if op.startswith("s_nop"):
        n = int(args.strip(), 0) + 1
        pending = {r: d + n for r, d in pending.items()}
        continue
    parts = [p.strip() for p in args.split(",")]
    dst = regs(parts[0]) if parts else set()
    srcs = regs(",".join(parts[1:])) if len(parts) > 1 else set()
    is_mfma = op.startswith("v_mfma")
    if not is_mfma:
        reads = srcs if not op.startswith(("global_store", "buffer_store", "scratch_store", "ds_write", "global_atomic", "flat_store")) else regs(args)
        for r in reads:
            if r in pending and pending[r] < NEED:
                hits += 1
                print(f"{func}: line {ln}: '{s}' reads v{r} {pending[r]} states after an f16 MFMA wrote it")
    pending = {r: d + 1 for r, d in pending.items()}
    for r in dst:
        pending.pop(r, None)
    if is_mfma and ("16x16x32_f16" in op or "16x16x32_bf16" in op):
        for r in dst:
            pending[r] = 0
print("hazards:", hits)
