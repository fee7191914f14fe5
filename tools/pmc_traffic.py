"""Per-kernel HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes (separate runs; tools/prof_session.sh), with the gfx950 correction of
MI355X_MICROARCH.md § HBM: FETCH_SIZE counts half the bytes of wide coalesced
reads (x2); WRITE_SIZE is exact for 16-B stores and float atomics.
FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB.

    python tools/pmc_traffic.py [--atomic <atomic pass>] <fetch pass> <write pass> [out.json [bench args...]]

--atomic: a --pmc TCC_EA0_ATOMIC_sum pass.  Float atomics execute at the memory side; each
256-B wave-instruction leaves L2 as four 64-B atomic requests (MI355X_MICROARCH.md "Global
float atomics"), so atomic_bytes = TCC_EA0_ATOMIC x 64 per launch -- the bytes the chip-wide
float-atomic ceiling (~1.3 TB/s of added bytes) applies to.

With bench args (the same ones the profiled bench.py run had), the summary gets the
"config" key bench.py's read_traffic() matches (bench.traffic_config), so a bench line
only ever quotes traffic measured on its own workload.
"""
import csv
import json
import sys
from collections import defaultdict


def _csv(path):
    """A counter_collection.csv, or the rocprofv3 output directory holding one."""
    import glob
    import os
    if os.path.isdir(path):
        hits = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))
        if not hits:
            raise SystemExit(f"no counter_collection.csv under {path}")
        return hits[0]
    return path


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(_csv(path))):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if name.startswith("void "):
            name = name[5:]
        if not name.startswith("nc::"):
            continue
        # "nc::k_mlp_dx<false>(nc::MlpCtx)" -> "k_mlp_dx"
        acc[name.split("(")[0].split("<")[0].replace("nc::", "")].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


if __name__ == "__main__":
    atomic = {}
    if len(sys.argv) > 2 and sys.argv[1] == "--atomic":
        atomic = per_kernel(sys.argv[2], "TCC_EA0_ATOMIC_sum")
        del sys.argv[1:3]
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f_kib, nf = fetch.get(k, (0.0, 0))
        w_kib, nw = write.get(k, (0.0, 0))
        rd = 2.0 * f_kib * 1024
        wr = w_kib * 1024
        out[k] = {"hbm_bytes": round(rd + wr), "read_bytes_corrected": round(rd), "write_bytes": round(wr),
                  "fetch_size_kib_raw": round(f_kib, 1), "write_size_kib_raw": round(w_kib, 1),
                  "launches": [nf, nw]}
        if k in atomic:
            a_req, na = atomic[k]
            out[k]["atomic_requests"] = round(a_req)
            out[k]["atomic_bytes"] = round(64 * a_req)
            out[k]["launches"].append(na)
        print(f"{k:22s} read {rd / 1e6:9.2f} MB  write {wr / 1e6:9.2f} MB  atomic {out[k].get('atomic_bytes', 0) / 1e6:8.2f} MB  "
              f"({nf}/{nw} launches)")
    if len(sys.argv) > 3:
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        bargs = sys.argv[4:]
        saved, sys.argv = sys.argv, ["bench.py", *bargs]
        cfg = bench.traffic_config(bench.parse())
        sys.argv = saved
        json.dump({"note": "HBM bytes per launch, rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) "
                           "and WRITE_SIZE in separate passes; atomic_bytes = TCC_EA0_ATOMIC_sum x 64 B "
                           "(memory-side float-atomic requests) from a third pass; see tools/pmc_traffic.py",
                   "config": cfg, "bench_args": bargs, "kernels": out}, open(sys.argv[3], "w"), indent=1)
