"""Timing ablations of the render core: build variant libraries (compile-time
NC_ABL_* switches that remove one piece of work; results are WRONG, timing only)
and print the per-kernel breakdown of the C2 bench step for each.

    python tools/ablate.py build            # in the build container (hipcc)
    python tools/ablate.py run [variants]   # on the GPU box
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nice-slam-annotation_amd"))
DBG = os.path.join(REPO, "dbg")
VARIANTS = {
    "ref": [],
    "cur": [],
    "no_gather": ["-DNC_ABL_NO_GATHER"],
    "no_trig": ["-DNC_ABL_NO_TRIG"],
    "no_recstore": ["-DNC_ABL_NO_RECSTORE"],
    "no_mask": ["-DNC_ABL_NO_MASK"],
    "fwd_nolds": ["-DNC_ABL_FWD_NOLDS"],
    "fwd_nolds_notrig": ["-DNC_ABL_FWD_NOLDS", "-DNC_ABL_NO_TRIG", "-DNC_ABL_NO_RECSTORE"],
    "dx_no_scatter": ["-DNC_ABL_DX_NO_SCATTER"],
    "dx_no_atomic": ["-DNC_ABL_DX_NO_ATOMIC"],
    "dx_no_coord": ["-DNC_ABL_DX_NO_COORD"],
    "dx_no_trilinear": ["-DNC_ABL_DX_NO_SCATTER", "-DNC_ABL_DX_NO_COORD"],
    "dx512": ["-DNC_DX_THREADS=512"],
    "no_sort": ["-DNC_ABL_NO_SORT"],
    "dw512_16": ["-DNC_DW_THREADS=512", "-DNC_DW_NPTS=16"],
    "dw256_16": ["-DNC_DW_THREADS=256", "-DNC_DW_NPTS=16"],
    "dw1024_16": ["-DNC_DW_THREADS=1024", "-DNC_DW_NPTS=16"],
    "dw768_16": ["-DNC_DW_THREADS=768", "-DNC_DW_NPTS=16"],
    "dw512_32": ["-DNC_DW_THREADS=512", "-DNC_DW_NPTS=32"],
    "dw256_32": ["-DNC_DW_THREADS=256", "-DNC_DW_NPTS=32"],
    "dw768_32": ["-DNC_DW_THREADS=768", "-DNC_DW_NPTS=32"],
    "dw_no_emb": ["-DNC_ABL_DW_NO_EMB"],
    "dw_no_maskpass": ["-DNC_ABL_DW_NO_MASKPASS"],
    "dw_no_stage": ["-DNC_ABL_DW_NO_STAGE"],
    "dw_no_load": ["-DNC_ABL_DW_NO_LOAD"],
    "dw_no_mfma": ["-DNC_ABL_DW_NO_MFMA"],
    "mfma_f32": ["-DNC_MFMA_F32"],
    "no_zero_fill": ["-DNC_ABL_NO_ZERO_FILL"],
    "fwd_no_stores": ["-DNC_ABL_NO_ZERO_FILL", "-DNC_ABL_NO_RECSTORE"],
    "exact1": ["-DNC_EXACT_WGS=1"],
    "fwd_b2": ["-DNC_FWD_GATHER_B2"],
    "dx_novec": ["-DNC_DX_NO_VEC"],
    "dx_no_bgrad": ["-DNC_ABL_DX_NO_BGRAD"],
    "exact4": ["-DNC_EXACT_WGS=4"],
    "fused4": ["-DNC_FUSED_RAYS=4"],
    "fused8": ["-DNC_FUSED_RAYS=8"],
    "fwd_t2_512": ["-DNC_FWD_TILES=2", "-DNC_FWD_THREADS=512"],
    "fwd_t1_1024": ["-DNC_FWD_THREADS=1024"],
    "fwd_t2_768": ["-DNC_FWD_TILES=2"],
    "fwd_cost_macs": ["-DNC_FWD_COST_MACS"],
    "dw_pad_chains": ["-DNC_DW_PAD_CHAINS"],
    "gather8": ["-DNC_GATHER_CH=8"],
    "gather_one": ["-DNC_GATHER_ONE_KERNEL"],
    "gather_minb8": ["-DNC_GATHER_MINB=8"],
    "dw_serial": ["-DNC_DW_SERIAL"],
    "dw_npts48": ["-DNC_DW_NPTS=48"],
    "no_fuse_gather": ["-DNC_NO_FUSE_GATHER"],
    "fused768": ["-DNC_FWD_THREADS_FUSED=768"],
    "fused1024": ["-DNC_FWD_THREADS_FUSED=1024"],
    "dw_core": ["-DNC_DW_SERIAL", "-DNC_ABL_DW_NO_STAGE", "-DNC_ABL_DW_NO_EMB", "-DNC_ABL_DW_NO_MASKPASS",
                "-DNC_ABL_DW_NO_LOAD"],
    "dw_none": ["-DNC_DW_SERIAL", "-DNC_ABL_DW_NO_STAGE", "-DNC_ABL_DW_NO_EMB", "-DNC_ABL_DW_NO_MASKPASS",
                "-DNC_ABL_DW_NO_LOAD", "-DNC_ABL_DW_NO_MFMA"],
    "dw_serial_nomfma": ["-DNC_DW_SERIAL", "-DNC_ABL_DW_NO_MFMA"],
    "dw_split16": ["-DNC_DW_SPLIT16"],
    "dw_split16_r3": ["-DNC_DW_SPLIT16", "-DNC_DW_RING=3"],
    "dwh_no_build": ["-DNC_DW_SPLIT16", "-DNC_ABL_DWH_NO_BUILD"],
    "dwh_no_dma": ["-DNC_DW_SPLIT16", "-DNC_ABL_DWH_NO_DMA"],
    "dwh_no_mfma": ["-DNC_DW_SPLIT16", "-DNC_ABL_DWH_NO_MFMA"],
    "dwh_none": ["-DNC_DW_SPLIT16", "-DNC_ABL_DWH_NO_BUILD", "-DNC_ABL_DWH_NO_DMA", "-DNC_ABL_DWH_NO_MFMA"],
    "fill2": ["-DNC_FILL_WGS_PER_CU=2"],
    "fill3": ["-DNC_FILL_WGS_PER_CU=3"],
    "scat_u2": ["-DNC_SCAT_UNROLL=2"],
    "scat_u4": ["-DNC_SCAT_UNROLL=4"],
    "scat_u16": ["-DNC_SCAT_UNROLL=16"],
    "rs_r16": ["-DNC_RS_ROUNDS=16"],  # NC_DETERMINISTIC=1 runs
    "rs_r4": ["-DNC_RS_ROUNDS=4"],
    "rs_r32": ["-DNC_RS_ROUNDS=32"],
    "dsub32": ["-DNC_DET_DSUB=32"],  # NC_DETERMINISTIC=1 runs
    "det_no_keys_hist": ["-DNC_DET_NO_KEYS_HIST"],
    "det_rg4": ["-DNC_DET_RG=4"],  # NC_DETERMINISTIC=1 runs
    "det_rg16": ["-DNC_DET_RG=16"],
    "no_split": ["-DNC_ABL_NO_SPLIT"],
    "split_rtz": ["-DNC_SPLIT_RTZ"],
    "fwd_w2": ["-DNC_FWD_W2"],
    "ft2_512": ["-DNC_FWD_TILES=2", "-DNC_FWD_THREADS_FUSED=512"],
    "ft2_768": ["-DNC_FWD_TILES=2"],
    "ft1_512": ["-DNC_FWD_THREADS_FUSED=512"],
    "ft1_1024": ["-DNC_FWD_THREADS_FUSED=1024"],
    "no_triw": ["-DNC_ABL_NO_TRIW"],
    "pr8": ["-DNC_PR_AHEAD=8"],
    "pr12": ["-DNC_PR_AHEAD=12"],
    "scan_d8": ["-DNC_RS_SCAN_DIG=8"],
    "scan_d4": ["-DNC_RS_SCAN_DIG=4"],
    "scan_d32": ["-DNC_RS_SCAN_DIG=32"],
}
# variants built by hand (source edits) are run by name if dbg/abl_<name>.so exists

if __name__ == "__main__":
    cmd = sys.argv[1]
    names = sys.argv[2:] or list(VARIANTS)
    if cmd == "build":
        from nicecore import build as B
        os.makedirs(DBG, exist_ok=True)
        for n in names:
            print(B.build(force=True, extra=VARIANTS[n], out=os.path.join(DBG, f"abl_{n}.so")), flush=True)
    else:
        for n in names:
            if not os.path.exists(os.path.join(DBG, f"abl_{n}.so")):
                print(n, "missing", flush=True)
                continue
            env = dict(os.environ, NICECORE_LIB=os.path.join(DBG, f"abl_{n}.so"))
            r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "3",
                                "--cpu-seconds", "0"], env=env, capture_output=True, text=True, timeout=300)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            if r.returncode != 0 or not line:
                print(n, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
                break
            import json
            d = json.loads(line[-1])
            ks = d["kernels_ms"]
            print(f"{n:14s} step {d['ms_per_step']:.4f} ms  " +
                  "  ".join(f"{k.replace('k_', '')} {v * 1e3:.1f}" for k, v in ks.items()), flush=True)
