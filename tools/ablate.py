"""Timing ablations of the render core: build variant libraries and print the per-kernel
breakdown of the C2 bench step for each.

The product sources carry no ablation switches.  A variant here is
either compile-time tunables (-D flags the sources define defaults for: thread counts,
tile counts, unroll depths) or a SOURCE PATCH: text substitutions applied to a temporary
copy of csrc/ that remove one piece of work (results WRONG, timing only), compiled by
nicecore.build with ``csrc=`` and a variant build id (``<source hash>+<variant>``).
Every patch anchor must match exactly once, so a patch that no longer applies to the
current sources fails loudly instead of silently timing the product kernel.

    python tools/ablate.py build [variants]   # in the build container (hipcc)
    python tools/ablate.py run [variants]     # on the GPU box
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "nice-slam-annotation_amd"))
DBG = os.path.join(REPO, "dbg")

_VSREV = """__device__ __forceinline__ float _vs_rev(float x) {  // round-5 reduce_2pi, in revolutions
  const float k = __builtin_rintf(x * 0.15915494309189535f);
  float r = __builtin_fmaf(-k, 6.28125f, x);
  r = __builtin_fmaf(-k, 1.9353071795864769e-3f, r);
  r = __builtin_fmaf(-k, 1.2537033403800354e-11f, r);
  return r * 0.15915494309189535f;
}
"""
_VSIN2 = "  return f2{__builtin_amdgcn_sinf(_vs_rev(x.x)), __builtin_amdgcn_sinf(_vs_rev(x.y))};\n"

# (file, anchor, replacement): the anchor must occur exactly once in the file
PATCHES = {
    "no_gather": [
        ("nc_device.h", "  const int64_t sC = G.stride[0];\n  float v[8][8];",
         "  for (int j = 0; j < 8; ++j) out[j] = c.w[j] * 0.01f;\n  return;\n  const int64_t sC = G.stride[0];\n"
         "  float v[8][8];"),
        ("nc_device.h", "  float v[2][8][8];",
         "  for (int j = 0; j < 8; ++j) { out1[j] = c1.w[j] * 0.01f; out2[j] = c2.w[j] * 0.01f; }\n  return;\n"
         "  float v[2][8][8];"),
    ],
    "no_trig": [
        ("nc_device.h", "__device__ __forceinline__ f2 fourier_sin2(f2 x) {\n",
         "__device__ __forceinline__ f2 fourier_sin2(f2 x) {\n  return x;\n"),
    ],
    "no_recstore": [
        ("nc_mlp.hip", "      rec[t] = (ctx.save_rec && pt[t] < ctx.P) ? ctx.rec + job.rec_off + pt[t] * Rec<KIND>::STRIDE "
                       ": nullptr;", "      rec[t] = nullptr;"),
    ],
    "no_split": [
        ("nc_device.h", "    lo[j] = (_Float16)((x[j] - (float)h) * SPLIT_SCALE);", "    lo[j] = (_Float16)0.f;"),
    ],
    "dx_no_scatter": [
        ("nc_mlp.hip", "          grid_scatter(G, co, dcv, valid, slice, i, g, lane);", "          (void)slice;"),
    ],
    "dx_no_atomic": [
        ("nc_grid.h", "o[a] >= 0) atomicAdd(G.grad + o[a] + chs, v[a]);", "o[a] == -7) atomicAdd(G.grad + o[a] + chs, v[a]);"),
    ],
    "dx_no_coord": [
        ("nc_mlp.hip", "      if (need_coord) {\n        float gi[3]", "      if (false) {\n        float gi[3]"),
    ],
    "dw_no_mfma": [
        ("nc_mlp.hip", "      constexpr int NC = decltype(nchains)::value;\n",
         "      constexpr int NC = decltype(nchains)::value;\n      return;\n"),
    ],
    "no_sort": [
        ("nc_rays.hip", "  if (c.n_surf > 0 || c.n_extra > 0) {  // Renderer.py:222-224", "  if (false) {  // Renderer.py:222-224"),
    ],
    "vsin": [  # the round-5 Fourier sin / cos: [-pi, pi] Cody-Waite + hardware v_sin_f32 / v_cos_f32
        ("nc_device.h", "__device__ __forceinline__ f2 fourier_sin2(f2 x) {\n",
         "__device__ __forceinline__ f2 fourier_sin2(f2 x) {\n" + _VSIN2),
        ("nc_device.h", "__device__ __forceinline__ float fourier_sin(float x) {\n",
         "__device__ __forceinline__ float fourier_sin(float x) {\n  return __builtin_amdgcn_sinf(_vs_rev(x));\n"),
        ("nc_device.h", "__device__ __forceinline__ float fourier_cos(float x) {\n",
         "__device__ __forceinline__ float fourier_cos(float x) {\n  return __builtin_amdgcn_cosf(_vs_rev(x));\n"),
        ("nc_device.h", "// t = x - k pi and (-1)^k as a sign bit\n", _VSREV + "// t = x - k pi and (-1)^k as a sign bit\n"),
    ],
    "fwd_no_mlp": [  # k_mlp_fwd: prologue, gathers and feature stores only (no decoder MLP)
        ("nc_mlp.hip", "      wave_forward_h<KIND, T>(reinterpret_cast<const char*>(lds), i, g, R, out, rec, job.keep_h != 0, amax);",
         "      { for (int t = 0; t < T; ++t) for (int o = 0; o < 4; ++o) out[t][o] = R[t].c[o]; }"),
    ],
    "gather_hot": [  # every corner row read from grid row 0 (one line: L1 hits; timing only)
        ("nc_device.h", "  return ((c.inb >> k) & 1u) ? G.data + (c.base + corner_delta(G.stride, k)) : kZeroRow;",
         "  return ((c.inb >> k) & 1u) ? G.data : kZeroRow;"),
    ],
    "gather_1mb": [  # corner rows folded into the grid's first 1 MiB (L2-resident, few pages; timing only)
        ("nc_device.h", "  return ((c.inb >> k) & 1u) ? G.data + (c.base + corner_delta(G.stride, k)) : kZeroRow;",
         "  return ((c.inb >> k) & 1u) ? G.data + ((c.base + corner_delta(G.stride, k)) & 0x3ffe0) : kZeroRow;"),
    ],
    "gather_8mb": [  # corner rows folded into the grid's first 8 MiB (timing only)
        ("nc_device.h", "  return ((c.inb >> k) & 1u) ? G.data + (c.base + corner_delta(G.stride, k)) : kZeroRow;",
         "  return ((c.inb >> k) & 1u) ? G.data + ((c.base + corner_delta(G.stride, k)) & 0x1fffe0) : kZeroRow;"),
    ],
    "dx_no_wimage": [  # k_mlp_dx: no copy of its prebuilt f32 weight image (garbage LDS weights;
        # timing only): the prologue's remaining share
        ("nc_mlp.hip", "    for (int e = threadIdx.x; e < Net<KIND, PADW_BWD>::WEIGHTS / 4; e += DX_THREADS) "
                       "reinterpret_cast<float4*>(lds)[e] = src[e];", "    (void)src;"),
    ],
    "wimg_last": [  # k_ray_setup: the weight-image builders after the ray and fill workgroups (round 6's first form)
        ("nc_rays.hip", "  if (blockIdx.x < nbuild) {\n    wimg_block(wi, (int)blockIdx.x);\n    return;\n  }\n"
                        "  const unsigned blk = blockIdx.x - nbuild;\n"
                        "  const unsigned nb = (unsigned)((c.N + RAY_WAVES - 1) / RAY_WAVES);  // ray workgroups\n",
         "  const unsigned nb = (unsigned)((c.N + RAY_WAVES - 1) / RAY_WAVES);  // ray workgroups\n"
         "  if (blockIdx.x >= nb + ray_fill_wgs(c)) {\n    wimg_block(wi, (int)(blockIdx.x - nb - ray_fill_wgs(c)));\n"
         "    return;\n  }\n  const unsigned blk = blockIdx.x;\n  (void)nbuild;\n"),
    ],
    "exact_nolds": [  # k_mlp_fwd_exact (the range guard's no-op pass) launched without its dynamic LDS
        # (timing only: a flagged job would fault; never flagged at C2): what the LDS request costs
        ("nc_mlp.hip", "    hipLaunchKernelGGL(k_mlp_fwd_exact<true>, xgrid, dim3(FWD_THREADS_FUSED), mlp_fwd_exact_lds_bytes(), s, x);",
         "    hipLaunchKernelGGL(k_mlp_fwd_exact<true>, xgrid, dim3(FWD_THREADS_FUSED), 0, s, x);"),
    ],
    "no_exact": [  # no k_mlp_fwd_exact launch at all (timing only): the guard pass's whole cost in the step
        ("nc_mlp.hip", "  if (FWD_F32 || c.range_flag == nullptr) return 0;", "  return 0;"),
    ],
    "swz3_old": [  # the round-5 third-plane swizzle (2-way LDS bank conflicts on its reads; results valid)
        ("nc_device.h", "return 16 * (g ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3));", "return 16 * (g ^ ((row >> 2) & 3));"),
    ],
    "no_zero_fill": [
        ("nc_abi.hip", "  if (a->grad_zero && a->grad_zero_floats > 0) {", "  if (false) {"),
    ],
}
PATCHES["fwd_no_stores"] = PATCHES["no_zero_fill"] + PATCHES["no_recstore"]
PATCHES["dx_no_trilinear"] = PATCHES["dx_no_scatter"] + PATCHES["dx_no_coord"]

DEFINES = {
    "ref": [],
    "mfma_f32": ["-DNC_MFMA_F32"],  # the exact-f32 MFMA forward (a numerics A/B, results valid)
    "wimg4": ["-DNC_WIMG_WGS=4"],  # weight-image builder workgroups per decoder and image
    "wimg16": ["-DNC_WIMG_WGS=16"],
    "dx512": ["-DNC_DX_THREADS=512"],
    "dx1024": ["-DNC_DX_THREADS=1024"],  # 16 waves: 4 per SIMD at <= 128 VGPRs
    "dw512_16": ["-DNC_DW_THREADS=512", "-DNC_DW_NPTS=16"],
    "dw256_16": ["-DNC_DW_THREADS=256", "-DNC_DW_NPTS=16"],
    "dw1024_16": ["-DNC_DW_THREADS=1024", "-DNC_DW_NPTS=16"],
    "dw512_32": ["-DNC_DW_THREADS=512", "-DNC_DW_NPTS=32"],
    "exact1": ["-DNC_EXACT_WGS=1"],
    "exact4": ["-DNC_EXACT_WGS=4"],
    "fused4": ["-DNC_FUSED_RAYS=4"],
    "fused8": ["-DNC_FUSED_RAYS=8"],
    "ft2_512": ["-DNC_FWD_TILES=2", "-DNC_FWD_THREADS_FUSED=512"],
    "ft2_768": ["-DNC_FWD_TILES=2"],
    "ft1_512": ["-DNC_FWD_THREADS_FUSED=512"],
    "ft1_1024": ["-DNC_FWD_THREADS_FUSED=1024"],
    "gather8": ["-DNC_GATHER_CH=8"],
    "fill2": ["-DNC_FILL_WGS_PER_CU=2"],
    "fill3": ["-DNC_FILL_WGS_PER_CU=3"],
    "scat_u2": ["-DNC_SCAT_UNROLL=2"],
    "scat_u4": ["-DNC_SCAT_UNROLL=4"],
    "scat_u16": ["-DNC_SCAT_UNROLL=16"],
    "rs_r4": ["-DNC_RS_ROUNDS=4"],  # NC_DETERMINISTIC=1 runs
    "rs_r16": ["-DNC_RS_ROUNDS=16"],
    "rs_r32": ["-DNC_RS_ROUNDS=32"],
    "dsub32": ["-DNC_DET_DSUB=32"],
    "det_rg4": ["-DNC_DET_RG=4"],
    "det_rg16": ["-DNC_DET_RG=16"],
    "pr8": ["-DNC_PR_AHEAD=8"],
    "pr12": ["-DNC_PR_AHEAD=12"],
    "scan_d4": ["-DNC_RS_SCAN_DIG=4"],
    "scan_d8": ["-DNC_RS_SCAN_DIG=8"],
    "scan_d32": ["-DNC_RS_SCAN_DIG=32"],
}
VARIANTS = sorted(set(DEFINES) | set(PATCHES))


def patched_sources(name, dst):
    """Copy csrc/ to ``dst`` and apply the variant's patches (each anchor exactly once)."""
    from nicecore import build as B
    shutil.copytree(B.CSRC, dst)
    for fname, old, new in PATCHES[name]:
        p = os.path.join(dst, fname)
        with open(p) as fh:
            s = fh.read()
        if s.count(old) != 1:
            raise RuntimeError(f"ablation {name}: anchor found {s.count(old)} times in {fname}: {old[:60]!r}")
        with open(p, "w") as fh:
            fh.write(s.replace(old, new))


def build_variant(name):
    from nicecore import build as B
    out = os.path.join(DBG, f"abl_{name}.so")
    if name in PATCHES:
        with tempfile.TemporaryDirectory(prefix="nicecore_abl_") as tmp:
            src = os.path.join(tmp, "csrc")
            patched_sources(name, src)
            return B.build(force=True, out=out, csrc=src, variant="patch:" + name)
    return B.build(force=True, extra=DEFINES[name], out=out)


def run_variant(name):
    """``cur``: the in-tree product library; any other name: dbg/abl_<name>.so."""
    env = dict(os.environ)
    if name != "cur":
        lib = os.path.join(DBG, f"abl_{name}.so")
        if not os.path.exists(lib):
            print(name, "missing", flush=True)
            return True
        env["NICECORE_LIB"] = lib
        env["NICECORE_ALLOW_STALE"] = "1"  # a variant may be built from another revision (A/B)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "3",
                        "--cpu-seconds", "0"], env=env, capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not line:
        print(name, "FAILED", r.returncode, r.stderr[-2000:], flush=True)
        return False
    d = json.loads(line[-1])
    ks = d["kernels_ms"]
    print(f"{name:14s} step {d['ms_per_step']:.4f} ms  " +
          "  ".join(f"{k.replace('k_', '')} {v * 1e3:.1f}" for k, v in ks.items()), flush=True)
    return True


if __name__ == "__main__":
    cmd = sys.argv[1]
    names = sys.argv[2:] or VARIANTS
    if cmd == "build":
        os.makedirs(DBG, exist_ok=True)
        for n in names:
            print(build_variant(n), flush=True)
    elif cmd == "check":  # every patch still applies (CPU test)
        for n in PATCHES:
            with tempfile.TemporaryDirectory() as tmp:
                patched_sources(n, os.path.join(tmp, "csrc"))
        print("all", len(PATCHES), "patches apply")
    else:
        for n in names:
            if not run_variant(n):
                break
