"""ctypes binding of libnicecore.so (include/nicecore.h).

The product path calls ONLY this library for the render hot path; if it cannot
be loaded on a HIP device the call fails loudly (no PyTorch fallback).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int, c_int32, c_int64, c_size_t, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libnicecore.so")

NC_ABI_VERSION = 11
NC_SAVE_FOR_BACKWARD = 1
NC_DETERMINISTIC = 2
NC_SAVE_POINT_JACOBIAN = 4
NC_DEFER_PARAM_GRADS = 8


def NC_NO_WEIGHT_GRAD(kind: int) -> int:
    """include/nicecore.h: the backward will not ask for decoder ``kind``'s weight gradient."""
    return 16 << kind


NC_LOSS_NONE, NC_LOSS_MAPPER, NC_LOSS_TRACKER = 0, 1, 2
NC_LOSS_COLOR, NC_LOSS_DYNAMIC = 1, 2
NC_MAX_SAMPLES = 64
NC_MAX_SURF = 32

STAGES = {"coarse": 0, "middle": 1, "fine": 2, "color": 3}
DEC_COARSE, DEC_MIDDLE, DEC_FINE, DEC_COLOR = 0, 1, 2, 3
DECODER_NAMES = ("coarse", "middle", "fine", "color")
GRID_KEYS = ("grid_coarse", "grid_middle", "grid_fine", "grid_color")
# decoders (enum nc_decoder) evaluated per stage (decoder.py:341-370)
STAGE_DECODERS = {0: (DEC_COARSE,), 1: (DEC_MIDDLE,), 2: (DEC_FINE, DEC_MIDDLE),
                  3: (DEC_FINE, DEC_MIDDLE, DEC_COLOR)}
# grids each stage reads (the fine decoder also samples grid_middle, decoder.py:199-201)
STAGE_GRIDS = {0: (0,), 1: (1,), 2: (1, 2), 3: (1, 2, 3)}


class NcGrid(ctypes.Structure):
    _fields_ = [("data", c_void_p), ("grad", c_void_p), ("dims", c_int64 * 3),
                ("stride", c_int64 * 4), ("grad_stride", c_int64 * 4),
                ("grad_rows", c_void_p), ("row_voxel", c_void_p), ("row_count", c_void_p),
                ("row_capacity", c_int64)]


class NcDecoderParams(ctypes.Structure):
    _fields_ = [("fc_w", c_void_p * 5), ("fc_b", c_void_p * 5), ("fourier_B", c_void_p),
                ("lin_w", c_void_p * 5), ("lin_b", c_void_p * 5), ("out_w", c_void_p),
                ("out_b", c_void_p), ("grad", c_void_p), ("bound", (c_double * 2) * 3)]


class NcRenderArgs(ctypes.Structure):
    _fields_ = [("abi_version", c_int32), ("stage", c_int32), ("n_rays", c_int64),
                ("n_strat", c_int32), ("n_surf", c_int32), ("flags", c_int32), ("lindisp", c_int32),
                ("rays_o", c_void_p), ("rays_d", c_void_p), ("gt_depth", c_void_p),
                ("depth_max", c_void_p), ("bound", (c_double * 2) * 3),
                ("t_strat", c_float * NC_MAX_SAMPLES), ("t_surf", c_double * NC_MAX_SURF),
                ("grids", NcGrid * 4), ("dec", NcDecoderParams * 4),
                ("depth", c_void_p), ("var", c_void_p), ("color", c_void_p),
                ("g_depth", c_void_p), ("g_var", c_void_p), ("g_color", c_void_p),
                ("g_rays_o", c_void_p), ("g_rays_d", c_void_p),
                ("loss", c_int32), ("loss_flags", c_int32), ("w_color", c_double),
                ("loss_depth", c_void_p), ("loss_color", c_void_p), ("loss_out", c_void_p), ("g_loss", c_void_p),
                ("grad_zero", c_void_p), ("grad_zero_floats", c_int64),
                ("z_extra", c_void_p), ("n_extra", c_int32), ("reserved3", c_int32),
                ("z_out", c_void_p), ("weights_out", c_void_p), ("t_rand", c_void_p),
                ("ray_valid", c_void_p)]


class NcPointsArgs(ctypes.Structure):
    _fields_ = [("abi_version", c_int32), ("stage", c_int32), ("n_points", c_int64),
                ("flags", c_int32), ("reserved", c_int32), ("pts", c_void_p), ("grids", NcGrid * 4), ("dec", NcDecoderParams * 4),
                ("raw", c_void_p), ("g_raw", c_void_p), ("g_pts", c_void_p)]


NC_POSE_F32, NC_POSE_F64 = 0, 1


class NcSampleArgs(ctypes.Structure):
    _fields_ = [("abi_version", c_int32), ("pose_dtype", c_int32), ("n_frames", c_int64),
                ("n_per_frame", c_int64), ("H0", c_int64), ("H1", c_int64), ("W0", c_int64),
                ("W1", c_int64), ("fx", c_float), ("fy", c_float), ("cx", c_float), ("cy", c_float),
                ("c2w", c_void_p), ("c2w_stride", c_int64 * 3), ("indices", c_void_p),
                ("pix_i", c_void_p), ("pix_j", c_void_p), ("frame_ids", c_void_p), ("depth", c_void_p), ("depth_stride", c_int64 * 3), ("color", c_void_p),
                ("color_stride", c_int64 * 4), ("bound", c_void_p), ("rays_o", c_void_p),
                ("rays_d", c_void_p), ("gt_depth", c_void_p), ("gt_color", c_void_p),
                ("inside", c_void_p), ("g_rays_o", c_void_p), ("g_rays_d", c_void_p),
                ("g_c2w", c_void_p), ("cam", c_void_p), ("cam_stride", c_int64 * 2), ("g_cam", c_void_p)]


class NcFrustumArgs(ctypes.Structure):
    _fields_ = [("abi_version", c_int32), ("reserved", c_int32), ("nx", c_int64), ("ny", c_int64),
                ("nz", c_int64), ("xs", c_void_p), ("ys", c_void_p), ("zs", c_void_p),
                ("w2c", c_float * 16), ("cam_o", c_float * 3), ("reserved2", c_float),
                ("fx", c_double), ("fy", c_double), ("cx", c_double), ("cy", c_double),
                ("depth", c_void_p), ("H", c_int64), ("W", c_int64), ("depth_stride", c_int64 * 2),
                ("mask", c_void_p), ("scratch", c_void_p)]


class NcGridRowsArgs(ctypes.Structure):
    _fields_ = [("abi_version", c_int32), ("op", c_int32), ("n_rows", c_int64), ("rows", c_void_p),
                ("grid", c_void_p), ("channels", c_int64), ("dims", c_int64 * 3), ("stride", c_int64 * 4),
                ("packed", c_void_p)]


NC_ROWS_GATHER, NC_ROWS_SCATTER, NC_ROWS_ZERO = 0, 1, 2


class NcSparseRows(ctypes.Structure):
    _fields_ = [("grad_rows", c_void_p), ("n_voxels", c_int64), ("row_voxel", c_void_p),
                ("row_count", c_void_p), ("capacity", c_int64), ("values", c_void_p)]


class NcPdfArgs(ctypes.Structure):
    _fields_ = [("abi_version", c_int32), ("det", c_int32), ("n_rays", c_int64), ("n_bins", c_int64),
                ("n_samples", c_int64), ("bins", c_void_p), ("bins_stride", c_int64),
                ("weights", c_void_p), ("weights_stride", c_int64), ("u", c_void_p), ("u_stride", c_int64),
                ("samples", c_void_p), ("samples_stride", c_int64)]


class NcAdamArgs(ctypes.Structure):
    _fields_ = [("abi_version", c_int32), ("mode", c_int32), ("n", c_int64), ("param", c_void_p),
                ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p), ("row_voxel", c_void_p),
                ("row_count", c_void_p), ("row_capacity", c_int64), ("voxel_stride", c_int64),
                ("channel_stride", c_int64), ("lr", c_double), ("beta1", c_double), ("beta2", c_double),
                ("eps", c_double), ("weight_decay", c_double), ("step", c_double)]


class NcAdamSegment(ctypes.Structure):
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("n", c_int64), ("lr", c_double), ("weight_decay", c_double), ("step", c_double),
                ("step_dev", c_void_p)]


class NcImapParams(ctypes.Structure):
    _fields_ = [("fourier_B", c_void_p), ("lin_w", c_void_p * 4), ("lin_b", c_void_p * 4),
                ("out_w", c_void_p), ("out_b", c_void_p), ("grad", c_void_p)]


class NcImapRenderArgs(ctypes.Structure):
    _fields_ = [("abi_version", c_int32), ("flags", c_int32), ("n_rays", c_int64),
                ("n_strat", c_int32), ("n_extra", c_int32),
                ("rays_o", c_void_p), ("rays_d", c_void_p), ("gt_depth", c_void_p), ("depth_max", c_void_p),
                ("bound", (c_double * 2) * 3), ("t_strat", c_float * NC_MAX_SAMPLES), ("dec", NcImapParams),
                ("depth", c_void_p), ("var", c_void_p), ("color", c_void_p),
                ("g_depth", c_void_p), ("g_var", c_void_p), ("g_color", c_void_p),
                ("g_rays_o", c_void_p), ("g_rays_d", c_void_p),
                ("z_extra", c_void_p), ("z_out", c_void_p), ("weights_out", c_void_p)]


class NcImapPointsArgs(ctypes.Structure):
    _fields_ = [("abi_version", c_int32), ("flags", c_int32), ("n_points", c_int64), ("pts", c_void_p),
                ("dec", NcImapParams), ("raw", c_void_p), ("g_raw", c_void_p), ("g_pts", c_void_p)]


NC_ADAM_DENSE = 0
NC_ADAM_SPARSE_ROWS = 1

EXPORTS = {
    "nc_abi_version": (c_int, []),
    "nc_last_error": (ctypes.c_char_p, []),
    "nc_build_id": (ctypes.c_char_p, []),
    "nc_param_count": (c_int64, [c_int]),
    "nc_struct_size": (c_size_t, [c_int]),
    "nc_render_workspace_bytes": (c_size_t, [POINTER(NcRenderArgs)]),
    "nc_render_forward": (c_int, [POINTER(NcRenderArgs), c_void_p, c_size_t, c_void_p]),
    "nc_render_backward": (c_int, [POINTER(NcRenderArgs), c_void_p, c_size_t, c_void_p]),
    "nc_render_backward_params": (c_int, [POINTER(NcRenderArgs), c_void_p, c_size_t, c_void_p]),
    "nc_timing_start": (c_int, [ctypes.c_uint32]),
    "nc_timing_stop": (c_int, [POINTER(c_double), POINTER(c_int64), c_int]),
    "nc_profile_report": (c_int, []),
    "nc_kernel_name": (ctypes.c_char_p, [c_int]),
    "nc_points_workspace_bytes": (c_size_t, [POINTER(NcPointsArgs)]),
    "nc_points_forward": (c_int, [POINTER(NcPointsArgs), c_void_p, c_size_t, c_void_p]),
    "nc_points_backward": (c_int, [POINTER(NcPointsArgs), c_void_p, c_size_t, c_void_p]),
    "nc_sample_rays_forward": (c_int, [POINTER(NcSampleArgs), c_void_p]),
    "nc_sample_rays_backward": (c_int, [POINTER(NcSampleArgs), c_void_p]),
    "nc_frustum_mask": (c_int, [POINTER(NcFrustumArgs), c_void_p]),
    "nc_grid_rows": (c_int, [POINTER(NcGridRowsArgs), c_void_p]),
    "nc_sample_pdf": (c_int, [POINTER(NcPdfArgs), c_void_p]),
    "nc_adam_step": (c_int, [POINTER(NcAdamArgs), c_void_p]),
    "nc_adam_step_multi": (c_int, [POINTER(NcAdamArgs), POINTER(NcAdamSegment), c_int32, c_void_p]),
    "nc_sparse_rows_clear": (c_int, [POINTER(NcSparseRows), c_void_p]),
    "nc_imap_param_count": (c_int64, []),
    "nc_imap_render_workspace_bytes": (c_size_t, [POINTER(NcImapRenderArgs)]),
    "nc_imap_render_forward": (c_int, [POINTER(NcImapRenderArgs), c_void_p, c_size_t, c_void_p]),
    "nc_imap_render_backward": (c_int, [POINTER(NcImapRenderArgs), c_void_p, c_size_t, c_void_p]),
    "nc_imap_points_workspace_bytes": (c_size_t, [POINTER(NcImapPointsArgs)]),
    "nc_imap_points_forward": (c_int, [POINTER(NcImapPointsArgs), c_void_p, c_size_t, c_void_p]),
    "nc_imap_points_backward": (c_int, [POINTER(NcImapPointsArgs), c_void_p, c_size_t, c_void_p]),
    "nc_imap_points_activation_offset": (c_int64, [POINTER(NcImapPointsArgs), c_int]),
    "nc_sparse_merge_temp_bytes": (c_size_t, [c_int64, c_int64]),
    "nc_sparse_rows_merge": (c_int, [POINTER(NcSparseRows), POINTER(NcSparseRows), c_void_p, c_void_p,
                                     c_int32, c_int64, c_void_p, c_size_t, c_void_p]),
}

_lib = None


class NiceCoreError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and type the exports of libnicecore.so."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or os.environ.get("NICECORE_LIB", LIB_PATH)
    if p == LIB_PATH:
        _ensure_current(p)
    if not os.path.exists(p):
        raise NiceCoreError(
            f"libnicecore.so not found at {p}; build it with `python -m nicecore.build` "
            "(hipcc --offload-arch=gfx950). There is no CPU/PyTorch fallback.")
    lib = ctypes.CDLL(p)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.nc_abi_version() != NC_ABI_VERSION:
        raise NiceCoreError("libnicecore.so ABI version mismatch; rebuild it")
    want = tree_build_id()
    got = lib.nc_build_id().decode()
    if want is not None and p != LIB_PATH and "+" in got and got.split("+")[0] == want:
        import sys  # a variant build of these sources (tools/ablate.py), named explicitly
        print(f"nicecore: loading variant library {p} (build id {got})", file=sys.stderr, flush=True)
    elif want is not None and got != want and os.environ.get("NICECORE_ALLOW_STALE") != "1":
        raise NiceCoreError(f"{p} was built from other sources (nc_build_id {got}, this tree {want}); "
                            "rebuild it with `python -m nicecore.build`")
    _lib = lib
    if os.environ.get("NICE_CORE_PROFILE") == "1":  # per-kernel timings at exit
        import atexit
        atexit.register(lib.nc_profile_report)
    return lib


def tree_build_id() -> str | None:
    """The source hash of the csrc/ tree next to this package (None when the sources
    are not there, e.g. an installed copy without them)."""
    from . import build as B
    if not os.path.isdir(B.CSRC) or not os.path.exists(os.path.join(B.INCLUDE, "nicecore.h")):
        return None
    return B.source_hash()


def _ensure_current(p: str):
    """The in-tree library must be built from the tree's sources: a stale or missing
    binary is rebuilt when hipcc is present (a message on stderr says so), and the
    load below refuses it otherwise -- a forgotten rebuild cannot run old kernels."""
    from . import build as B
    want = tree_build_id()
    if want is None or B.library_build_id(p) == want or os.environ.get("NICECORE_ALLOW_STALE") == "1":
        return
    if B.have_hipcc() and os.environ.get("NICECORE_NO_AUTOBUILD") != "1":
        import sys
        print(f"nicecore: {p} does not match the sources (build id {B.library_build_id(p)} vs {want}); "
              "rebuilding", file=sys.stderr, flush=True)
        B.build()  # under the build lock: concurrent ranks build once


def raw_stream(device) -> int:
    """hipStream_t of torch's current stream on ``device`` (the value of
    torch.cuda.current_stream(device).cuda_stream, without building the stream object)."""
    import torch
    if not isinstance(device, torch.device):
        device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return torch._C._cuda_getCurrentRawStream(idx)


def check(rc: int, what: str):
    if rc != 0:
        msg = load().nc_last_error()
        raise NiceCoreError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


KERNEL_IDS = {"k_depth_max": 0, "k_ray_setup": 1, "k_mlp_fwd": 2, "k_composite_fwd": 3,
              "k_composite_bwd": 4, "k_mlp_dx": 5, "k_param_reduce": 6, "k_ray_grads": 7,
              "k_points_assemble": 8, "k_points_split_grad": 9, "k_points_grads": 10,
              "k_grid_bwd": 11, "k_mlp_dw": 12, "k_grid_gather": 13, "k_loss": 14, "k_det_scatter": 15,
              "k_sample_rays": 16, "k_sample_pose_grad": 17, "k_frustum_mask": 18,
              "k_rows_clear": 19, "k_rows_merge": 20, "k_rows_compact": 21,
              "k_param_ray_reduce": 22, "k_sample_pdf": 23, "k_adam": 24,
              "k_imap_gemm": 25, "k_imap_fourier": 26, "k_grid_rows": 27, "k_composite_fwd_loss": 28}


class KernelTimer:
    """HIP-event timing of the library's kernels on their launch stream."""

    def __init__(self, kernels=None):
        ids = KERNEL_IDS.values() if kernels is None else [KERNEL_IDS[k] for k in kernels]
        self.mask = 0
        for i in ids:
            self.mask |= 1 << i
        self.result = {}

    def __enter__(self):
        load().nc_timing_start(self.mask)
        return self

    def __exit__(self, *exc):
        lib = load()
        n = 32
        ms = (c_double * n)()
        cnt = (c_int64 * n)()
        k = lib.nc_timing_stop(ms, cnt, n)
        if k < 0:
            check(k, "nc_timing_stop")
        self.result = {lib.nc_kernel_name(i).decode(): (ms[i], cnt[i]) for i in range(k) if cnt[i] > 0}
        return False
