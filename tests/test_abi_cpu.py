"""C-ABI checks that need no GPU: the library loads, exports every symbol the
header declares, the ctypes mirror matches the C struct layout, and the flat
parameter counts match the decoder modules."""
import ctypes
import os
import re

import pytest

from conftest import REPO
from nicecore import _lib as L
from nicecore import build as B
from nicecore import decoder as D
from nicecore.render_fn import decoder_params


@pytest.fixture(scope="module")
def lib():
    B.build()
    return L.load()


def declared_symbols():
    hdr = open(os.path.join(REPO, "include", "nicecore.h")).read()
    return sorted(set(re.findall(r"\b(nc_[a-z_]+)\s*\(", hdr)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(L.EXPORTS)


def test_every_declared_symbol_is_exported(lib):
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_library_binds_every_symbol_now():
    """dlopen with RTLD_NOW: an internal function left undefined (a launcher removed while
    a caller remains) fails here instead of at its first call on the GPU."""
    ctypes.CDLL(B.LIB, mode=os.RTLD_NOW | os.RTLD_LOCAL)


def test_build_id_matches_the_tree(lib):
    """The loaded library was compiled from these sources: its
    nc_build_id() is the tree's source hash, also readable from the file's bytes."""
    want = B.source_hash()
    assert lib.nc_build_id().decode() == want
    assert B.library_build_id(B.LIB) == want
    assert not B.needs_build()
    print("nc_build_id", want)


def test_stale_library_is_refused(tmp_path, monkeypatch):
    """A binary built from other sources is refused by load() (no silent old kernels)."""
    stale = tmp_path / "libnicecore.so"
    data = open(B.LIB, "rb").read()
    i = data.find(B.BUILD_ID_TAG) + len(B.BUILD_ID_TAG)
    stale.write_bytes(data[:i] + b"0123456789abcdef" + data[i + 16:])
    assert B.library_build_id(str(stale)) == "0123456789abcdef"
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(L.NiceCoreError, match="other sources"):
        L.load(str(stale))
    monkeypatch.setattr(L, "_lib", None)
    L.load()


def test_struct_layouts_match(lib):
    assert lib.nc_struct_size(0) == ctypes.sizeof(L.NcRenderArgs)
    assert lib.nc_struct_size(1) == ctypes.sizeof(L.NcPointsArgs)
    assert lib.nc_struct_size(2) == ctypes.sizeof(L.NcGrid)
    assert lib.nc_struct_size(3) == ctypes.sizeof(L.NcDecoderParams)
    assert lib.nc_struct_size(4) == ctypes.sizeof(L.NcSampleArgs)
    assert lib.nc_struct_size(5) == ctypes.sizeof(L.NcFrustumArgs)
    assert lib.nc_struct_size(6) == ctypes.sizeof(L.NcSparseRows)
    assert lib.nc_struct_size(7) == ctypes.sizeof(L.NcPdfArgs)
    assert lib.nc_struct_size(10) == ctypes.sizeof(L.NcImapRenderArgs)
    assert lib.nc_struct_size(11) == ctypes.sizeof(L.NcImapPointsArgs)
    assert lib.nc_struct_size(12) == ctypes.sizeof(L.NcImapParams)
    assert lib.nc_struct_size(13) == ctypes.sizeof(L.NcGridRowsArgs)
    assert lib.nc_abi_version() == L.NC_ABI_VERSION


def test_grid_rows_argument_errors(lib):
    """nc_grid_rows validates before touching the device (no GPU here)."""
    a = L.NcGridRowsArgs()
    a.abi_version = L.NC_ABI_VERSION
    a.op, a.n_rows, a.channels = 7, 0, 32
    a.dims[0] = a.dims[1] = a.dims[2] = 4
    assert lib.nc_grid_rows(ctypes.byref(a), None) == -1  # unknown op
    a.op = L.NC_ROWS_GATHER
    a.n_rows = 5  # NULL rows / grid / packed
    assert lib.nc_grid_rows(ctypes.byref(a), None) == -1
    a.abi_version = 7
    assert lib.nc_grid_rows(ctypes.byref(a), None) == -2
    a.abi_version, a.n_rows = L.NC_ABI_VERSION, 0
    assert lib.nc_grid_rows(ctypes.byref(a), None) == 0  # nothing to move


def test_kernel_timer_ids_match_library(lib):
    """KernelTimer's name -> id table is the library's own (nc_kernel_name), every id."""
    lib.nc_kernel_name.restype = ctypes.c_char_p
    n = lib.nc_timing_stop(None, None, 0)
    names = {lib.nc_kernel_name(i).decode(): i for i in range(n)}
    assert names == L.KERNEL_IDS
    assert n <= 32  # one bit per kernel in nc_timing_start's mask


def test_param_counts_match_modules(lib):
    m = D.build_default_nice(seed=0)
    mods = [m.coarse_decoder, m.middle_decoder, m.fine_decoder, m.color_decoder]
    total = 0
    for k, mod in enumerate(mods):
        ps = decoder_params(mod, k)
        assert [id(p) for p in ps] == [id(p) for p in mod.parameters()]  # flat order == parameters()
        n = sum(p.numel() for p in ps)
        assert lib.nc_param_count(k) == n
        total += n
    assert total == 58956


def test_bad_args_fail_loudly(lib):
    a = L.NcRenderArgs()
    a.abi_version = 999
    assert lib.nc_render_workspace_bytes(ctypes.byref(a)) == 0
    assert b"ABI" in lib.nc_last_error()
    a.abi_version = L.NC_ABI_VERSION
    a.stage = 7
    assert lib.nc_render_forward(ctypes.byref(a), None, 0, None) < 0
    assert b"stage" in lib.nc_last_error()


def test_loss_args_validated(lib):
    """The fused-loss fields (ABI v3) are checked before any launch."""
    def args(**kw):
        a = L.NcRenderArgs()
        a.abi_version = L.NC_ABI_VERSION
        a.stage = L.STAGES["color"]
        a.n_rays, a.n_strat, a.n_surf = 4, 32, 0
        for k, v in kw.items():
            setattr(a, k, v)
        return a

    for kw, msg in ((dict(loss=5), b"unknown loss"),
                    (dict(loss_flags=L.NC_LOSS_COLOR), b"without a loss"),
                    (dict(loss=L.NC_LOSS_MAPPER), b"loss_depth and loss_out"),
                    (dict(loss=L.NC_LOSS_MAPPER, loss_flags=L.NC_LOSS_DYNAMIC, loss_out=8, loss_depth=8),
                     b"handle_dynamic"),
                    (dict(loss=L.NC_LOSS_TRACKER, loss_flags=L.NC_LOSS_COLOR, loss_out=8, loss_depth=8),
                     b"loss_color"),
                    (dict(loss=L.NC_LOSS_TRACKER, loss_flags=8, loss_out=8, loss_depth=8), b"loss_flags")):
        a = args(**kw)
        assert lib.nc_render_workspace_bytes(ctypes.byref(a)) == 0, kw
        assert msg in lib.nc_last_error(), (kw, lib.nc_last_error())


def test_sample_args_validated(lib):
    """nc_sample_rays_* (ABI v4) reject bad arguments before any launch."""
    a = L.NcSampleArgs()
    a.abi_version = L.NC_ABI_VERSION
    a.n_frames, a.n_per_frame = 1, 4
    a.H0, a.H1, a.W0, a.W1 = 0, 4, 0, 4
    a.pose_dtype = 3
    assert lib.nc_sample_rays_forward(ctypes.byref(a), None) < 0
    assert b"pose dtype" in lib.nc_last_error()
    a.pose_dtype = L.NC_POSE_F32
    a.H1 = 0
    assert lib.nc_sample_rays_forward(ctypes.byref(a), None) < 0
    assert b"region" in lib.nc_last_error()
    a.H1 = 4
    assert lib.nc_sample_rays_forward(ctypes.byref(a), None) < 0
    assert b"needs c2w" in lib.nc_last_error() and b"and indices" in lib.nc_last_error()
    a.c2w, a.indices = 8, 8
    assert lib.nc_sample_rays_forward(ctypes.byref(a), None) < 0
    assert b"ray outputs" in lib.nc_last_error()
    a.rays_o, a.rays_d, a.inside = 8, 8, 8
    assert lib.nc_sample_rays_forward(ctypes.byref(a), None) < 0
    assert b"pre-filter" in lib.nc_last_error()
    assert lib.nc_sample_rays_backward(ctypes.byref(a), None) < 0
    assert b"pose gradient" in lib.nc_last_error()


def test_adam_args_validated(lib):
    """nc_adam_step (ABI v7) rejects bad arguments before any launch."""
    assert lib.nc_adam_step(None, None) < 0
    a = L.NcAdamArgs()
    a.abi_version = L.NC_ABI_VERSION - 1
    assert lib.nc_adam_step(ctypes.byref(a), None) == -2
    a.abi_version = L.NC_ABI_VERSION
    a.lr, a.beta1, a.beta2, a.eps, a.step = 1e-3, 0.9, 0.999, 1e-8, 0.0
    assert lib.nc_adam_step(ctypes.byref(a), None) < 0
    assert b"step count" in lib.nc_last_error()
    a.step, a.beta2 = 1.0, 1.0
    assert lib.nc_adam_step(ctypes.byref(a), None) < 0
    assert b"beta" in lib.nc_last_error()
    a.beta2, a.n = 0.999, 16
    assert lib.nc_adam_step(ctypes.byref(a), None) < 0
    assert b"NULL" in lib.nc_last_error()
    a.mode, a.weight_decay = L.NC_ADAM_SPARSE_ROWS, 0.1
    assert lib.nc_adam_step(ctypes.byref(a), None) < 0
    assert b"weight_decay" in lib.nc_last_error()
    a.mode = 7
    assert lib.nc_adam_step(ctypes.byref(a), None) < 0
    assert b"mode" in lib.nc_last_error()


def test_adam_optimizer_contract():
    """nicecore.optim.Adam's constructor: the Mapper's param groups are accepted, the
    unsupported variants are refused (no silent CPU / torch fallback)."""
    import torch
    from nicecore.optim import Adam, _dense_layout
    p = [torch.nn.Parameter(torch.zeros(4)), torch.nn.Parameter(torch.zeros(2, 3))]
    opt = Adam([{"params": [p[0]], "lr": 0}, {"params": [p[1]], "lr": 0.1}])
    assert [g["lr"] for g in opt.param_groups] == [0, 0.1]
    with pytest.raises(NotImplementedError):
        Adam(p, amsgrad=True)
    assert _dense_layout(torch.zeros(1, 32, 3, 4, 5).contiguous(memory_format=torch.channels_last_3d))
    assert not _dense_layout(torch.zeros(4, 6)[:, :3])


def test_imap_param_count_matches_module(lib):
    """nc_imap_param_count == the iMAP* MLP's parameter count (config.py:28-32)."""
    m = D.build_imap(seed=0)
    assert lib.nc_imap_param_count() == sum(p.numel() for p in m.parameters()) == 222747


def test_host_abi_under_address_sanitizer():
    """the host side of the ABI (argument validation, stage plans, workspace
    layouts of every entry point over the BASELINE shapes, malformed calls) built with
    -Xarch_host -fsanitize=address,undefined (tools/asan/build.py) and run without a GPU:
    no sanitizer report, every documented result holds."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("nicecore_asan_build", os.path.join(REPO, "tools", "asan", "build.py"))
    asan_build = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(asan_build)
    exe = asan_build.build()
    r = asan_build.run(exe)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert "abi_host_check: ok" in out
