"""Build libnicecore.so (HIP, gfx950) in-tree with hipcc.

    python -m nicecore.build            # from nice-slam-annotation_amd/
    python nice-slam-annotation_amd/nicecore/build.py

The library is plain C ABI (include/nicecore.h); it does not link against torch.
-ffp-contract=off keeps the reference's float association (ray sampling and
trilinear weights are bit-identical to the CPU path); FMAs the kernels want are
explicit (__builtin_fmaf, MFMA).
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
REPO = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(HERE, "libnicecore.so")
SOURCES = ["nc_abi.hip", "nc_rays.hip", "nc_mlp.hip", "nc_grid.hip", "nc_det.hip", "nc_sample.hip", "nc_frustum.hip", "nc_adam.hip",
           "nc_sparse.hip", "nc_pdf.hip", "nc_imap.hip"]
ARCH = os.environ.get("NICECORE_ARCH", "gfx950")


SRC_EXT = (".hip", ".h", ".hpp", ".cpp")
BUILD_ID_TAG = b"nicecore-src-"


def source_hash() -> str:
    """sha256 (first 16 hex digits) over the library's sources: every csrc/ file and
    include/nicecore.h, by name and content.  Compiled into the library
    (``nc_build_id()``) so that a loaded binary can be matched to the tree it sits in."""
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith(SRC_EXT))
    for name, path in [(f, os.path.join(CSRC, f)) for f in files] + [("nicecore.h", os.path.join(INCLUDE, "nicecore.h"))]:
        h.update(name.encode() + b"\0")
        with open(path, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def variant_suffix(extra=(), arch: str | None = None) -> str:
    """'' for the product library (gfx950, no extra flags); '+<8 hex>' over the extra
    compile flags and the target otherwise, so a variant library (tools/ablate.py timing
    builds, another arch) carries a build id of its own: ``<source hash>+<variant>``."""
    arch = arch or ARCH
    if not extra and arch == "gfx950":
        return ""
    return "+" + hashlib.sha256((" ".join(extra) + "|" + arch).encode()).hexdigest()[:8]


def library_build_id(path: str = LIB) -> str | None:
    """The build id embedded in a built library (source hash, plus ``+<variant>`` for a
    variant build), read from its bytes (no dlopen)."""
    try:
        with open(path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    i = data.find(BUILD_ID_TAG)
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + len(BUILD_ID_TAG):j if j > 0 else i + len(BUILD_ID_TAG) + 25].decode("ascii", "replace")


def have_hipcc() -> bool:
    try:
        hipcc()
        return True
    except RuntimeError:
        return False


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libnicecore.so)")


def needs_build() -> bool:
    """True unless the library exists and was built from exactly these sources."""
    return library_build_id(LIB) != source_hash()


def build(force: bool = False, verbose: bool = False, extra=(), out: str | None = None,
          csrc: str | None = None, variant: str = "") -> str:
    """Compile libnicecore.so (or, with ``out``, a variant library at that path --
    timing ablations, tools/ablate.py: extra compile flags, or ``csrc`` = a patched copy
    of the sources, named by ``variant`` in the build id).

    Several processes may call this at once (every rank of a multi-process run loads the
    library): the build runs under an exclusive lock on ``<lib>.lock``, a process that
    waited for the lock re-checks the build id before compiling (so N ranks build once),
    and the link goes to a per-process temporary that is renamed into place atomically
    (a rank never dlopens a half-written file)."""
    import fcntl
    lib = out or LIB
    if out is None and not force and not needs_build():
        return LIB
    with open(lib + ".lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            if out is None and not force and not needs_build():  # built while we waited
                return LIB
            return _build_locked(lib, verbose, extra, csrc or CSRC, variant)
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)


def _build_locked(lib: str, verbose: bool, extra, csrc: str, variant: str) -> str:
    vid = variant_suffix([*extra, variant] if variant else extra)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
             "-Wno-unused-function", "-Wno-unused-variable", "-I", INCLUDE, "-I", csrc,
             f'-DNC_SRC_HASH="{source_hash()}{vid}"', *extra]
    # one hipcc per source in parallel, then one link: the wall time is the slowest file
    with tempfile.TemporaryDirectory(prefix="nicecore_build_") as tmp:
        objs = [os.path.join(tmp, os.path.splitext(s)[0] + ".o") for s in SOURCES]

        def compile_one(k):
            cmd = [hipcc(), *flags, "-c", "-o", objs[k], os.path.join(csrc, SOURCES[k])]
            if verbose:
                print(" ".join(cmd), flush=True)
            return subprocess.run(cmd, capture_output=True, text=True)

        jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
        with ThreadPoolExecutor(jobs) as ex:
            results = list(ex.map(compile_one, range(len(SOURCES))))
        for src, r in zip(SOURCES, results):
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n" + r.stdout + r.stderr)
            if verbose and (r.stdout or r.stderr):
                print(r.stdout + r.stderr)
        tmp_lib = f"{lib}.{os.getpid()}.tmp"
        r = subprocess.run([hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp_lib, *objs],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc link failed:\n" + r.stdout + r.stderr)
    os.replace(tmp_lib, lib)
    return lib


if __name__ == "__main__":
    force = "--force" in sys.argv
    extra = ["-Rpass-analysis=kernel-resource-usage"] if "--resources" in sys.argv else []
    print(build(force=force or bool(extra), verbose=True, extra=extra))
