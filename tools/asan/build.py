"""Build tools/asan/abi_host_check: the host side of libnicecore under AddressSanitizer +
UndefinedBehaviorSanitizer.

Every csrc/*.hip is compiled with ``-Xarch_host -fsanitize=address -Xarch_host
-fsanitize=undefined`` (the sanitizers on host code only, as the GPU pool requires; the
gfx950 device code is built unchanged, and the driver never launches it), then linked with
abi_host_check.cpp.  Output: build/asan/abi_host_check (git-ignored).

    python tools/asan/build.py [--run]
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "nice-slam-annotation_amd"))
from nicecore import build as B  # noqa: E402

OUT_DIR = os.path.join(REPO, "build", "asan")
EXE = os.path.join(OUT_DIR, "abi_host_check")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]
FLAGS = [f"--offload-arch={B.ARCH}", "-O1", "-g", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-I", B.INCLUDE, "-I", B.CSRC, *SAN]


def _stale(exe, deps):
    if not os.path.exists(exe):
        return True
    t = os.path.getmtime(exe)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False) -> str:
    srcs = [os.path.join(B.CSRC, s) for s in B.SOURCES]
    driver = os.path.join(HERE, "abi_host_check.cpp")
    deps = srcs + [driver, os.path.join(B.INCLUDE, "nicecore.h")] + \
        [os.path.join(B.CSRC, f) for f in os.listdir(B.CSRC) if f.endswith(".h")]
    if not force and not _stale(EXE, deps):
        return EXE
    os.makedirs(OUT_DIR, exist_ok=True)
    objs = [os.path.join(OUT_DIR, os.path.basename(s) + ".o") for s in srcs]

    def cc(k):
        return subprocess.run([B.hipcc(), *FLAGS, "-c", srcs[k], "-o", objs[k]], capture_output=True, text=True)
    with ThreadPoolExecutor(min(8, os.cpu_count() or 4)) as ex:
        res = list(ex.map(cc, range(len(srcs))))
    for s, r in zip(srcs, res):
        if r.returncode:
            raise RuntimeError(f"hipcc (asan, host only) failed on {s}:\n{r.stdout}{r.stderr}")
    drv_o = os.path.join(OUT_DIR, "abi_host_check.o")
    r = subprocess.run([B.hipcc(), "-O1", "-g", "-std=c++17", *SAN, "-I", B.INCLUDE, "-c", driver, "-o", drv_o],
                       capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(f"driver compile failed:\n{r.stdout}{r.stderr}")
    r = subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", *SAN, "-o", EXE + ".tmp", drv_o, *objs],
                       capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(f"link failed:\n{r.stdout}{r.stderr}")
    os.replace(EXE + ".tmp", EXE)
    return EXE


def run(exe: str | None = None) -> subprocess.CompletedProcess:
    env = dict(os.environ)
    # the HIP runtime keeps allocations alive to process exit: leaks are not this check's subject
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    return subprocess.run([exe or EXE], capture_output=True, text=True, env=env, timeout=300)


if __name__ == "__main__":
    exe = build(force="--force" in sys.argv)
    print(exe)
    if "--run" in sys.argv:
        r = run(exe)
        print(r.stdout + r.stderr)
        sys.exit(r.returncode)
