"""Host-side build plumbing (no GPU, no hipcc run).

* Concurrent loads of a stale library build it ONCE: every rank of a multi-process run
  calls nicecore._lib.load(), which rebuilds a stale in-tree library; nicecore.build takes
  an exclusive lock on <lib>.lock and re-checks the build id after waiting for it, and
  links to a per-process temporary renamed into place.
* Variant builds carry their own build id (<source hash>+<variant>), so a timing or
  numerics variant can never pass for the product library.
* Every timing-ablation patch of tools/ablate.py still applies to the product sources
  (each anchor exactly once): the ablations live outside the product kernels.
"""
import os
import subprocess
import sys
import textwrap

from conftest import REPO

WORKER = textwrap.dedent('''
    import os, sys, time
    sys.path.insert(0, os.path.join({repo!r}, "nice-slam-annotation_amd"))
    from nicecore import build as B
    B.LIB = {lib!r}
    def fake_build(lib, verbose, extra, csrc, variant):  # stands in for hipcc: slow, then one rename
        with open({log!r}, "a") as f:
            f.write(str(os.getpid()) + "\\n")
        time.sleep(1.0)
        tmp = lib + "." + str(os.getpid()) + ".tmp"
        with open(tmp, "wb") as f:
            f.write(b"ELF..." + B.BUILD_ID_TAG + B.source_hash().encode() + b"\\0")
        os.replace(tmp, lib)
        return lib
    B._build_locked = fake_build
    print(B.build())
''')


def test_concurrent_stale_builds_build_once(tmp_path):
    lib = str(tmp_path / "libnicecore.so")
    log = str(tmp_path / "builds.log")
    with open(lib, "wb") as f:
        f.write(b"stale nicecore-src-0000000000000000\0")
    code = WORKER.format(repo=REPO, lib=lib, log=log)
    procs = [subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE)
             for _ in range(4)]
    for p in procs:
        out, err = p.communicate(timeout=120)
        assert p.returncode == 0, err.decode()
    with open(log) as f:
        builders = f.read().split()
    assert len(builders) == 1, builders  # one process compiled, the others found it current
    sys.path.insert(0, os.path.join(REPO, "nice-slam-annotation_amd"))
    from nicecore import build as B
    assert B.library_build_id(lib) == B.source_hash()
    assert not [n for n in os.listdir(tmp_path) if n.endswith(".tmp")]


def test_variant_build_ids():
    sys.path.insert(0, os.path.join(REPO, "nice-slam-annotation_amd"))
    from nicecore import build as B
    assert B.variant_suffix(()) == ""
    a, b = B.variant_suffix(["-DNC_MFMA_F32"]), B.variant_suffix(["-DNC_MFMA_F32", "patch:no_gather"])
    assert a.startswith("+") and len(a) == 9 and a != b
    assert B.variant_suffix((), arch="gfx942") != ""


def test_ablation_patches_apply():
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "ablate.py"), "check"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "patches apply" in r.stdout


def test_product_sources_have_no_ablation_switches():
    csrc = os.path.join(REPO, "nice-slam-annotation_amd", "csrc")
    for name in os.listdir(csrc):
        with open(os.path.join(csrc, name)) as f:
            s = f.read()
        for bad in ("NC_ABL_", "NC_DW_SPLIT16", "NC_FWD_W2", "NC_SPLIT_RTZ", "NC_FWD_GATHER_B2", "NC_DW_PAD_CHAINS"):
            assert bad not in s, (name, bad)
