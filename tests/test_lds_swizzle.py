"""LDS bank conflicts of k_mlp_fwd's split-f16 weight image reads (nc_device.h hchunk /
hchunk3), checked on the host from the header's own constexpr functions.

mac_fwd reads row r = 32 kb + 16 ob + i, 16-byte chunk g of the hi / lo planes (128-B rows)
and of the third plane (64-B rows) with ds_read_b128, lane (i, g) = lane i + 16 g.
MI355X_MICROARCH.md's LDS table: a ds_read_b128 is served in four lane groups
{0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32, one LDS cycle per group when
its lanes touch distinct 16-B slots of the 256-B bank line (identical addresses broadcast).
Round 6 found the third plane 2-way conflicted under that grouping (its swizzle had been
designed for contiguous 16-lane groups); this test pins every plane conflict-free."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "nice-slam-annotation_amd", "csrc")

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[l + 32 for l in grp] for grp in B128_GROUPS]

PROBE = r"""
#include "nc_device.h"
#include <cstdio>
int main() {
  for (int r = 0; r < 64; ++r)
    for (int g = 0; g < 4; ++g)
      std::printf("%d %d %d %d %d\n", r, g, nc::hchunk(r, g, 0), nc::hchunk(r, g, 1), nc::hchunk3(r, g));
}
"""


@pytest.fixture(scope="module")
def chunks(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("swizzle")
    src, exe = d / "probe.cpp", d / "probe"
    src.write_text(PROBE)
    subprocess.run([hipcc, "-x", "hip", "--offload-host-only", "-std=c++17", "-I", os.path.join(REPO, "include"),
                    "-I", CSRC, str(src), "-o", str(exe)], check=True, capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    tab = {}
    for ln in out.split("\n"):
        if ln.strip():
            r, g, c0, c1, c3 = map(int, ln.split())
            tab[(r, g)] = (c0, c1, c3)
    return tab


def _worst_way(addr):
    """max number of distinct 16-B addresses on one bank slot within a b128 lane group"""
    worst = 0
    for base in range(0, 64, 16):  # row blocks 32 kb + 16 ob
        for grp in B128_GROUPS:
            slots = {}
            for lane in grp:
                i, g = lane & 15, lane >> 4
                a = addr(base + i, g)
                slots.setdefault((a // 16) % 16, set()).add(a)
            worst = max(worst, max(len(v) for v in slots.values()))
    return worst


def test_lane_groups_cover_the_wave():
    assert sorted(sum(B128_GROUPS, [])) == list(range(64))


@pytest.mark.parametrize("plane", [0, 1])
def test_hi_lo_planes_conflict_free(chunks, plane):
    assert _worst_way(lambda r, g: r * 128 + chunks[(r, g)][plane]) == 1


def test_third_plane_conflict_free(chunks):
    assert _worst_way(lambda r, g: r * 64 + chunks[(r, g)][2]) == 1


def test_chunks_are_permutations(chunks):
    """every row stores its four chunks (per plane) at four distinct positions"""
    for r in range(64):
        assert sorted([chunks[(r, g)][0] for g in range(4)] + [chunks[(r, g)][1] for g in range(4)]) == \
            [16 * k for k in range(8)]
        assert sorted(chunks[(r, g)][2] for g in range(4)) == [0, 16, 32, 48]
