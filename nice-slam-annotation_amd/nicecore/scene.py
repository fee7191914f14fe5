"""Scene description for the render core: bounds, feature-grid shapes, presets and
seeded synthetic rays.

The grid *store* stays a dict of user-owned torch tensors keyed exactly like the
reference (``grid_coarse``, ``grid_middle``, ``grid_fine``, ``grid_color``), each
``[1, C, Dz, Dy, Dx]`` float32.  Any strides are accepted by the kernels;
``channels_last_3d`` (channel stride 1) is the fast layout because one trilinear
corner is then one 128-byte line.

Reference behaviour restated here:
  * bound snapping            -- src/NICE_SLAM.py:188-208 (load_bound)
  * grid shapes + init        -- src/NICE_SLAM.py:243-320 (grid_init)
  * camera rays from pixels   -- src/common.py:74-89 (get_rays_from_uv)
  * caller-side bbox filter   -- src/Tracker.py:100-111, src/Mapper.py:580-596
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

GRID_KEYS = ("grid_coarse", "grid_middle", "grid_fine", "grid_color")

# Scene presets: mapping.bound + cam intrinsics of the configs the benchmark names.
#   Replica room0     configs/Replica/room0.yaml:3, configs/Replica/replica.yaml:28-34
#   ScanNet 0000      configs/ScanNet/scene0000.yaml:3, configs/ScanNet/scannet.yaml:26-33
#   Apartment         configs/Apartment/apartment.yaml:24-32
# grid_len / rendering / model defaults: configs/nice_slam.yaml:9-14, :121-136
PRESETS = {
    "replica_room0": dict(
        bound=[[-2.9, 8.9], [-3.2, 5.5], [-3.5, 3.3]],
        marching_cubes_bound=[[-2.9, 8.9], [-3.2, 5.5], [-3.5, 3.3]],  # room0.yaml:4
        H=680, W=1200, fx=600.0, fy=600.0, cx=599.5, cy=339.5, crop_edge=0),
    "scannet_scene0000": dict(
        bound=[[-2.0, 11.0], [-2.0, 11.5], [-2.0, 5.5]],
        H=480, W=640, fx=577.590698, fy=578.729797, cx=318.905426, cy=242.683609,
        crop_edge=10),
    "apartment": dict(
        bound=[[-5.8, 11.3], [-4.0, 4.5], [-7.9, 4.9]],
        H=720, W=1280, fx=607.4694213867188, fy=607.4534912109375,
        cx=636.9967041015625, cy=369.2689514160156, crop_edge=0),
    # BASELINE.json configs[4] (C5): synthetic 10 m x 10 m x 3 m scene whose fine and
    # colour grids (0.0118 m) hold ~204M voxels = 26.1 GB each (SURVEY.md §8 header);
    # Replica intrinsics for the synthetic rays.
    "synthetic_c5": dict(
        bound=[[0.0, 10.0], [0.0, 10.0], [0.0, 3.0]],
        H=680, W=1200, fx=600.0, fy=600.0, cx=599.5, cy=339.5, crop_edge=0,
        grid_len=dict(coarse=2.0, middle=0.0236, fine=0.0118, color=0.0118, bound_divisible=0.32)),
    # Tiny scene used by the golden fixtures (grids of a few tens of KB).
    "tiny": dict(
        bound=[[-1.0, 1.0], [-0.5, 0.5], [-0.5, 0.5]],
        H=48, W=64, fx=40.0, fy=40.0, cx=31.5, cy=23.5, crop_edge=0),
}

DEFAULT_GRID_LEN = dict(coarse=2.0, middle=0.32, fine=0.16, color=0.16,
                        bound_divisible=0.32)
DEFAULT_RENDERING = dict(N_samples=32, N_surface=16, N_importance=0,
                         lindisp=False, perturb=0.0)
C_DIM = 32
COARSE_BOUND_ENLARGE = 2


def snap_bound(bound, bound_divisible: float, scale: float = 1.0) -> torch.Tensor:
    """float64 [3,2] bound whose upper edge is enlarged to a multiple of
    ``bound_divisible`` (src/NICE_SLAM.py:196-201).

    The multiple is formed as an int32 tensor times a Python float, which torch
    evaluates in float32; that rounding is part of the contract (e.g. Replica's
    x-max becomes 8.94000015258789), so the same torch expression is used.
    """
    b = torch.from_numpy(np.array(bound, dtype=np.float64) * scale)
    k = ((b[:, 1] - b[:, 0]) / bound_divisible).int() + 1
    b[:, 1] = k * bound_divisible + b[:, 0]
    return b


def grid_shapes(bound: torch.Tensor, grid_len: dict, coarse: bool = True,
                coarse_bound_enlarge: float = COARSE_BOUND_ENLARGE) -> dict:
    """Voxel counts per level as ``[Dz, Dy, Dx]`` (src/NICE_SLAM.py:265-317):
    ``int(len / grid_len)`` per axis, then axes 0 and 2 swapped."""
    xyz_len = bound[:, 1] - bound[:, 0]
    out = {}
    levels = (["coarse"] if coarse else []) + ["middle", "fine", "color"]
    for lv in levels:
        if lv == "coarse":
            s = list(map(int, (xyz_len * coarse_bound_enlarge / grid_len[lv]).tolist()))
        else:
            s = list(map(int, (xyz_len / grid_len[lv]).tolist()))
        s[0], s[2] = s[2], s[0]
        out["grid_" + lv] = s
    return out


GRID_STD = {"grid_coarse": 0.01, "grid_middle": 0.01, "grid_fine": 0.0001,
            "grid_color": 0.01}


def init_grids(shapes: dict, c_dim: int = C_DIM, generator=None, device="cpu",
               channels_last: bool = False, std: dict | None = None) -> dict:
    """N(0, std) feature grids (src/NICE_SLAM.py:289-319; fine uses 1e-4).
    Generated on the CPU in the reference's order so a seed reproduces it."""
    std = GRID_STD if std is None else std
    grids = {}
    for key in GRID_KEYS:
        if key not in shapes:
            continue
        t = torch.zeros([1, c_dim, *shapes[key]]).normal_(mean=0, std=std[key],
                                                          generator=generator)
        t = t.to(device)
        if channels_last:
            t = t.contiguous(memory_format=torch.channels_last_3d)
        grids[key] = t
    return grids


def init_grids_device(shapes: dict, seed: int, device, c_dim: int = C_DIM, channels_last: bool = True,
                      std: dict | None = None) -> dict:
    """N(0, std) grids generated directly in device memory (the multi-GB grids of C5:
    no host copy).  Seeded by a device generator, so not the CPU init's values."""
    std = GRID_STD if std is None else std
    gen = torch.Generator(device=device).manual_seed(seed)
    fmt = torch.channels_last_3d if channels_last else torch.contiguous_format
    grids = {}
    for key in GRID_KEYS:
        if key in shapes:
            t = torch.empty([1, c_dim, *shapes[key]], device=device, memory_format=fmt)
            grids[key] = t.normal_(mean=0, std=std[key], generator=gen)
    return grids


def grids_bytes(shapes: dict, c_dim: int = C_DIM) -> int:
    return sum(4 * c_dim * int(np.prod(s)) for s in shapes.values())


def decoder_bounds(bound: torch.Tensor, coarse_bound_enlarge=COARSE_BOUND_ENLARGE):
    """Per-decoder ``.bound`` as assigned by src/NICE_SLAM.py:202-208."""
    return {"coarse": bound * coarse_bound_enlarge, "middle": bound,
            "fine": bound, "color": bound}


@dataclass
class SceneSpec:
    """Everything needed to build a benchmark / fixture scene."""
    name: str
    bound: torch.Tensor
    shapes: dict
    H: int
    W: int
    fx: float
    fy: float
    cx: float
    cy: float
    grid_len: dict = field(default_factory=lambda: dict(DEFAULT_GRID_LEN))
    # meshing.marching_cubes_bound of the scene's config (Mesher.py:443), else the raw
    # mapping bound
    marching_cubes_bound: torch.Tensor | None = None


def make_scene(name: str, grid_len: dict | None = None) -> SceneSpec:
    p = PRESETS[name]
    gl = dict(grid_len if grid_len is not None else p.get("grid_len", DEFAULT_GRID_LEN))
    bound = snap_bound(p["bound"], gl["bound_divisible"])
    H, W, cx, cy = p["H"], p["W"], p["cx"], p["cy"]
    ce = p.get("crop_edge", 0)
    if ce > 0:  # src/NICE_SLAM.py:181-185
        H, W, cx, cy = H - 2 * ce, W - 2 * ce, cx - ce, cy - ce
    mcb = torch.tensor(p.get("marching_cubes_bound", p["bound"]), dtype=torch.float64)
    return SceneSpec(name, bound, grid_shapes(bound, gl), H, W, p["fx"], p["fy"],
                     cx, cy, gl, mcb)


def mesher_lattice(mc_bound: torch.Tensor, resolution: int, padding: float = 0.05) -> torch.Tensor:
    """Mesher.get_grid_uniform (src/utils/Mesher.py:443-472): a resolution^3 lattice
    over marching_cubes_bound widened by ``padding`` on every side, float32 [R^3, 3] in
    the reference's np.meshgrid ('xy') order."""
    b = np.asarray(mc_bound, dtype=np.float64)
    x, y, z = (np.linspace(b[k][0] - padding, b[k][1] + padding, resolution) for k in range(3))
    xx, yy, zz = np.meshgrid(x, y, z)
    return torch.tensor(np.vstack([xx.ravel(), yy.ravel(), zz.ravel()]).T, dtype=torch.float)


def _random_rotation(gen: torch.Generator) -> torch.Tensor:
    q = torch.randn(4, generator=gen, dtype=torch.float64)
    q = q / q.norm()
    w, x, y, z = q.tolist()
    return torch.tensor([
        [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
        [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
        [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]],
        dtype=torch.float32)


def ray_exit_t(bound: torch.Tensor, rays_o: torch.Tensor, rays_d: torch.Tensor):
    """Slab exit distance ``min_axis max(t0, t1)`` (Renderer.py:145-150), float64."""
    t = (bound.unsqueeze(0) - rays_o.unsqueeze(-1).double()) / rays_d.unsqueeze(-1).double()
    return torch.min(torch.max(t, dim=2)[0], dim=1)[0]


def synth_rays(scene: SceneSpec, n_rays: int, n_poses: int = 40, seed: int = 1,
               edge: int = 0, zero_depth_frac: float = 0.1, outside_frac: float = 0.0, poses_out=None):
    """Seeded synthetic rays per SURVEY.md §8(d).

    Camera centres uniform in the central 60% of the bound, random unit-quaternion
    rotations, pixels uniform in the image (minus ``edge``), rays by
    src/common.py:82-88; gt_depth ~ U(0.3, 0.9 t_exit) with ``zero_depth_frac``
    exact zeros; gt_color ~ U(0,1).  ``outside_frac`` of the cameras are placed
    just outside the bound looking in, so some samples fall out of bound.
    Rays that fail the callers' bbox filter (t_exit >= gt_depth) are redrawn.
    Returns float32 CPU tensors rays_o [N,3], rays_d [N,3], gt_depth [N], gt_color [N,3];
    ``poses_out`` (a list), if given, receives the cameras' (R, t) (c2w = [R | t]).
    """
    gen = torch.Generator().manual_seed(seed)
    b = scene.bound.float()
    lo, hi = b[:, 0], b[:, 1]
    ctr, span = (lo + hi) / 2, (hi - lo)
    poses = []
    for k in range(n_poses):
        R = _random_rotation(gen)
        if k < int(round(outside_frac * n_poses)):
            # outside the box on a random face, looking towards the centre
            axis = int(torch.randint(0, 3, (1,), generator=gen))
            sgn = 1.0 if torch.rand(1, generator=gen).item() < 0.5 else -1.0
            t = ctr + (torch.rand(3, generator=gen) - 0.5) * 0.3 * span
            t[axis] = ctr[axis] + sgn * 0.55 * span[axis]
            fwd = (ctr - t)
            fwd = fwd / fwd.norm()
            # build R so that camera -z looks along fwd
            up = torch.tensor([0.0, 0.0, 1.0]) if abs(fwd[2]) < 0.9 else torch.tensor([0.0, 1.0, 0.0])
            right = torch.linalg.cross(fwd, up); right = right / right.norm()
            up2 = torch.linalg.cross(right, fwd)
            R = torch.stack([right, up2, -fwd], dim=1)
        else:
            t = ctr + (torch.rand(3, generator=gen) - 0.5) * 0.6 * span
        poses.append((R, t))
    if poses_out is not None:
        poses_out.extend(poses)
    out_o, out_d, out_dep = [], [], []
    need = n_rays
    while need > 0:
        m = max(need * 2, 16)
        pid = torch.randint(0, n_poses, (m,), generator=gen)
        i = edge + torch.rand(m, generator=gen) * (scene.W - 2 * edge)
        j = edge + torch.rand(m, generator=gen) * (scene.H - 2 * edge)
        dirs = torch.stack([(i - scene.cx) / scene.fx, -(j - scene.cy) / scene.fy,
                            -torch.ones_like(i)], -1)
        Rs = torch.stack([poses[p][0] for p in pid.tolist()])
        ts = torch.stack([poses[p][1] for p in pid.tolist()])
        rays_d = torch.sum(dirs[:, None, :] * Rs, -1)
        rays_o = ts.clone()
        t_exit = ray_exit_t(scene.bound, rays_o, rays_d).float()
        u = torch.rand(m, generator=gen)
        dep = (0.3 + u * (0.9 * t_exit - 0.3)).clamp_min(0.05)
        zero = torch.rand(m, generator=gen) < zero_depth_frac
        dep = torch.where(zero, torch.zeros_like(dep), dep)
        ok = (t_exit >= dep) & torch.isfinite(t_exit) & (t_exit > 0.35)
        out_o.append(rays_o[ok]); out_d.append(rays_d[ok]); out_dep.append(dep[ok])
        need -= int(ok.sum())
    rays_o = torch.cat(out_o)[:n_rays].contiguous()
    rays_d = torch.cat(out_d)[:n_rays].contiguous()
    gt_depth = torch.cat(out_dep)[:n_rays].contiguous()
    gt_color = torch.rand(n_rays, 3, generator=gen)
    return rays_o, rays_d, gt_depth, gt_color


def bbox_filter(bound: torch.Tensor, rays_o, rays_d, gt_depth, *extra):
    """Callers' pre-filter (src/Tracker.py:100-111, src/Mapper.py:580-596)."""
    with torch.no_grad():
        t = ray_exit_t(bound.to(rays_o.device), rays_o, rays_d)
        keep = t >= gt_depth
    return (rays_o[keep], rays_d[keep], gt_depth[keep]) + tuple(e[keep] for e in extra)


def linspace_tables(n_strat: int, n_surf: int):
    """The reference's sample-position tables exactly as torch builds them on
    the CPU: ``linspace(0,1,N_samples)`` float32 (Renderer.py:203) and
    ``linspace(0,1,N_surface).double()`` (Renderer.py:182-183; float32 values
    promoted to float64)."""
    t = torch.linspace(0.0, 1.0, steps=n_strat)
    ts = torch.linspace(0.0, 1.0, steps=n_surf).double() if n_surf > 0 else torch.zeros(0, dtype=torch.float64)
    return t, ts


def points_per_ray(n_strat: int, n_surf: int) -> int:
    return n_strat + n_surf


def roofline_per_ray(stage: str, S: int, mode: str = "mapper_ba"):
    """Algorithmic FLOPs and bytes per ray (SURVEY.md §8(d) convention)."""
    mac = {"coarse": 6176, "middle": 15479, "fine": 20599, "color": 15575}
    decs = {"coarse": ["coarse"], "middle": ["middle"], "fine": ["fine", "middle"],
            "color": ["fine", "middle", "color"]}[stage]
    lookups_fwd = {"coarse": 1, "middle": 1, "fine": 3, "color": 4}[stage]
    lookups_grad = {"coarse": 1, "middle": 1, "fine": 2, "color": 3}[stage]
    macs = sum(mac[d] for d in decs)
    tri = 8 * C_DIM * 2
    fwd = 2 * macs + tri * lookups_fwd
    dx = 2 * macs + 2 * tri * lookups_grad
    dw = 2 * macs
    lookup_b = 8 * C_DIM * 4
    if mode == "forward":
        fl, by = fwd, lookup_b * lookups_fwd
    elif mode == "tracker":
        fl, by = fwd + dx, lookup_b * (lookups_fwd + lookups_grad)
    else:
        fl = fwd + dx + dw
        by = lookup_b * (lookups_fwd + lookups_grad + 2 * lookups_grad)
    return fl * S, by * S


__all__ = [n for n in dir() if not n.startswith("_")]
