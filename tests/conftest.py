"""Shared pytest setup: markers, import paths and golden-fixture loading."""
import json
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "nice-slam-annotation_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) to run")


def gpu_available():
    return torch.cuda.is_available()


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def load_meta():
    with open(os.path.join(GOLDEN, "golden_meta.json")) as f:
        return json.load(f)


def load_scene(which="tiny"):
    """The golden scene: "tiny" (make_golden.py, scaled grids) or "initstd"
    (make_golden_initstd.py, the reference's grid_init statistics)."""
    z = np.load(os.path.join(GOLDEN, f"scene_{which}.npz"))
    bound = torch.from_numpy(z["bound"])
    grids = {k: torch.from_numpy(z[k]) for k in z.files if k.startswith("grid_")}
    params = {k[len("param/"):]: torch.from_numpy(z[k]) for k in z.files if k.startswith("param/")}
    return bound, torch.from_numpy(z["coarse_bound"]), grids, params


def load_case(name):
    z = np.load(os.path.join(GOLDEN, f"case_{name}.npz"))
    return {k: torch.from_numpy(z[k]) for k in z.files}


CASE_NAMES = [c["name"] for c in load_meta()["cases"]]


def load_initstd_meta():
    with open(os.path.join(GOLDEN, "initstd_meta.json")) as f:
        return json.load(f)


INITSTD_CASES = [c["name"] for c in load_initstd_meta()["cases"]]
