"""The Fourier-feature sin / cos of the HIP kernels (nc_device.h fourier_sin / fourier_cos /
fourier_sin2), emulated in float32 on the CPU with the constants read from the header:
the error against float64 stays at the level of a float32 libm (decoder.py:26-30 computes
torch.sin of the float32 argument), far below the former hardware v_sin_f32 form's 3.8e-7
-- the error that failed the fine_depth golden case's per-element gate."""
import os
import re
import sys

import numpy as np

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
import sin_fit as SF  # noqa: E402


def _header_constants():
    with open(os.path.join(REPO, "nice-slam-annotation_amd", "csrc", "nc_device.h")) as f:
        s = f.read()
    vals = dict(re.findall(r"\b(k[A-Z][A-Za-z0-9]*) = ([-0-9.e]+)f", s))
    return {k: np.float32(float(v)) for k, v in vals.items()}


def test_header_constants_match_the_fit_and_pi_split():
    c = _header_constants()
    assert c["kPi1"] == SF.PI1 and c["kPi2"] == SF.PI2 and c["kPi3"] == SF.PI3
    assert float(c["kPi1"]) + float(c["kPi2"]) + float(c["kPi3"]) == np.float64(np.pi).item() or \
        abs(float(c["kPi1"]) + float(c["kPi2"]) + float(c["kPi3"]) - np.pi) < 1e-18
    assert c["kRoundMagic"] == np.float32(1.5 * 2 ** 23)
    # pi1 has 8 significant bits: k * pi1 is exact for |k| < 2^16
    m = float(c["kPi1"]) * 2 ** 6
    assert m == int(m) and int(m) < 2 ** 8


def test_sin_cos_emulation_accuracy():
    c = _header_constants()
    rng = np.random.default_rng(7)
    x = np.concatenate([(rng.standard_normal(400000) * 400).astype(np.float32),
                        rng.uniform(-4, 4, 100000).astype(np.float32),
                        np.float32([0.0, -0.0, np.pi / 2, -np.pi / 2, np.pi, 1e-6, 3000.0])])
    x64 = x.astype(np.float64)
    s = SF.emulate_sin([c["kS1"], c["kS2"], c["kS3"], c["kS4"]], x)
    co = SF.emulate_cos([c["kC1"], c["kC2"], c["kC3"], c["kC4"], c["kC5"]], x)
    es, ec = np.abs(s - np.sin(x64)), np.abs(co - np.cos(x64))
    assert es.max() < 1.3e-7 and es.mean() < 2.0e-8, (es.max(), es.mean())
    assert ec.max() < 1.5e-7 and ec.mean() < 2.5e-8, (ec.max(), ec.mean())
    assert s[-7] == 0.0 and s[-6] == 0.0  # sin(+-0) = 0 (the sign of a zero feature multiplies into nothing)
