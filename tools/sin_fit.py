"""Fit and check the Fourier-feature sin / cos of nc_device.h (fourier_sin, fourier_cos,
fourier_sin2) -- CPU only.

Fits sin t = t + t^3 P(t^2) (4 coefficients) and cos t = 1 + t^2 Q(t^2) (5) near-minimax
on [-pi/2, pi/2] by iteratively reweighted least squares on Chebyshev nodes, then emulates
the kernel's float32 evaluation (magic-number round of x / pi, three-part Cody-Waite pi,
Horner in fma, the (-1)^k sign) on arguments like the Fourier features' (|x| up to ~1e3)
and prints the max / mean absolute error against float64, beside a float32 libm sin / cos.

    python tools/sin_fit.py
"""
import numpy as np

f32 = np.float32


def fma(a, b, c):
    # float32 fma: the product of two float32s is exact in float64, one rounding of the sum
    # (a double rounding through float64 is possible in principle; not at these magnitudes)
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


def fit(powers, target):
    n = 4000
    t = (np.cos(np.linspace(0, np.pi, n)) + 1) / 2 * (np.pi / 2)
    t = t[t > 1e-6]
    A = np.stack([t ** p for p in powers], 1)
    b = target(t)
    w = np.ones_like(t)
    for _ in range(60):  # reweight toward the equi-oscillating (minimax) solution
        c, *_ = np.linalg.lstsq(A * w[:, None], b * w, rcond=None)
        e = np.abs(A @ c - b)
        w = w * (1 + 5 * e / e.max())
        w /= w.mean()
    return [f32(v) for v in c], float(e.max())


PI1 = f32(3.140625)
PI2 = f32(np.pi - 3.140625)
PI3 = f32(np.pi - 3.140625 - np.float64(PI2))
MAGIC = f32(12582912.0)


def reduce_pi(x):
    y = fma(x, f32(1 / np.pi), MAGIC)
    k = (y - MAGIC).astype(np.float32)
    t = fma(-k, PI1, x)
    t = fma(-k, PI2, t)
    t = fma(-k, PI3, t)
    return t, (y.view(np.int32) & 1).astype(bool)


def horner(t2, cs):
    p = cs[-1]
    for v in reversed(cs[:-1]):
        p = fma(t2, p, v)
    return p


def emulate_sin(cs, x):
    t, odd = reduce_pi(x)
    t2 = (t * t).astype(np.float32)
    s = fma((t2 * t).astype(np.float32), horner(t2, cs), t)
    return np.where(odd, -s, s)


def emulate_cos(cs, x):
    t, odd = reduce_pi(x)
    t2 = (t * t).astype(np.float32)
    c = fma(t2, horner(t2, cs), f32(1.0))
    return np.where(odd, -c, c)


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    x = np.concatenate([(rng.standard_normal(2000000) * 400).astype(np.float32),
                        rng.uniform(-4, 4, 500000).astype(np.float32)])
    x64 = x.astype(np.float64)
    cs, es = fit([3, 5, 7, 9], lambda t: np.sin(t) - t)
    cc, ec = fit([2, 4, 6, 8, 10], lambda t: np.cos(t) - 1)
    print("pi parts", repr(PI1), repr(PI2), repr(PI3), " max |k|", int(np.abs(np.rint(x64 / np.pi)).max()))
    for name, coef, em, emu, ref in (("sin", cs, es, emulate_sin, np.sin), ("cos", cc, ec, emulate_cos, np.cos)):
        e = np.abs(emu(coef, x) - ref(x64))
        e32 = np.abs(ref(x).astype(np.float64) - ref(x64))
        print(f"{name}: coefficients {[repr(v) for v in coef]}  approximation error {em:.2e}")
        print(f"   float32 evaluation: max {e.max():.3e} mean {e.mean():.3e}   "
              f"(float32 libm: max {e32.max():.3e} mean {e32.mean():.3e})")
