"""Which rounding does torch.optim.Adam(fused=True) use on this device?  Emulates
candidate formulas with elementwise torch ops and reports the fraction of exact
matches for exp_avg and param (diagnostic)."""
import math

import torch

g = torch.Generator().manual_seed(0)
n = 1 << 16
p0 = torch.randn(n, generator=g).cuda()
grads = [(torch.randn(n, generator=g) * 1e-2).cuda() for _ in range(4)]
ref = torch.nn.Parameter(p0.clone())
b1, b2, lr, eps = 0.9, 0.999, 1e-2, 1e-8
opt = torch.optim.Adam([ref], lr=lr, fused=True)
for gr in grads[:3]:
    ref.grad = gr
    opt.step()
st = opt.state[ref]
p, m, v = ref.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone()
gr = grads[3]
ref.grad = gr
opt.step()
M, V, P = st["exp_avg"], st["exp_avg_sq"], ref.detach()
f = lambda x: torch.tensor(x, dtype=torch.float32).item()
d = torch.float64
cands = {
    "double": (b1 * m.to(d) + (1 - b1) * gr.to(d)).float(),
    "float": (f(b1) * m + f(1 - b1) * gr),
    "float_b1m_first": (m * f(b1)) + (gr * f(1 - b1)),
    "lerp": m + f(1 - b1) * (gr - m),
    "lerp_torch": torch.lerp(m, gr, 1 - b1),
}
for k, c in cands.items():
    print("m", k, float((c == M).float().mean()))
vc = {"double": (b2 * v.to(d) + (1 - b2) * gr.to(d) * gr.to(d)).float(),
      "float": f(b2) * v + f(1 - b2) * gr * gr}
for k, c in vc.items():
    print("v", k, float((c == V).float().mean()))
bc1 = 1 - b1 ** 4
bc2s = math.sqrt(1 - b2 ** 4)
pc = {
    "f_bc": p - (f(lr / f(bc1)) * M) / ((M.new_tensor(0) + (V.sqrt() / f(bc2s)).to(d) + eps).float()),
    "d_bc": p - (f(lr / bc1) * M) / (((V.sqrt().to(d) / bc2s) + eps).float()),
    "all_float": p - (f(lr / f(bc1)) * M) / (V.sqrt() / f(bc2s) + f(eps)),
    "foreach_like": p + f(-lr / bc1) * (M / (V.sqrt() / f(bc2s) + f(eps))),
    "mul_first": p - f(lr / f(bc1)) * (M / ((V.sqrt() / f(bc2s)).to(d) + eps).float()),
}
for k, c in pc.items():
    print("p", k, float((c == P).float().mean()))

from fractions import Fraction as Fr  # noqa: E402
c = cands["double"]
bad = (c != M).nonzero().flatten()[:6].tolist()
for i in bad:
    mo, gi = float(m[i]), float(gr[i])
    exact = Fr(b1) * Fr(mo) + Fr(1 - b1) * Fr(gi)
    fma_d = float(Fr(b1) * Fr(mo) + Fr(float(Fr(1 - b1) * Fr(gi))))  # fma(b1, m, (1-b1)*g)
    fma_d2 = float(Fr(1 - b1) * Fr(gi) + Fr(float(Fr(b1) * Fr(mo))))  # fma(1-b1, g, b1*m)
    print(i, mo.hex(), gi.hex(), "torch", float(M[i]).hex(), "double", float(c[i]).hex(),
          "exact->f32", torch.tensor(float(exact)).float().item().hex(),
          "fma1", torch.tensor(fma_d).float().item().hex(), "fma2", torch.tensor(fma_d2).float().item().hex())
