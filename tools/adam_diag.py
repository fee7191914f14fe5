"""Per-tensor ulp distance of nicecore's Adam step vs torch.optim.Adam(fused=True) from
one identical state (diagnostic for k_adam_dense's rounding; NICECORE_LIB picks the build)."""
import sys

import torch

sys.path.insert(0, "nice-slam-annotation_amd")
sys.path.insert(0, "tests")
from nicecore.optim import adam_step_  # noqa: E402
from test_gpu_adam import _ulps  # noqa: E402

for wd in (0.0, 1e-2):
    g = torch.Generator().manual_seed(0)
    n = 1 << 16
    p0 = torch.randn(n, generator=g).cuda()
    grads = [(torch.randn(n, generator=g) * 1e-2).cuda() for _ in range(4)]
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.Adam([ref], lr=1e-2, weight_decay=wd, fused=True)
    for gr in grads[:3]:
        ref.grad = gr
        opt.step()
    st = opt.state[ref]
    p, m, v = ref.detach().clone(), st["exp_avg"].clone(), st["exp_avg_sq"].clone()
    ref.grad = grads[3]
    opt.step()
    adam_step_(p, grads[3], m, v, lr=1e-2, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=wd, step=4)
    torch.cuda.synchronize()
    print(f"wd={wd}: p {_ulps(p, ref)} m {_ulps(m, st['exp_avg'])} v {_ulps(v, st['exp_avg_sq'])} "
          f"p-exact {float((p == ref).float().mean()):.4f} m-exact {float((m == st['exp_avg']).float().mean()):.4f} "
          f"v-exact {float((v == st['exp_avg_sq']).float().mean()):.4f}")
