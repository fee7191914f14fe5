"""Rank worker of tests/test_gpu_defer.py::test_split_allreduce_two_gloo_ranks: the
bench.py N > 1 exchange with the split backward (grid all-reduce issued before the
deferred weight gradients, decoder all-reduce after) on its half of a batch; saves the
reduced gradients."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "nice-slam-annotation_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out):
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    from test_gpu_defer import _body, _leaves, _setup
    from nicecore import distributed as ND
    from nicecore.render_fn import DeferParamGrads
    sc, g, model, ro, rd, gt, gtc, r = _setup()
    sl = slice(150 * rank, 150 * (rank + 1))
    ro_s, rd_s = ro[sl].detach().clone().requires_grad_(True), rd[sl].detach().clone().requires_grad_(True)
    dmax = gt.max().reshape(1)
    defer = DeferParamGrads()
    for t in _leaves(g, model, ro_s, rd_s):
        t.grad = None
    d, u, c, L = r.render_batch_loss(g, model, rd_s, ro_s, "cuda", "color", gt[sl], gtc[sl], loss="mapper",
                                     color_term=True, depth_max=dmax, defer_param_grads=defer)
    L.backward()
    finish = ND.allreduce_grads_async(list(g.values()))
    defer.run()
    finish()
    ND.allreduce_grads(list(model.parameters()))
    torch.cuda.synchronize()
    res = {k: v.grad.cpu() for k, v in g.items() if v.grad is not None}
    res.update({"param/" + n: p.grad.cpu() for n, p in model.named_parameters() if p.grad is not None})
    torch.save(res, os.path.join(out, f"defer_rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
