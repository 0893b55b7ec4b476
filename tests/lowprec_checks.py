"""Checks shared by the 16-bit train-step tests at the config shapes (tests/test_trainstep_lowprec_gpu.py,
tests/test_config_batch_gpu.py); the bounds are tests/tolerances.py's LP_* constants."""
import numpy as np
import torch

from tolerances import LP_ADAM_ABS, LP_GRAD_REL, LP_UPDATE_WEIGHTED


def torch_adam_first_step(p0, g, lr):
    """torch.optim.Adam's first step (betas 0.9 / 0.999, eps 1e-8) in its operation order (fp32)."""
    m = (1 - 0.9) * g
    v = (1 - 0.999) * g * g
    denom = v.sqrt() / np.sqrt(1 - 0.999) + 1e-8
    return p0 - (lr / (1 - 0.9)) * (m / denom)


def normwise(g, ref):
    """||g - ref||_2 / ||ref||_2 in float64 (None when ref is exactly zero)."""
    g, ref = g.double(), ref.double()
    n = ref.norm().item()
    return None if n == 0.0 else ((g - ref).norm() / n).item()


def check_grads(grads, want, bound=None):
    """Every gradient tensor norm-wise within bound(name) (default LP_GRAD_REL) of want[name];
    exactly-zero reference gradients must be exactly zero.  Returns {name: error}."""
    worst = {}
    for n, g in grads.items():
        e = normwise(g, want[n])
        if e is None:
            assert g.abs().max().item() == 0.0, n
            worst[n] = 0.0
            continue
        worst[n] = e
    bad = {n: e for n, e in worst.items() if not e <= (bound(n) if bound else LP_GRAD_REL)}
    assert not bad, (bad, worst)
    return worst


def check_adam(named_params_after, p0, grads, p0_ref, g_ref, lr, update_bound=None):
    """(a) the fused Adam kernel == torch's first-step formula on the HIP path's own (unscaled)
    gradient, <= LP_ADAM_ABS; (b) the update moves like the fp32 oracle's Adam step on the oracle
    gradient: disagreement weighted by |g_oracle| <= LP_UPDATE_WEIGHTED."""
    for n, p in named_params_after:
        p1 = p.detach().cpu()
        assert torch.equal(p0[n], p0_ref[n]), n
        assert (p1 - torch_adam_first_step(p0[n], grads[n], lr)).abs().max().item() <= LP_ADAM_ABS, n
        d_gpu = (p1 - p0[n]).double()
        d_ref = (torch_adam_first_step(p0_ref[n], g_ref[n], lr) - p0_ref[n]).double()
        w = g_ref[n].double().abs()
        if w.sum().item() == 0.0:
            assert torch.equal(d_gpu, d_ref), n
            continue
        dis = ((w * (d_gpu - d_ref).abs()).sum() / (w * d_ref.abs()).sum()).item()
        assert dis <= (update_bound(n) if update_bound else LP_UPDATE_WEIGHTED), (n, dis)
