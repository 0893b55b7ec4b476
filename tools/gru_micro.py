"""Micro-benchmark of the GRU recurrence step kernels (per-launch time vs batch)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from speechrecognitionproject_amd import _lib
from speechrecognitionproject_amd.nn import _GRULayerFn

H, T, IN = 512, 51, 1024
res = {}
for B in [64, 128, 256, 512, 1024]:
    x = torch.randn(B, T, IN, device="cuda", requires_grad=True)
    w_ih = torch.randn(2, 3 * H, IN, device="cuda") * 0.03
    w_hh = (torch.randn(2, 3 * H, H, device="cuda") * 0.04).requires_grad_(True)
    b = torch.zeros(2, 3 * H, device="cuda")
    for it in range(3):
        y = _GRULayerFn.apply(x, w_ih, w_hh, b, b)
        y.sum().backward()
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    for it in range(3):
        y = _GRULayerFn.apply(x, w_ih, w_hh, b, b)
        y.sum().backward()
    torch.cuda.synchronize()
    r = {}
    for k in ("gru_fwd_step", "gru_bwd_step", "gemm_f32"):
        c, ms, w = _lib.prof_read(k)
        r[k] = {"us_per_launch": round(ms / c * 1e3, 2), "tflops": round(w / (ms * 1e-3) / 1e12, 1)}
    _lib.prof_enable(False)
    res[B] = r
    print(B, json.dumps(r), flush=True)
