"""Conv micro-benchmark: fwd / dgrad / wgrad of the model_fbanks_cnn layers (B = 512) and the
model_resnet_bgru stage convs (B = 512), timed with srk_prof events (algorithmic flops / time)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speechrecognitionproject_amd import _lib, nn as snn  # noqa: E402

SHAPES = {  # name: N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw
    "fb_conv1": (512, 98, 120, 1, 64, 7, 3, 3, 1, 1, 1),
    "fb_conv2": (512, 98, 40, 64, 128, 1, 7, 0, 3, 1, 1),
    "fb_conv3": (512, 98, 10, 128, 256, 1, 10, 0, 0, 1, 1),
    "fb_conv4": (512, 98, 1, 256, 512, 7, 1, 3, 0, 1, 1),
    "rn_stem": (512, 1, 16000, 1, 64, 1, 80, 0, 38, 1, 16),
    "rn_l1": (512, 1, 1000, 64, 64, 1, 15, 0, 7, 1, 1),
    "rn_l2": (512, 1, 500, 128, 128, 1, 15, 0, 7, 1, 1),
    "rn_l4": (512, 1, 125, 512, 512, 1, 15, 0, 7, 1, 1),
}
res = {}
for name, (N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw) in SHAPES.items():
    x = torch.randn(N, H, W, Ci, device="cuda", requires_grad=Ci > 1)
    w = (torch.randn(Co, Ci, KH, KW, device="cuda") * 0.05).requires_grad_(True)
    b = torch.zeros(Co, device="cuda", requires_grad=True)
    for it in range(3):
        if it == 2:
            _lib.prof_enable(True)
        y = snn._Conv2dNHWCFn.apply(x, w, b, (ph, pw), (sh, sw))
        y.backward(torch.ones_like(y))
    r = {}
    for k in ("conv_fwd", "conv_dgrad", "conv_wgrad"):
        c, ms, fl = _lib.prof_read(k)
        if c:
            r[k] = {"us": round(ms / c * 1e3, 1), "TF": round(fl / (ms * 1e-3) / 1e12, 1)}
    _lib.prof_enable(False)
    res[name] = r
    print(name, json.dumps(r), flush=True)
