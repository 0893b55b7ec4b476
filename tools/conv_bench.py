"""Conv micro-benchmark: fwd / dgrad / wgrad of the model_fbanks_cnn layers (B = 512) and the
model_resnet_bgru stage convs (B = 512), timed with srk_prof events (algorithmic flops / time).

    python tools/conv_bench.py [--prec bf16] [--only fb_conv2,rn_l1] [--var "" --var "conv_ring_qs=0" ...]

Each --var is a comma-separated srk option list applied with srk_set_option before the shape runs; options
stay set afterwards, so give every variant the full list it compares (e.g. "conv_ring_qs=6" / "conv_ring_qs=0"); fb_conv2 runs as the fused conv + (1, 4) max pool model_fbanks_cnn uses."""
import argparse
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
MEAS = 5   # measured passes (per-pass means)
CATS = ("conv_fwd", "conv_dgrad", "conv_wgrad", "conv_fwd_lp", "conv_dgrad_lp", "conv_wgrad_lp", "conv_to16",
        "conv_colsum")


def parse_opts(s):
    out = []
    for kv in filter(None, (t.strip() for t in s.split(","))):
        k, v = kv.split("=")
        out.append((k, int(v)))
    return out


def run_shape(name, prec, opts):
    N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw = SHAPES[name]
    x = torch.randn(N, H, W, Ci, device="cuda", requires_grad=Ci > 1)
    w = (torch.randn(Co, Ci, KH, KW, device="cuda") * 0.05).requires_grad_(True)
    b = torch.zeros(Co, device="cuda", requires_grad=True)
    pooled = name == "fb_conv2"
    _lib.set_matmul_precision(prec)
    for k, v in opts:
        _lib.set_option(k, v)
    try:
        r = {}
        for it in range(3 + MEAS):
            if it == 3:
                _lib.prof_enable(True)
            if pooled:
                y = snn._ConvPoolNHWCFn.apply(x, w, b, (ph, pw), 4)
            else:
                y = snn._Conv2dNHWCFn.apply(x, w, b, (ph, pw), (sh, sw))
            y.backward(torch.ones_like(y))
        torch.cuda.synchronize()
        for k in CATS:
            c, ms, work = _lib.prof_read(k)
            if c:
                unit = "GB/s" if k in ("conv_to16", "conv_colsum") else "TF"
                r[k] = {"us": round(ms * 1e3 / MEAS, 1), unit: round(work / (ms * 1e-3) / (1e9 if unit == "GB/s" else 1e12), 1)}
        r["kernels"] = [{"kernel": e["kernel"], "us": round(e["ms_total"] * 1e3 / MEAS, 1)} for e in _lib.prof_kernels()]
        _lib.prof_enable(False)
        return r
    finally:
        _lib.set_matmul_precision("fp32")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="fp32")
    ap.add_argument("--only", default="")
    ap.add_argument("--var", action="append", default=None)
    a = ap.parse_args()
    names = [n for n in SHAPES if not a.only or n in a.only.split(",")]
    for var in a.var or [""]:
        for name in names:
            r = run_shape(name, a.prec, parse_opts(var))
            print(json.dumps({"shape": name, "prec": a.prec, "opts": var, **r}), flush=True)


if __name__ == "__main__":
    main()
