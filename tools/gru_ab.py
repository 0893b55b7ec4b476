"""A/B timing of the persistent GRU recurrence variants (srk options) on the cfg2 shapes.

    python tools/gru_ab.py [--B 256] [--T 51] [--reps 10]

For each variant: one BiGRU layer (H = 512) fwd + bwd, layer-0 (IN = 39, fused projection) and
layer-1 (IN = 1024) shapes; prints the per-launch time of the recurrence kernels (gru_fwd_seq /
gru_bwd_seq, HIP events) and us per step.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speechrecognitionproject_amd import _lib  # noqa: E402
from speechrecognitionproject_amd import nn as snn  # noqa: E402

DEFAULTS = {"gru_fp32_dual_chain": 1, "gru_dc_offset_ns": 2000, "gru_fp32_fast_cell": 1, "gru_dc_prio": 0}
VARIANTS = {"dc": {"gru_fp32_dual_chain": 1, "gru_dc_offset_ns": 0, "gru_fp32_fast_cell": 0},
            "dc_off2us": {"gru_dc_offset_ns": 2000}, "dc_off4us": {"gru_dc_offset_ns": 4000},
            "dc_fast": {"gru_dc_offset_ns": 0, "gru_fp32_fast_cell": 1},
            "4wave": {"gru_fp32_dual_chain": 0, "gru_fp32_fast_cell": 0},
            # round 4: static priority of one chain (defaults otherwise)
            "default": {}, "prio_c0": {"gru_dc_prio": 1}, "prio_c1": {"gru_dc_prio": 2},
            "prio_c0_off0": {"gru_dc_prio": 1, "gru_dc_offset_ns": 0},
            "prio_c1_off0": {"gru_dc_prio": 2, "gru_dc_offset_ns": 0}}


def run(B, T, IN, reps, opts):
    for k, v in opts.items():
        _lib.set_option(k, v)
    torch.manual_seed(0)
    m = snn.BiGRU(IN, 512, num_layers=1).cuda()
    x = torch.randn(B, T, IN, device="cuda", requires_grad=True)
    for _ in range(2):
        y, _ = m(x)
        y.sum().backward()
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    for _ in range(reps):
        y, _ = m(x)
        y.sum().backward()
    torch.cuda.synchronize()
    r = {}
    for k in ("gru_fwd_seq", "gru_bwd_seq"):
        c, ms, w = _lib.prof_read(k)
        if c:
            r[k] = {"us_per_launch": round(ms / c * 1e3, 1), "us_per_step": round(ms / c * 1e3 / T, 2),
                    "tflops": round(w / (ms * 1e-3) / 1e12, 1)}
    _lib.prof_enable(False)
    assert _lib.spin_timeouts() == 0
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--T", type=int, default=51)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default=",".join(VARIANTS), help="comma-separated names (each on top of the defaults)")
    a = ap.parse_args()
    for name in a.variants.split(","):
        for IN in (39, 1024):
            print(name, "IN=%d" % IN, json.dumps(run(a.B, a.T, IN, a.reps, dict(DEFAULTS, **VARIANTS[name]))), flush=True)
    for k, v in DEFAULTS.items():
        _lib.set_option(k, v)


if __name__ == "__main__":
    main()
