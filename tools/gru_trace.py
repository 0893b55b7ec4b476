"""Per-step timeline of the persistent GRU kernels (srk_set_option("gru_trace_ptr")).

Runs one BiGRU(39 -> 512, 1 layer) fwd + bwd at B = 256, T = 51 with tracing on and prints, per
kernel, the mean over workgroups and steps of: wait (step start -> arrival wait done), loads_mfma
(-> the MFMAs retired: h / dg loads + matrix work), epilogue (-> cell math + LDS transpose done),
publish (-> arrival), in microseconds.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speechrecognitionproject_amd import _lib  # noqa: E402
from speechrecognitionproject_amd import nn as snn  # noqa: E402

B, T, IN, H = int(os.environ.get("B", 256)), 51, int(os.environ.get("IN", 1024)), 512
nwg = 256
_lib.set_matmul_precision(os.environ.get("PREC", "fp32"))
_lib.set_option("gru_fp32_dual_chain", int(os.environ.get("DC", 1)))   # bf16 / fp16: the 16-bit recurrence kernels
res = {}
m = snn.BiGRU(IN, H, 1).cuda()
x = torch.randn(B, T, IN, device="cuda", requires_grad=True)
for it in range(3):
    buf = torch.zeros(nwg * T * 8, dtype=torch.int64, device="cuda")
    _lib.set_option("gru_trace_ptr", buf.data_ptr() if it == 2 else 0)
    y, _ = m(x)
    torch.cuda.synchronize()
    fwd = buf.clone()
    buf.zero_()
    y.backward(torch.randn_like(y))
    torch.cuda.synchronize()
    bwd = buf.clone()
_lib.set_option("gru_trace_ptr", 0)
for name, b in (("fwd", fwd), ("bwd", bwd)):
    ts = b.view(nwg, T, 8).double().cpu() * 0.01   # 100 MHz ticks -> us
    wait = (ts[:, 1:, 1] - ts[:, 1:, 0]).mean().item()
    mfma = (ts[:, 1:, 2] - ts[:, 1:, 1]).mean().item()
    epi = (ts[:, 1:, 3] - ts[:, 1:, 2]).mean().item()
    pub = (ts[:, 1:, 4] - ts[:, 1:, 3]).mean().item()
    step = ((ts[:, -1, 4] - ts[:, 0, 0]) / T).mean().item()
    prologue = (ts[:, 0, 0] - ts[:, 0, 6]).mean().item() if bool((ts[:, 0, 6] > 0).all()) else float("nan")
    span = (ts[:, -1, 4].max() - ts[:, 0, 6].min()).item() if bool((ts[:, 0, 6] > 0).all()) else float("nan")
    start_skew = (ts[:, 0, 0].max() - ts[:, 0, 0].min()).item()
    # group membership: the (direction, group) pair each workgroup ran, recorded by the kernel (trace_id)
    grp = (b.view(nwg, T, 8)[:, 0, 5].cpu() >> 8)
    npairs = int(grp.max().item()) + 1
    spread, prop = [], []
    for g in range(npairs):
        m = grp == g
        pubs = ts[m][:, :, 4]                              # [slices, T] publish stamps
        spread.append((pubs.max(0).values - pubs.min(0).values)[:-1])
        # wait done at step s + 1 minus the group's LAST publish of step s: flag propagation
        prop.append(ts[m][:, 1:, 1] - pubs.max(0).values[None, :-1])
    spread, prop = torch.cat(spread), torch.cat(prop)
    # two-chain kernels: chain 1's wait end (slot 7) relative to chain 0's, as a fraction of the step
    c1 = ts[:, 1:, 7]
    chain_offset = float("nan")
    if bool((c1 > 0).all()):
        d = (c1 - ts[:, 1:, 1])
        chain_offset = round((d.remainder(step) / step).mean().item(), 3)
    res[name] = {"chain1_offset_frac": chain_offset, "us_per_step": round(step, 2), "prologue_us": round(prologue, 2), "entry_to_last_publish_us": round(span, 2), "wait": round(wait, 2), "loads_mfma": round(mfma, 2),
                 "epilogue": round(epi, 2), "publish": round(pub, 2), "launch_skew_us": round(start_skew, 2),
                 "publish_spread_us": round(spread.mean().item(), 2),
                 "last_publish_to_wait_done_us": round(prop.mean().item(), 2)}
print(json.dumps(res))
