"""Is the cfg4-bf16 gradient error inherent?  The resnet_bgru oracle step (oracle/models.py) with every Conv1d's
operands rounded to bf16 — x and w in the forward, x, w and dY in the backward — fp32 accumulation (the HIP
16-bit conv contract), vs float64; the fp32 oracle beside it.  CPU only.  Prints norm-wise errors per tensor.

    python tools/bf16_emul_resnet.py [B] [--json tests/golden/cfg4_bf16_emul_nw.json]

With --json (B = 512, the cfg4 rank-shard case of tests/test_config_batch_gpu.py: synthetic_clips(512, seed=45),
the seeded state_dict) the per-tensor norm-wise errors are written as the fixture that test reads."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import models as OM  # noqa: E402
from speechrecognitionproject_amd.synthetic import synthetic_clips  # noqa: E402


def r16(t):
    return t.to(torch.bfloat16).to(t.dtype)


class Conv1dBF16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, padding):
        xr, wr = r16(x), r16(w)
        ctx.save_for_backward(xr, wr)
        ctx.geom = (stride, padding)
        return F.conv1d(xr, wr, None, stride, padding)

    @staticmethod
    def backward(ctx, gy):
        xr, wr = ctx.saved_tensors
        stride, padding = ctx.geom
        g = r16(gy)
        gx = torch.nn.grad.conv1d_input(xr.shape, wr, g, stride, padding)
        gw = torch.nn.grad.conv1d_weight(xr, wr.shape, g, stride, padding)
        return gx, gw, None, None


def patch_convs(net):
    for m in net.modules():
        if isinstance(m, torch.nn.Conv1d) and m.in_channels % 8 == 0:   # the 16-bit path needs 8-aligned channels
            def fwd(x, m=m):
                return Conv1dBF16.apply(x, m.weight, m.stride[0], m.padding[0])
            m.forward = fwd


def step(net, x, y, dtype):
    net = net.to(dtype).train()
    out = net.gru(net.resnet(torch.from_numpy(x).to(dtype).unsqueeze(1)))
    torch.nn.CrossEntropyLoss()(out, torch.from_numpy(y)).backward()
    return {n: p.grad.double().clone() for n, p in net.named_parameters() if p.grad is not None}


args = [a for a in sys.argv[1:] if not a.startswith("--")]
B = int(args[0]) if args else 64
out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
x, y = synthetic_clips(B, seed=45)
sd = OM.seeded_state_dict(OM.ResnetBGRU(), 0)
res = {}
for name, dtype, emul in (("f64", torch.float64, False), ("fp32", torch.float32, False), ("bf16conv", torch.float32, True)):
    net = OM.ResnetBGRU()
    net.load_state_dict(sd)
    if emul:
        patch_convs(net)
    res[name] = step(net, x, y, dtype)
# the first Adam step (lr 1e-4) on the emulated gradient vs on the fp32 oracle's, disagreement weighted by
# |g_fp32| (tests/lowprec_checks.py check_adam (b))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from lowprec_checks import torch_adam_first_step  # noqa: E402
p0 = {n: v.float() for n, v in sd.items()}
adam_dis = {}
for n, g32 in res["fp32"].items():
    w = g32.abs()
    if w.sum().item() == 0.0 or n not in p0:
        continue
    d_e = (torch_adam_first_step(p0[n], res["bf16conv"][n].float(), 1e-4) - p0[n]).double()
    d_r = (torch_adam_first_step(p0[n], g32.float(), 1e-4) - p0[n]).double()
    adam_dis[n] = round(((w * (d_e - d_r).abs()).sum() / (w * d_r.abs()).sum()).item(), 5)
rows = []
for n, g64 in res["f64"].items():
    nn64 = g64.norm().item()
    if nn64 == 0:
        continue
    rows.append((n, round((res["fp32"][n] - g64).norm().item() / nn64, 5), round((res["bf16conv"][n] - g64).norm().item() / nn64, 4)))
for r in rows:
    if "resnet" in r[0]:
        print(json.dumps(r))
if out_json:
    with open(out_json, "w") as f:
        json.dump({"B": B, "seed": 45, "what": "norm-wise error vs float64 of the resnet_bgru oracle step with bf16-rounded "
                   "Conv1d operands (tools/bf16_emul_resnet.py)", "bf16conv_nw": {r[0]: r[2] for r in rows},
                   "fp32_nw": {r[0]: r[1] for r in rows}, "bf16conv_adam_dis": adam_dis}, f, indent=1,
                  sort_keys=True)
print("B", B, "worst fp32", max(r[1] for r in rows), "worst bf16conv", max(r[2] for r in rows))
