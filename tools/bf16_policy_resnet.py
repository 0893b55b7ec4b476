"""Which conv passes must keep fp32 operands for a faithful resnet_bgru bf16 training step?  (VERDICT r05
"missing" #1.)  The resnet_bgru oracle step (oracle/models.py) with each Conv1d pass given bf16-rounded or
fp32 operands by a POLICY — forward (x, w), data gradient (dY, w), weight gradient (x, dY) — fp32
accumulation (the HIP 16-bit conv contract), against float64.  CPU only.  Prints the worst norm-wise
error over the ResNet's parameter gradients per policy (bf16 everywhere = tools/bf16_emul_resnet.py).

    python tools/bf16_policy_resnet.py [B] [policy ...]      policy = three letters f/b for fwd, dgrad, wgrad
                                                              (default: bbb bbf bfb bff fbb fff); a policy may
                                                              end in @prefix1+prefix2: only the convs whose
                                                              module name starts with one of them take it, the
                                                              others stay bbb (e.g. fbb@conv1+layer1)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import models as OM  # noqa: E402
from speechrecognitionproject_amd.synthetic import synthetic_clips  # noqa: E402


def r16(t, on):
    return t.to(torch.bfloat16).to(t.dtype) if on else t


class Conv1dPolicy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, padding, pol):
        ctx.save_for_backward(x, w)
        ctx.geom = (stride, padding, pol)
        return F.conv1d(r16(x, pol[0]), r16(w, pol[0]), None, stride, padding)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, padding, pol = ctx.geom
        gx = torch.nn.grad.conv1d_input(x.shape, r16(w, pol[1]), r16(gy, pol[1]), stride, padding)
        gw = torch.nn.grad.conv1d_weight(r16(x, pol[2]), w.shape, r16(gy, pol[2]), stride, padding)
        return gx, gw, None, None, None


def patch_convs(net, pol, prefixes=None):
    for name, m in net.resnet.named_modules():
        if isinstance(m, torch.nn.Conv1d) and m.in_channels % 8 == 0:   # the 16-bit path needs 8-aligned channels
            p = pol if prefixes is None or any(name.startswith(q) for q in prefixes) else (True, True, True)

            def fwd(x, m=m, p=p):
                return Conv1dPolicy.apply(x, m.weight, m.stride[0], m.padding[0], p)
            m.forward = fwd


def step(net, x, y, dtype):
    net = net.to(dtype).train()
    out = net.gru(net.resnet(torch.from_numpy(x).to(dtype).unsqueeze(1)))
    torch.nn.CrossEntropyLoss()(out, torch.from_numpy(y)).backward()
    return {n: p.grad.double().clone() for n, p in net.named_parameters() if p.grad is not None}


def main():
    args = [a for a in sys.argv[1:]]
    B = int(args[0]) if args and args[0].isdigit() else 128
    pols = [a for a in args if not a.isdigit()] or ["bbb", "bbf", "bfb", "bff", "fbb", "fff"]
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    x, y = synthetic_clips(B, seed=45)
    sd = OM.seeded_state_dict(OM.ResnetBGRU(), 0)
    net = OM.ResnetBGRU()
    net.load_state_dict(sd)
    ref = step(net, x, y, torch.float64)
    for p in pols:
        spec, _, pre = p.partition("@")
        pol = tuple(c == "b" for c in spec)
        net = OM.ResnetBGRU()
        net.load_state_dict(sd)
        patch_convs(net, pol, pre.split("+") if pre else None)
        g = step(net, x, y, torch.float32)
        errs = {n: (g[n] - r).norm().item() / r.norm().item() for n, r in ref.items()
                if "resnet" in n and r.norm().item() > 0}
        worst = sorted(errs.items(), key=lambda kv: -kv[1])[:4]
        print("B %d policy %s (fwd/dgrad/wgrad, b = bf16): worst %.4f  %s" % (
            B, p, worst[0][1], ", ".join("%s %.4f" % (n.replace("resnet.", ""), e) for n, e in worst)), flush=True)


if __name__ == "__main__":
    main()
