"""Diagnostic: fbanks_cnn conv1 + pool backward weight / bias gradient on fixed inputs, saved to a file
(A/B of two builds through SRK_LIB: python tools/c1w_dump.py OUT.pt [EARLIER.pt] — with a second file it
reports whether dW / db are bitwise equal to that earlier dump)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speechrecognitionproject_amd import nn as snn  # noqa: E402

g = torch.Generator().manual_seed(5)
out = {}
for (N, H, W, KH, KW, pool) in ((64, 98, 120, 7, 3, 3), (8, 51, 100, 3, 7, 5)):
    x = torch.randn(N, H, W, generator=g).cuda()
    w = (torch.randn(64, 1, KH, KW, generator=g) * 0.2).cuda().requires_grad_(True)
    b = torch.randn(64, generator=g).cuda().requires_grad_(True)
    y = snn._Conv1PoolFn.apply(x, w, b, (KH // 2, KW // 2), pool)
    y.backward(torch.randn(y.shape, generator=g).cuda())
    torch.cuda.synchronize()
    out["%dx%d" % (KH, KW)] = (w.grad.cpu(), b.grad.cpu())
torch.save(out, sys.argv[1])
print("saved", {k: float(v[0].abs().sum()) for k, v in out.items()})
if len(sys.argv) > 2:   # compare with an earlier dump
    ref = torch.load(sys.argv[2], weights_only=True)
    for k in out:
        print(k, "dw", "equal" if torch.equal(out[k][0], ref[k][0]) else "DIFF %.3g" % (out[k][0] - ref[k][0]).abs().max(),
              "db", "equal" if torch.equal(out[k][1], ref[k][1]) else "DIFF %.3g" % (out[k][1] - ref[k][1]).abs().max())
