"""K9 BatchNorm training statistics vs float64 (diagnostic): mean / invstd / running var errors for a
few shapes of the resnet_bgru layers (M = 512 x L rows, C channels)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechrecognitionproject_amd.nn import BatchNorm1d   # noqa: E402

torch.manual_seed(0)
for (M, C, mu, sd) in ((512 * 1000, 64, 0.5, 1.0), (512 * 125, 512, 3.0, 0.7), (512 * 125, 512, 0.0, 1e-2),
                       (512 * 250, 256, 10.0, 1.0), (2 * 1000, 64, 0.5, 1.0), (2 * 63, 512, 1.0, 1.0),
                       (2 * 125, 256, 1.0, 1.0), (2 * 250, 128, 1.0, 1.0)):
    x = (torch.randn(M, C, dtype=torch.float64) * sd + mu + torch.randn(C, dtype=torch.float64) * sd)
    x32 = x.float()
    bn = BatchNorm1d(C).cuda().train()
    y = bn(x32.cuda().view(-1, C)).double().cpu().view(M, C)
    x64 = x32.double()
    m = x64.mean(0)
    v = x64.var(0, unbiased=False)
    want = (x64 - m) / torch.sqrt(v + 1e-5)
    rv = 0.9 + 0.1 * x64.var(0, unbiased=True)
    print("M %d C %d mean %.1f std %g: y max err %.3g (of %.3g)  mean(y) max %.3g  running_var rel %.3g" % (
        M, C, mu, sd, (y - want).abs().max().item(), want.abs().max().item(), y.mean(0).abs().max().item(),
        ((bn.running_var.double().cpu() - rv).abs() / rv).max().item()))
