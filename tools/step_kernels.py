"""Per-launch kernel table of one model's train step (eager, srk_prof): every GEMM / conv / GRU launch
with its shape, mean time and achieved TFLOP/s (or GB/s), for picking the next kernel to work on.

    python tools/step_kernels.py [model] [precision] [batch] [steps]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from oracle import models as OM
from speechrecognitionproject_amd import _lib
from speechrecognitionproject_amd.nn import CrossEntropyLoss
from speechrecognitionproject_amd.optim import Adam, FlatParams
from speechrecognitionproject_amd.synthetic import synthetic_clips
import importlib

name = sys.argv[1] if len(sys.argv) > 1 else "mfcc_bgru"
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
B = int(sys.argv[3]) if len(sys.argv) > 3 else 256
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
_lib.set_matmul_precision(prec)
net = importlib.import_module("speechrecognitionproject_amd.models.model_" + name).Network().cuda()
flat = FlatParams(net.parameters())
opt = Adam(net.parameters(), lr=1e-4, flat=flat)
crit = CrossEntropyLoss()
x, y = synthetic_clips(B, seed=3)
xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()


def step():
    opt.zero_grad()
    crit(net(xd), yd).backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
_lib.prof_enable(True)
for _ in range(steps):
    step()
torch.cuda.synchronize()
rows = _lib.prof_kernels()
_lib.prof_enable(False)
tot = sum(r["ms_total"] for r in rows) / steps
print("%s %s B=%d: kernel sum %.3f ms/step" % (name, prec, B, tot))
for r in sorted(rows, key=lambda r: -r["ms_total"]):
    per = r["ms_total"] / r["launches"]
    rate = r["work"] / r["launches"] / (per * 1e-3) / 1e12 if per > 0 else 0.0
    print("%-58s %4d  %8.1f us  %8.3f ms/step  %7.1f T/s" % (r["kernel"][:58], r["launches"] // steps, per * 1e3,
                                                         r["ms_total"] / steps, rate))
