"""Diagnose the HIP-graph capture hazard torch warns about ("AccumulateGrad node's stream does not
match ..."): after the warm-up steps of GraphedStep, list every autograd node object that is still
alive (and who holds it) right before the capture starts.

    python tools/graph_hazard.py [--model fbanks_cnn] [--batch 64]
"""
import argparse
import gc
import os
import sys
import warnings

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from speechrecognitionproject_amd import nn as snn  # noqa: E402
from speechrecognitionproject_amd.optim import Adam, FlatParams  # noqa: E402
from speechrecognitionproject_amd.synthetic import synthetic_clips  # noqa: E402


def alive_nodes():
    return [o for o in gc.get_objects() if isinstance(o, torch.autograd.function.BackwardCFunction)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="fbanks_cnn")
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    import importlib
    mod = importlib.import_module("speechrecognitionproject_amd.models.model_" + a.model)
    torch.manual_seed(0)
    net = mod.Network().cuda().train()
    flat = FlatParams(net.parameters())
    opt = Adam(net.parameters(), lr=1e-4, flat=flat)
    crit = snn.CrossEntropyLoss()
    x, y = synthetic_clips(a.batch, seed=1)
    x, y = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()

    def body():
        opt.zero_grad()
        loss = crit(net(x), y)
        loss.backward()
        opt.step()
        return loss

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        out = None
        for _ in range(2):
            out = body()
    torch.cuda.current_stream().wait_stream(side)
    out = None
    torch.cuda.synchronize()
    nodes = alive_nodes()
    print("alive autograd Function nodes before capture (no gc):", [type(n).__name__ for n in nodes])
    for n in nodes[:3]:
        for r in gc.get_referrers(n):
            print("   held by", type(r).__name__, str(r)[:160])
    del nodes
    gc.collect()
    print("after gc.collect():", [type(n).__name__ for n in alive_nodes()])
    warnings.simplefilter("always")
    g = torch.cuda.CUDAGraph()
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        with torch.cuda.graph(g):
            out = body()
        torch.cuda.synchronize()
    print("capture warnings:", [str(m.message)[:100] for m in w])
    g.replay()
    torch.cuda.synchronize()
    print("replay ok, loss", out.item())


if __name__ == "__main__":
    main()
