"""Benchmark: utterances/s of the MFCC + BiGRU train step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 256] [--model mfcc_bgru]

For N > 1 the driver launches one process per GPU with torch.distributed.run; each rank takes its
own shard of synthetic clips (weak scaling: per-GPU batch fixed) and the flat gradient buffer is
all-reduced through RCCL once per step.  Rank 0 prints ONE JSON line.

Workload (BASELINE.json configs[1], reference shapes per SURVEY.md §0.1): MFCC [39 x 51] computed
on the device from raw 1-s 16 kHz PCM (K1), then model_mfcc_bgru's 2-layer BiGRU(39->512) + FC,
cross-entropy, backward and Adam — the full training.py:85-91 step.  Clips are pre-staged in HBM
(the timed region starts with inputs resident).  "value" = clips processed by all ranks / time.

Measurement extras on the same line:
  roofline     — the dominant kernel of the timed steps, timed live with HIP events on its launch
                 stream (srk_prof_*), algorithmic flops / avg launch time vs the fp32 MFMA peak;
  mfcc_roofline— K1 alone on 65,536 clips (HBM-bound): algorithmic bytes / time vs 8 TB/s;
  cpu_baseline — the CPU restatement (oracle/: numpy MFCC per clip + torch-CPU GRU step) timed on
                 this host's cores on a bounded sample (rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from speechrecognitionproject_amd import _lib, features, parallel   # noqa: E402
from speechrecognitionproject_amd.nn import CrossEntropyLoss          # noqa: E402
from speechrecognitionproject_amd.optim import Adam, FlatParams       # noqa: E402
from speechrecognitionproject_amd.synthetic import synthetic_clips    # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3     # MI355X_MICROARCH.md, dense fp32 matrix (= vector) peak
PEAK_HBM_GBS = 8000.0             # MI355X HBM3E spec
MFCC_BYTES_PER_CLIP = 71956       # 64,000 in + 7,956 out
TRAIN_GFLOP_PER_UTT = {"mfcc_bgru": 1.9434, "spec_bgru": 2.0367}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_model(name):
    if name == "mfcc_bgru":
        from speechrecognitionproject_amd.models.model_mfcc_bgru import Network
    elif name == "spec_bgru":
        from speechrecognitionproject_amd.models.model_spec_bgru import Network
    else:
        raise SystemExit("unknown --model %s" % name)
    return Network()


def cpu_baseline(model_name, batch, seconds):
    """The oracle CPU path on a bounded sample: per-clip numpy features + torch-CPU train step."""
    from oracle import models as OM
    threads = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    cls = {"mfcc_bgru": OM.MfccBGRU, "spec_bgru": OM.SpecBGRU}[model_name]
    torch.manual_seed(0)
    net = cls()
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    x, y = synthetic_clips(batch, seed=99)
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    OM.train_step(net, xt, yt, optimizer=opt)      # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        OM.train_step(net, xt, yt, optimizer=opt)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 50:
            break
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        pass
    return {"value": round(n * batch / el, 2), "unit": "utt/s", "cores": threads, "kind": "port",
            "sample": "%d train steps x %d clips (%s CPU restatement: per-clip numpy features + torch-CPU "
                      "fp32 BiGRU fwd/bwd + Adam), %.1f s, %s" % (n, batch, model_name, el, cpu)}


def mfcc_roofline(n_clips=65536):
    x, _ = synthetic_clips(1024, seed=123)
    xd = torch.from_numpy(x).cuda().repeat(n_clips // 1024, 1)
    out = torch.empty((n_clips, 39, 51), device="cuda")
    for _ in range(2):
        features.mfcc(xd, out=out)
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    for _ in range(5):
        features.mfcc(xd, out=out)
    cnt, ms, work = _lib.prof_read("mfcc")
    _lib.prof_enable(False)
    gbs = work / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": None,
            "clips_per_launch": n_clips, "ms_per_launch": round(ms / cnt, 4),
            "bytes_per_clip": MFCC_BYTES_PER_CLIP}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="clips per GPU per step")
    ap.add_argument("--model", default="mfcc_bgru")
    ap.add_argument("--pool", type=int, default=4, help="distinct pre-staged batches per rank")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prof", action="store_true")
    ap.add_argument("--no-mfcc-roofline", action="store_true")
    args = ap.parse_args()

    rank, world, local = parallel.init_from_env()
    features.require_gpu()
    _lib.lib()
    dev = torch.device("cuda", local)
    torch.manual_seed(0)
    model = build_model(args.model).to(dev)
    flat = FlatParams(model.parameters())
    opt = Adam(model.parameters(), lr=1e-4, flat=flat)
    opt.grad_scale = 1.0 / world
    parallel.broadcast_flat(flat)
    crit = CrossEntropyLoss()

    B = args.batch
    x, y = synthetic_clips(args.pool * B, seed=1000 + rank)
    pcm = torch.from_numpy(x).to(dev).view(args.pool, B, -1)
    lab = torch.from_numpy(y).to(dev).view(args.pool, B)

    def step(i):
        opt.zero_grad()
        out = model(pcm[i % args.pool])
        loss = crit(out, lab[i % args.pool])
        loss.backward()
        parallel.allreduce_grads(flat)
        opt.step()
        return loss

    for i in range(args.warmup):
        loss = step(i)
    torch.cuda.synchronize()
    if not torch.isfinite(loss).item():
        raise SystemExit("non-finite loss during warm-up")
    if world > 1:
        torch.distributed.barrier()
    if not args.no_prof:
        _lib.prof_enable(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    final_loss = float(loss.item())

    kernels = {}
    if not args.no_prof:
        for name in ("gru_fwd_seq", "gru_bwd_seq", "gru_fwd_step", "gru_bwd_step", "gemm_f32", "mfcc", "adam"):
            c, ms, w = _lib.prof_read(name)
            if c:
                kernels[name] = {"launches": c, "ms_total": round(ms, 3), "work": w}
        _lib.prof_enable(False)

    if rank != 0:
        return
    value = world * B * args.steps / el
    roof = None
    mm = {k: v for k, v in kernels.items() if k in ("gru_fwd_seq", "gru_bwd_seq", "gru_fwd_step", "gru_bwd_step", "gemm_f32")}
    if mm:
        dom = max(mm, key=lambda k: mm[k]["ms_total"])
        k = mm[dom]
        tf = k["work"] / (k["ms_total"] * 1e-3) / 1e12
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(tf, 2), "peak": PEAK_FP32_MFMA_TFLOPS,
                "unit": "TFLOP/s", "frac": round(tf / PEAK_FP32_MFMA_TFLOPS, 4), "traffic": None,
                "avg_launch_ms": round(k["ms_total"] / k["launches"], 5),
                "flops_per_launch": k["work"] / k["launches"]}
    res = {
        "metric": "utterances/sec (1 s @16 kHz) MFCC+CNN-BiGRU train step",
        "value": round(value, 2), "unit": "utt/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32", "data": "synthetic (SURVEY.md §8d clip mix, pre-staged in HBM)",
        "config": {"workload": "cfg2 %s: on-device MFCC[39x51] + 2-layer BiGRU(512) + FC, CE, backward, Adam "
                               "(full training.py step), per-GPU batch %d" % (args.model, B),
                   "global_batch": world * B, "clip_samples": 16000, "parallelism": "dp%d" % world},
        "model_tflops": round(value * TRAIN_GFLOP_PER_UTT.get(args.model, 0) / 1e3, 2),
        "final_loss": round(final_loss, 5),
        "roofline": roof,
        "kernels": {k: {"launches": v["launches"], "ms_total": v["ms_total"]} for k, v in kernels.items()},
    }
    if not args.no_mfcc_roofline:
        res["mfcc_roofline"] = mfcc_roofline()
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.model, 32, args.cpu_seconds)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
