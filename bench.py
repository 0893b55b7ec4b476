"""Benchmark: utterances/s of the MFCC + BiGRU train step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--model mfcc_bgru|fbanks_cnn|resnet_bgru|spec_bgru|mfrn_bgru|cnn_bgru|spec_cnn]
                    [--batch B]

--model selects the BASELINE.json config (default = configs[1], the metric's headline model):
  mfcc_bgru   cfg2: on-device MFCC[39x51] + model_mfcc_bgru, 256 clips per GPU
  fbanks_cnn  cfg3: on-device log-mel fbank[98x120] + model_fbanks_cnn (dropout on), 512 per GPU
  resnet_bgru cfg4: raw-wave model_resnet_bgru (BatchNorm, per-rank statistics), 512 per GPU
  spec_bgru   cfg5: K4 noise-mix of int16 PCM with a resident noise bank + log spectrogram +
              model_spec_bgru, 512 per GPU
  mfrn_bgru   SURVEY.md §8f rank 1: MFCC (+) raw-wave ResNet-1D -> BiGRU(551), 256 per GPU
  cnn_bgru    SURVEY.md §8f rank 3: raw-wave strided CNN (BN, ReLU) -> BiGRU(512) over 498 steps, 512 per GPU
  spec_cnn    SURVEY.md §8f rank 3: on-device log spectrogram[49x321] + 4 Conv2d + pools + dropout + 2 FC,
              512 per GPU

For N > 1 one process runs per GPU: under torch.distributed.run (WORLD_SIZE set) each process is a
rank; started plainly as `python bench.py --gpus N` it re-launches itself through
torch.distributed.run (127.0.0.1, a free port) BEFORE touching the GPU and exits with the
launcher's code.  Each rank asserts the world size equals --gpus, takes its own shard of synthetic
clips (weak scaling: per-GPU batch fixed) and the flat gradient buffer is all-reduced through RCCL
once per step.  Rank 0 prints ONE JSON line.  --cpu-plumbing runs the launcher / rendezvous /
barrier / max-over-ranks timing / JSON path over gloo with a CPU all-reduce as the "step" (no GPU,
no measurement: the CPU test of the multi-rank harness).

Workload (BASELINE.json configs[1], reference shapes per SURVEY.md §0.1): MFCC [39 x 51] computed
on the device from raw 1-s 16 kHz PCM (K1), then model_mfcc_bgru's 2-layer BiGRU(39->512) + FC,
cross-entropy, backward and Adam — the full training.py:85-91 step.  Clips are pre-staged in HBM
(the timed region starts with inputs resident).  "value" = clips processed by all ranks / time.

--precision fp32 (default: exact fp32 MFMA, the reference's arithmetic) | bf16 | fp16 selects the
matrix-core operand precision (srk_set_option "matmul_precision"; fp16 adds a static loss scale).
With fp32, the same line also carries "bf16": the identical step re-timed with bf16 operands
(BASELINE.json names bf16 for cfg2), with its own roofline against the dense bf16 peak.

Measurement extras on the same line:
  roofline     — the dominant kernel of the timed steps, timed live with HIP events on its launch
                 stream (srk_prof_*), algorithmic flops / avg launch time vs the MFMA peak of its
                 operand type (fp32 157.3 TF, bf16/fp16 2.5 PF dense);
  mfcc_roofline— K1 alone on 65,536 clips (HBM-bound): algorithmic bytes / time vs 8 TB/s;
  cpu_baseline — the CPU restatement (oracle/: numpy features per clip + torch-CPU train step) timed
                 on this host's cores (every core this process may use, plus a
                 1-thread figure) on a bounded sample at the config's batch (rank 0, N = 1 only);
                 "cfg1" = BASELINE.json configs[0]: the MFCC restatement alone on 32 clips.
"""
import argparse
import json
import os
import sys
import time
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from speechrecognitionproject_amd import _lib, features, parallel   # noqa: E402
from speechrecognitionproject_amd.nn import CrossEntropyLoss          # noqa: E402
from speechrecognitionproject_amd.optim import Adam, FlatParams       # noqa: E402
from speechrecognitionproject_amd.synthetic import synthetic_clips    # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3     # MI355X_MICROARCH.md, dense fp32 matrix (= vector) peak
PEAK_LP_MFMA_TFLOPS = 2500.0      # MI355X_MICROARCH.md, dense bf16 / fp16 MFMA peak (no sparsity)
FP16_LOSS_SCALE = 1024.0          # static loss scale of the fp16 mode (unscaled in the Adam kernel)
PEAK_HBM_GBS = 8000.0             # MI355X HBM3E spec
MFCC_BYTES_PER_CLIP = 71956       # 64,000 in + 7,956 out
# FlopCounterMode on the reference modules (cnn_bgru / spec_cnn: on the oracle restatements)
TRAIN_GFLOP_PER_UTT = {"mfcc_bgru": 1.9434, "fbanks_cnn": 2.1449, "resnet_bgru": 25.8191,
                       "spec_bgru": 2.0367, "mfrn_bgru": 10.5777, "cnn_bgru": 27.1020, "spec_cnn": 1.4726}
DEFAULT_BATCH = {"mfcc_bgru": 256, "fbanks_cnn": 512, "resnet_bgru": 512, "spec_bgru": 512, "mfrn_bgru": 256,
                 "cnn_bgru": 512, "spec_cnn": 512}
CFG = {"mfcc_bgru": "cfg2 mfcc_bgru: on-device MFCC[39x51] + 2-layer BiGRU(512) + FC",
       "fbanks_cnn": "cfg3 fbanks_cnn: on-device log-mel fbank[98x120] + 4 Conv2d + pools + dropout + 2 FC",
       "resnet_bgru": "cfg4 resnet_bgru: raw-wave ResNet-1D (BN, ReLU) + Linear + 2-layer BiGRU(512) + FC",
       "spec_bgru": "cfg5 spec_bgru: on-device noise-mix (K4) + log spectrogram[49x321] + 2-layer BiGRU(512) + FC",
       "mfrn_bgru": "§8f-1 mfrn_bgru: on-device MFCC[51x39] (+) raw-wave ResNet-1D(k640/s40) + fc1 -> 2-layer "
                    "BiGRU(551 -> 512) + FC",
       "cnn_bgru": "§8f-3 cnn_bgru: raw-wave Conv1d(k80/s4) + 3 Conv1d(k4/s2) (BN, ReLU) + fc -> 2-layer BiGRU(512) "
                   "over 498 steps + FC",
       "spec_cnn": "§8f-3 spec_cnn: on-device log spectrogram[49x321] + 4 Conv2d + pools + dropout + 2 FC"}
# feature kernel of each model and its algorithmic bytes per clip
FEATURE = {"mfcc_bgru": ("mfcc", 71956), "fbanks_cnn": ("fbank", 111040), "spec_bgru": ("spec", 126916),
           "mfrn_bgru": ("mfcc", 71956), "spec_cnn": ("spec", 126916)}
MATRIX_KERNELS = ("gru_fwd_seq", "gru_bwd_seq", "gru_fwd_step", "gru_bwd_step", "gemm_f32",
                  "conv_fwd", "conv_dgrad", "conv_wgrad", "gemm_bf16", "gemm_f16", "gru_fwd_seq_lp", "gru_bwd_seq_lp",
                  "conv_fwd_lp", "conv_dgrad_lp", "conv_wgrad_lp")
LP_KERNELS = ("gemm_bf16", "gemm_f16", "gru_fwd_seq_lp", "gru_bwd_seq_lp", "conv_fwd_lp", "conv_dgrad_lp",
              "conv_wgrad_lp")
OTHER_KERNELS = ("mfcc", "fbank", "spec", "noise_mix", "adam", "batchnorm_fwd", "batchnorm_bwd", "conv1_pool_fwd",
                 "conv1_pool_wgrad",
                 "maxpool_fwd", "maxpool_bwd", "conv_to16")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_model(name):
    import importlib
    if name not in DEFAULT_BATCH:
        raise SystemExit("unknown --model %s" % name)
    return importlib.import_module("speechrecognitionproject_amd.models.model_%s" % name).Network()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        return "unknown"


def cpu_baseline(model_name, batch, seconds):
    """SURVEY.md §8d CPU baseline: the oracle CPU path (per-clip numpy features exactly as the
    reference's forward loops, torch-CPU fp32 model fwd/bwd + Adam) on this host, single process:
    (1) every core this process may use, train steps at the config's batch until `seconds`;
    (2) the same code pinned to 1 thread, one train step on a 32-clip sample (a full-batch
    1-thread step would take minutes); (3) "cfg1" (BASELINE.json configs[0]): the MFCC
    restatement alone on 32 clips, clips/s."""
    from oracle import features as OF
    from oracle import models as OM
    cls = {"mfcc_bgru": OM.MfccBGRU, "spec_bgru": OM.SpecBGRU, "fbanks_cnn": OM.FbanksCNN,
           "resnet_bgru": OM.ResnetBGRU, "mfrn_bgru": OM.MfrnBGRU, "cnn_bgru": OM.CnnBGRU,
           "spec_cnn": OM.SpecCNN}[model_name]
    # the CPU share this process may use: OMP_NUM_THREADS where the host sets it (the GPU box gives
    # each GPU 16 CPUs under a quota while affinity / os.cpu_count() show the whole machine — more
    # threads than the quota only thrash), else the affinity mask
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    cores = max(1, min(affinity, int(omp))) if omp.isdigit() else affinity
    prev_threads = torch.get_num_threads()
    torch.manual_seed(0)
    net = cls()
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)

    def run(n_clips, threads, budget, max_steps):
        torch.set_num_threads(threads)
        x, y = synthetic_clips(n_clips, seed=99)
        xt, yt = torch.from_numpy(x), torch.from_numpy(y)
        n, t0 = 0, time.perf_counter()
        while True:
            OM.train_step(net, xt, yt, optimizer=opt)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget or n >= max_steps:
                return n, el

    log("cpu_baseline: %s on %d threads" % (model_name, cores))
    run(min(batch, 32), cores, 0.0, 1)                        # warm-up (allocator, thread pool)
    n, el = run(batch, cores, seconds, 50)
    log("cpu_baseline: %d steps x %d clips in %.1f s; 1-thread leg" % (n, batch, el))
    # 1 thread: the config batch when one step fits ~seconds, else the largest multiple of 32 that does
    n1, el1 = run(32, 1, 0.0, 1)
    b1 = int(min(batch, max(32, (seconds / (el1 / 32)) // 32 * 32)))
    if b1 > 32:
        n1, el1 = run(b1, 1, 0.0, 1)
    # cfg1: MFCC restatement on 32 clips, serial per clip like the reference's forward (:31-32)
    x32, _ = synthetic_clips(32, seed=98)
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or time.perf_counter() - t0 < 1.0:
        for c in x32:
            OF.compute_mfcc(c)
        reps += 1
    el_mfcc = (time.perf_counter() - t0) / reps
    torch.set_num_threads(prev_threads)
    cpu = _cpu_model()
    return {"value": round(n * batch / el, 2), "unit": "utt/s", "cores": cores, "kind": "port",
            "sample": "%d train steps x %d clips (the config batch; %s CPU restatement: per-clip numpy features + "
                      "torch-CPU fp32 fwd/bwd + Adam), %.1f s on %d threads, %s (affinity %d CPUs, os.cpu_count() = %s, "
                      "OMP_NUM_THREADS = %s)" % (n, batch, model_name, el, cores, cpu, affinity, os.cpu_count(), omp or "unset"),
            "one_thread": {"value": round(n1 * b1 / el1, 2), "unit": "utt/s", "cores": 1,
                           "sample": "%d train step x %d clips, %.1f s" % (n1, b1, el1)},
            "cfg1": {"value": round(32 / el_mfcc, 2), "unit": "clips/s", "cores": 1,
                     "sample": "BASELINE.json configs[0]: MFCC[39x51] restatement (numpy, float64 librosa-0.6 "
                               "semantics) on 32 x 1-s clips, serial, %.4f s per pass (mean of %d)" % (el_mfcc, reps)}}


def pmc_traffic(kernel, model="mfcc_bgru"):
    """HBM bytes per launch of `kernel` from the committed PMC summary of the same bench command
    (tools/pmc_traffic.py over separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected):
    profiles/pmc_traffic.json for the default cfg2 command, pmc_traffic_<model>.json for
    `--model <model>`; None if no summary is committed."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json" if model == "mfcc_bgru" else "pmc_traffic_%s.json" % model)
    try:
        with open(p) as f:
            v = json.load(f)["bytes_per_launch"].get(kernel)
        return None if v is None else v["total"]
    except (OSError, ValueError, KeyError):
        return None


def feature_roofline(model_name, n_clips=65536):
    """The model's feature kernel alone on a large batch (HBM-bound): algorithmic bytes / time."""
    name, per_clip = FEATURE[model_name]
    fn = {"mfcc": lambda x, out=None: features.mfcc(x, time_major=True, out=out), "fbank": features.fbank,
          "spec": lambda x, out=None: features.spec(x, transposed=True, out=out)}[name]   # the models' layouts
    x, _ = synthetic_clips(1024, seed=123)
    xd = torch.from_numpy(x).cuda().repeat(n_clips // 1024, 1)
    out = None
    for _ in range(2):
        out = fn(xd, out=out)
    torch.cuda.synchronize()
    _lib.prof_enable(True)
    for _ in range(5):
        fn(xd, out=out)
    cnt, ms, work = _lib.prof_read(name)
    _lib.prof_enable(False)
    gbs = work / (ms * 1e-3) / 1e9
    return {"kernel": name, "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": None,
            "clips_per_launch": n_clips, "ms_per_launch": round(ms / cnt, 4), "bytes_per_clip": per_clip}


def _relaunch(args):
    """`bench.py --gpus N` outside torch.distributed.run: start N ranks through it (a child
    process; nothing here has touched the GPU) and return its exit code."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log("bench: launching %d ranks: %s" % (args.gpus, " ".join(cmd)))
    return subprocess.run(cmd).returncode


PARAMS = {"mfcc_bgru": 6435852, "fbanks_cnn": 1439244, "spec_bgru": 7302156, "resnet_bgru": 27494573}


def plumbing(args, rank, world):
    """--cpu-plumbing: the multi-rank harness on CPU (gloo): a flat-buffer all-reduce of the model's
    gradient size as the step, the same barrier / max-over-ranks timing and rank-0 JSON line."""
    import torch.distributed as dist
    grad = torch.ones(PARAMS.get(args.model, 1 << 20))
    for _ in range(args.warmup):
        parallel.allreduce_grads(types.SimpleNamespace(grad=grad))
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        parallel.allreduce_grads(types.SimpleNamespace(grad=grad))
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "cpu plumbing check (not a measurement)", "value": None, "unit": "utt/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "none (gloo all-reduce only)",
                          "config": {"workload": "plumbing", "model": args.model, "parallelism": "dp%d" % world}}),
              flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="clips per GPU per step (default per model)")
    ap.add_argument("--model", default="mfcc_bgru")
    ap.add_argument("--pool", type=int, default=4, help="distinct pre-staged batches per rank")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--precision", default="fp32", choices=sorted(_lib.PRECISIONS),
                    help="matrix-core operand precision (fp32 = the reference's arithmetic; bf16 / fp16 "
                         "operands with fp32 accumulation)")
    ap.add_argument("--no-lowprec", dest="lowprec", action="store_false",
                    help="skip the extra bf16 measurement reported under \"bf16\" on the same line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prof", action="store_true")
    ap.add_argument("--no-feature-roofline", "--no-mfcc-roofline", dest="no_feature_roofline", action="store_true")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false",
                    help="N > 1: one blocking all-reduce after backward instead of bucketed all-reduces overlapped "
                         "with it (parallel.GradReducer)")
    ap.add_argument("--bucket-mb", type=float, default=8.0, help="gradient bucket size of the overlapped all-reduce")
    ap.add_argument("--sync-bn", action="store_true",
                    help="BatchNorm statistics over the global batch of all ranks (SyncBatchNorm1d; resnet_bgru, "
                         "cnn_bgru, mfrn_bgru)")
    ap.add_argument("--cpu-plumbing", action="store_true",
                    help="exercise the N-rank launch / timing / JSON path over gloo on CPU (no GPU; no measurement)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_relaunch(args))
    rank, world, local = parallel.init_from_env(backend="gloo" if args.cpu_plumbing else None)
    if world != args.gpus:
        raise SystemExit("bench: --gpus %d but the process group has %d ranks" % (args.gpus, world))
    if args.cpu_plumbing:
        plumbing(args, rank, world)
        return
    features.require_gpu()
    _lib.lib()
    loss_scale = 1.0
    dev = torch.device("cuda", local)
    torch.manual_seed(0)
    model = build_model(args.model).to(dev)
    if args.sync_bn:
        from speechrecognitionproject_amd.nn import convert_sync_batchnorm
        model = convert_sync_batchnorm(model)
    flat = FlatParams(model.parameters())
    opt = Adam(model.parameters(), lr=1e-4, flat=flat)
    parallel.broadcast_flat(flat)
    reducer = parallel.GradReducer(flat, bucket_mb=args.bucket_mb) if (world > 1 and args.overlap) else None
    crit = CrossEntropyLoss()

    B = args.batch or DEFAULT_BATCH[args.model]
    x, y = synthetic_clips(args.pool * B, seed=1000 + rank, clip=30000 if args.model == "spec_bgru" else 32767)
    lab = torch.from_numpy(y).to(dev).view(args.pool, B)
    if args.model == "spec_bgru":
        # cfg5: int16 PCM + resident noise bank; the per-clip (file, offset, gain) draws of
        # dataset.py:190-193 are made up front (numpy), the mix runs on the device every step.
        from speechrecognitionproject_amd.synthetic import synthetic_noise_bank, synthetic_noise_draws
        pcm16 = torch.from_numpy(x.astype(np.int16)).to(dev).view(args.pool, B, -1)
        bank = torch.from_numpy(synthetic_noise_bank()).to(dev)
        draws = [torch.from_numpy(a).to(dev).view(args.pool, B)
                 for a in synthetic_noise_draws(args.pool * B, seed=2 + rank)]
        mixed = torch.empty((B, 16000), device=dev)

        def inputs(i):
            j = i % args.pool
            return features.noise_mix(pcm16[j], bank, draws[0][j], draws[1][j], draws[2][j], out=mixed)
    else:
        pcm = torch.from_numpy(x).to(dev).view(args.pool, B, -1)

        def inputs(i):
            return pcm[i % args.pool]

    def step(i):
        opt.zero_grad()
        if reducer is not None:
            reducer.begin()
        out = model(inputs(i))
        loss = crit(out, lab[i % args.pool])
        (loss * loss_scale if loss_scale != 1.0 else loss).backward()
        if reducer is not None:
            reducer.finish()        # bucketed all-reduces launched during backward
        else:
            parallel.allreduce_grads(flat)
        opt.step()
        return loss

    def timed(precision):
        """W warm-up + K timed steps at one matrix precision -> (seconds, kernel records, loss)."""
        nonlocal loss_scale
        log("bench: %s %s, %d warm-up + %d timed steps" % (args.model, precision, args.warmup, args.steps))
        _lib.set_matmul_precision(precision)
        loss_scale = FP16_LOSS_SCALE if precision == "fp16" else 1.0
        opt.grad_scale = 1.0 / (world * loss_scale)
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
        kernels = {}
        if not args.no_prof:
            for name in MATRIX_KERNELS + OTHER_KERNELS:
                c, ms, w = _lib.prof_read(name)
                if c:
                    kernels[name] = {"launches": c, "ms_total": round(ms, 3), "work": w}
            _lib.prof_enable(False)
        return el, kernels, float(loss.item())

    def roofline(kernels, traffic_ok):
        mm = {k: v for k, v in kernels.items() if k in MATRIX_KERNELS}
        if not mm:
            return None
        dom = max(mm, key=lambda k: mm[k]["ms_total"])
        k = mm[dom]
        tf = k["work"] / (k["ms_total"] * 1e-3) / 1e12
        peak = PEAK_LP_MFMA_TFLOPS if dom in LP_KERNELS else PEAK_FP32_MFMA_TFLOPS
        return {"bound": "mfma", "kernel": dom, "achieved": round(tf, 2), "peak": peak,
                "unit": "TFLOP/s", "frac": round(tf / peak, 4),
                "traffic": pmc_traffic(dom, args.model) if traffic_ok else None, "traffic_unit": "bytes/launch",
                "avg_launch_ms": round(k["ms_total"] / k["launches"], 5),
                "flops_per_launch": k["work"] / k["launches"]}

    el, kernels, final_loss = timed(args.precision)
    # the same step with 16-bit matrix-core operands (BASELINE.json cfg2 names bf16), same line
    lp = None
    if args.lowprec and args.precision == "fp32":
        lp_el, lp_kernels, lp_loss = timed("bf16")
        lp = {"dtype": "bf16", "value": round(world * B * args.steps / lp_el, 2),
              "ms_per_step": round(lp_el / args.steps * 1e3, 3), "final_loss": round(lp_loss, 5),
              "roofline": roofline(lp_kernels, True),   # the PMC summary of the same command, if committed
              "kernels": {k: {"launches": v["launches"], "ms_total": v["ms_total"]} for k, v in lp_kernels.items()}}
        _lib.set_matmul_precision(args.precision)

    # a persistent kernel that timed out invalidates every number above: fail loudly
    _lib.check_health(sync=True)
    if rank != 0:
        return
    value = world * B * args.steps / el
    roof = roofline(kernels, True)
    res = {
        "metric": "utterances/sec (1 s @16 kHz) MFCC+CNN-BiGRU train step",
        "value": round(value, 2), "unit": "utt/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision, "data": "synthetic (SURVEY.md §8d clip mix, pre-staged in HBM)",
        "config": {"workload": "%s, CE, backward, Adam (full training.py step), per-GPU batch %d"
                               % (CFG[args.model], B), "model": args.model,
                   "global_batch": world * B, "clip_samples": 16000, "parallelism": "dp%d" % world,
                   "allreduce": ("bucketed %.0f MB, overlapped with backward" % args.bucket_mb
                                 if reducer is not None else ("one flat buffer after backward" if world > 1 else None)),
                   "sync_bn": bool(args.sync_bn)},
        "model_tflops": round(value * TRAIN_GFLOP_PER_UTT.get(args.model, 0) / 1e3, 2),
        "final_loss": round(final_loss, 5),
        "roofline": roof,
        "kernels": {k: {"launches": v["launches"], "ms_total": v["ms_total"]} for k, v in kernels.items()},
    }
    if lp is not None:
        res["bf16"] = lp
    if not args.no_feature_roofline and args.model in FEATURE:
        log("bench: feature roofline")
        res["feature_roofline"] = feature_roofline(args.model)
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.model, B, args.cpu_seconds)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
