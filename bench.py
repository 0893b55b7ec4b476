"""Benchmark: utterances/s of the MFCC + BiGRU train step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--model mfcc_bgru|fbanks_cnn|resnet_bgru|spec_bgru|mfrn_bgru|cnn_bgru|spec_cnn]
                    [--batch B]

--model selects the BASELINE.json config (default = configs[1], the metric's headline model):
  mfcc_bgru   cfg2: on-device MFCC[39x51] + model_mfcc_bgru, 256 clips per GPU
  fbanks_cnn  cfg3: on-device log-mel fbank[98x120] + model_fbanks_cnn (dropout on), 512 per GPU
  resnet_bgru cfg4: raw-wave model_resnet_bgru (BatchNorm, per-rank statistics), 512 per GPU
  spec_bgru   cfg5: K4 noise-mix of int16 PCM with a resident noise bank fused into the log spectrogram +
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

Step execution: after W warm-up steps the train step is captured into HIP graphs
(speechrecognitionproject_amd/graphs.py; per-step host values — the Adam step count and the dropout
seed — live on the device), one per pre-staged batch slot sharing one memory pool, and the K timed
steps are graph replays.  N > 1: the whole step is one graph — forward, backward with the bucketed
RCCL all-reduces forked where each bucket's gradients are final (on a process group used only under
capture, parallel.capture_group), the join and Adam; --allreduce-outside-graph replays forward +
backward and all-reduces the flat gradient buffer eagerly between the replay and the Adam launch.
--no-graph times the eager step instead (N > 1: bucketed all-reduces overlapped with backward).
The per-kernel HIP-event timers cannot run inside a graph: kernel times ("kernels", "roofline")
come from a separate eager pass of the same step (--prof-steps, default 5), reported with its own
"eager_ms_per_step".

Default run (no --model): the cfg2 headline, then compact records under "configs" for BASELINE.json's
other configs at their per-GPU batch — cfg3 fbanks_cnn fp32 512, cfg4 resnet_bgru fp32 512, cfg5
spec_bgru fp16 512 with the noise-mix in the step (static loss scale 1024 with the overflow check and
skip) — and the metric's literal MFCC+CNN-BiGRU model (mfrn_bgru fp32 256), each with value /
ms_per_step / roofline (--no-configs skips them); "h2d": the cfg2 step (fp32 and bf16) fed from
pinned host memory with a double-buffered upload (SURVEY.md §8d's second figure; --no-h2d skips it);
"feature_roofline_other": K2 (fbank) and K3 (spectrogram) alone on 65,536 clips.

Measurement extras on the same line:
  roofline     — the dominant kernel of the timed steps, timed live with HIP events on its launch
                 stream (srk_prof_*), algorithmic flops / avg launch time vs the MFMA peak of its
                 operand type (fp32 157.3 TF, bf16/fp16 2.5 PF dense);
  feature_roofline — K1 alone on 65,536 clips (HBM-bound): algorithmic bytes / time vs 8 TB/s;
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
from speechrecognitionproject_amd.optim import Adam, FlatParams, LossScaler   # noqa: E402
from speechrecognitionproject_amd.synthetic import synthetic_clips    # noqa: E402

PEAK_FP32_MFMA_TFLOPS = 157.3     # MI355X_MICROARCH.md, dense fp32 matrix (= vector) peak
PEAK_LP_MFMA_TFLOPS = 2500.0      # MI355X_MICROARCH.md, dense bf16 / fp16 MFMA peak (no sparsity)
FP16_LOSS_SCALE = 1024.0          # static loss scale of the fp16 mode (optim.LossScaler: unscaled in the Adam
                                  # kernel, a step with inf / NaN gradients skipped and counted)
PEAK_HBM_GBS = 8000.0             # MI355X HBM3E spec
MFCC_BYTES_PER_CLIP = 71956       # 64,000 in + 7,956 out
# FlopCounterMode on the reference modules (cnn_bgru / spec_cnn: on the oracle restatements)
TRAIN_GFLOP_PER_UTT = {"mfcc_bgru": 1.9434, "fbanks_cnn": 2.1449, "resnet_bgru": 25.8191,
                       "spec_bgru": 2.0367, "mfrn_bgru": 10.5777, "cnn_bgru": 27.1020, "spec_cnn": 1.4726,
                       "mfcc_bgru_40x98": 1.9434 * 98 / 51}   # (the 51-step figure scaled to 98 steps)
DEFAULT_BATCH = {"mfcc_bgru": 256, "fbanks_cnn": 512, "resnet_bgru": 512, "spec_bgru": 512, "mfrn_bgru": 256,
                 "cnn_bgru": 512, "spec_cnn": 512, "mfcc_bgru_40x98": 256}
CFG = {"mfcc_bgru": "cfg2 mfcc_bgru: on-device MFCC[39x51] + 2-layer BiGRU(512) + FC",
       "mfcc_bgru_40x98": "cfg2 literal, PERF-ONLY NON-REFERENCE variant: on-device MFCC[40x98] (DCT of the K2 "
                          "fbank) + 2-layer BiGRU(40 -> 512) over 98 steps + FC (SURVEY.md §0.1)",
       "fbanks_cnn": "cfg3 fbanks_cnn: on-device log-mel fbank[98x120] + 4 Conv2d + pools + dropout + 2 FC",
       "resnet_bgru": "cfg4 resnet_bgru: raw-wave ResNet-1D (BN, ReLU) + Linear + 2-layer BiGRU(512) + FC",
       "spec_bgru": "cfg5 spec_bgru: on-device noise-mix (K4) fused into the log spectrogram[49x321] (K3) + 2-layer BiGRU(512) + FC",
       "mfrn_bgru": "§8f-1 mfrn_bgru: on-device MFCC[51x39] (+) raw-wave ResNet-1D(k640/s40) + fc1 -> 2-layer "
                    "BiGRU(551 -> 512) + FC",
       "cnn_bgru": "§8f-3 cnn_bgru: raw-wave Conv1d(k80/s4) + 3 Conv1d(k4/s2) (BN, ReLU) + fc -> 2-layer BiGRU(512) "
                   "over 498 steps + FC",
       "spec_cnn": "§8f-3 spec_cnn: on-device log spectrogram[49x321] + 4 Conv2d + pools + dropout + 2 FC"}
# feature kernel of each model and its algorithmic bytes per clip
FEATURE = {"mfcc_bgru": ("mfcc", 71956), "fbanks_cnn": ("fbank", 111040), "spec_bgru": ("spec", 126916),
           "mfrn_bgru": ("mfcc", 71956), "spec_cnn": ("spec", 126916)}
FEATURE_BYTES = {k: b for k, b in FEATURE.values()}
MATRIX_KERNELS = ("gru_fwd_seq", "gru_bwd_seq", "gru_fwd_step", "gru_bwd_step", "gemm_f32",
                  "conv_fwd", "conv_dgrad", "conv_wgrad", "gemm_bf16", "gemm_f16", "gru_fwd_seq_lp", "gru_bwd_seq_lp",
                  "conv_fwd_lp", "conv_dgrad_lp", "conv_wgrad_lp")
LP_KERNELS = ("gemm_bf16", "gemm_f16", "gru_fwd_seq_lp", "gru_bwd_seq_lp", "conv_fwd_lp", "conv_dgrad_lp",
              "conv_wgrad_lp")
OTHER_KERNELS = ("mfcc", "fbank", "spec", "noise_mix", "adam", "grad_check", "batchnorm_fwd", "batchnorm_bwd", "conv1_pool_fwd",
                 "conv1_pool_wgrad",
                 "maxpool_fwd", "maxpool_bwd", "conv_to16", "conv_unpool16", "gru_dwhh_reduce", "conv_colsum",
                 "conv_to16_colsum", "conv_unpool16_colsum", "pitch_shift")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_model(name):
    import importlib
    if name not in DEFAULT_BATCH:
        raise SystemExit("unknown --model %s" % name)
    if name == "mfcc_bgru_40x98":   # the perf-only "MFCC (40x98)" variant of the cfg2 model
        from speechrecognitionproject_amd.models import model_mfcc_bgru
        return model_mfcc_bgru.Network(features="mfcc40x98")
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


def pmc_traffic(kernel, cmd):
    """(HBM bytes per launch, source) of the kernel category `kernel` from the committed PMC summary of
    THIS command and THIS build (tools/pmc_traffic.py over separate rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes, gfx950-corrected): profiles/pmc_traffic_<model>.json, used only when the command it records
    (model, per-GPU batch, world size, precisions, options) matches `cmd` AND its source stamp equals the
    loaded library's srk_source_stamp() — counters of other kernel sources describe other code; else
    (None, reason)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic_%s.json" % cmd["model"])
    try:
        with open(p) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC file"
    rec = doc.get("command") or {}
    same = (rec.get("model") == cmd["model"] and rec.get("batch") == cmd["batch"] and rec.get("world") == cmd["world"]
            and cmd["precision"] in rec.get("precisions", ()) and bool(rec.get("sync_bn")) == cmd["sync_bn"]
            and bool(rec.get("conv_fwd_fp32")) == cmd["conv_fwd_fp32"])
    if not same:
        return None, "PMC file of another command"
    stamp = doc.get("source_stamp")
    if stamp != _lib.source_stamp():
        return None, "PMC file of another build (stamp %s, library %s)" % (stamp, _lib.source_stamp())
    v = doc.get("bytes_per_launch", {}).get(kernel)
    if v is None:
        return None, "kernel not in PMC file"
    return v["total"], "profiles/pmc_traffic_%s.json (%s, stamp %s)" % (cmd["model"], doc.get("source", ""), stamp)


def feature_roofline(model_name=None, n_clips=65536, kernel=None):
    """A feature kernel alone on a large batch (HBM-bound): algorithmic bytes / time.  `kernel` (mfcc /
    fbank / spec) or the feature kernel of `model_name`."""
    name, per_clip = FEATURE[model_name] if kernel is None else next(v for v in FEATURE.values() if v[0] == kernel)
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
    res = {"kernel": name, "bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
           "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": None,
           "clips_per_launch": n_clips, "ms_per_launch": round(ms / cnt, 4), "bytes_per_clip": per_clip}
    res.update(feature_pmc(name, n_clips))
    return res


def feature_pmc(name, n_clips):
    """HBM bytes and SQ counters of this feature launch from profiles/pmc_feature.json
    (tools/feat_pmc.sh: rocprofv3 PMC passes over tools/mfcc_only.py, the same kernel, layout and
    clip count), used only when the recorded clip count matches."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_feature.json")
    try:
        with open(path) as fh:
            rec = json.load(fh)
    except (OSError, ValueError):
        return {}
    ent = rec.get("kernels", {}).get(name)
    if rec.get("clips_per_launch") != n_clips or not ent or "traffic_per_launch" not in ent:
        return {}
    if rec.get("source_stamp") != _lib.source_stamp():     # counters of another build: not this kernel
        return {"pmc_source": "none: profiles/pmc_feature.json is of another build (stamp %s, library %s)"
                              % (rec.get("source_stamp"), _lib.source_stamp())}
    pc = ent.get("per_clip", {})
    return {"traffic": ent["traffic_per_launch"], "traffic_per_clip": ent["traffic_per_clip"],
            "sq_insts_valu_per_clip": pc.get("SQ_INSTS_VALU"), "sq_wait_inst_any_per_clip": pc.get("SQ_WAIT_INST_ANY"),
            "sq_wave_cycles_per_clip": pc.get("SQ_WAVE_CYCLES"), "sq_insts_lds_per_clip": pc.get("SQ_INSTS_LDS"),
            "traffic_ratio": round(ent["traffic_per_clip"] / FEATURE_BYTES[name], 3),
            "pmc_source": "profiles/pmc_feature.json (%s, stamp %s)" % (rec.get("source", ""), rec.get("source_stamp"))}


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


EXTRA_CONFIGS = (  # BASELINE.json configs[2..4] at their per-GPU batch (the default run appends them), the
    ("cfg3", "fbanks_cnn", "fp32", 512, 10),     # metric's literal "MFCC+CNN-BiGRU" model, and the
    ("cfg4", "resnet_bgru", "fp32", 512, 4),     # 16-bit re-timings of the conv configs (the matrix cores' 16-bit
    ("cfg5", "spec_bgru", "fp16", 512, 20),      # conv path on the driver's line)
    ("mfrn", "mfrn_bgru", "fp32", 256, 10),
    ("cfg3-bf16", "fbanks_cnn", "bf16", 512, 10),
    ("cfg4-bf16", "resnet_bgru", "bf16", 512, 4),
    # the faithful 16-bit mode of the BatchNorm model: conv forwards on fp32 operands (srk option conv_fwd_fp32;
    # cfg4-bf16's gradients are 4-39 % norm-wise from float64, these <= 2e-2: tools/bf16_policy_resnet.py)
    ("cfg4-bf16-faithful", "resnet_bgru", "bf16", 512, 4),
    # BASELINE.json configs[1] read literally, "MFCC (40x98) ... bf16": a perf-only, non-reference variant
    ("cfg2-mfcc40x98-bf16", "mfcc_bgru_40x98", "bf16", 256, 20),
)
# what each 16-bit record's gradients are worth against float64 (tests/test_config_batch_gpu.py)
GRADIENTS = {"cfg3-bf16": "every gradient tensor <= 2e-2 norm-wise of the fp32 oracle",
             "cfg4-bf16": "NOT reference-faithful: conv / BatchNorm gradients 4-39 % norm-wise from float64 (the "
                          "forward's bf16 operand rounding amplified by the training-mode BatchNorm chain); "
                          "cfg4-bf16-faithful is the faithful 16-bit mode",
             "cfg4-bf16-faithful": "every gradient tensor <= max(2e-2, 1.25 x the fp32 oracle's) norm-wise of "
                                   "float64: conv forwards on fp32 operands, data / weight gradients, GEMMs and the "
                                   "recurrence on bf16",
             "cfg5": "every gradient tensor <= 2e-2 norm-wise of the fp32 oracle (fp16, loss scale 1024)"}


class Workload:
    """One model's train step on this rank (per-GPU batch B, `pool` distinct pre-staged batches),
    timed eagerly or as HIP-graph replays; the rank-0 JSON line is built from run()."""

    def __init__(self, args, model_name, B, rank, world, dev):
        self.args, self.name, self.B, self.rank, self.world, self.dev = args, model_name, B, rank, world, dev
        self.conv_fwd_fp32 = bool(args.conv_fwd_fp32)
        torch.manual_seed(0)
        model = build_model(model_name).to(dev)
        if args.sync_bn:
            from speechrecognitionproject_amd.nn import convert_sync_batchnorm
            model = convert_sync_batchnorm(model)
        self.model = model
        self.flat = FlatParams(model.parameters())
        self.opt = Adam(model.parameters(), lr=1e-4, flat=self.flat)
        parallel.broadcast_flat(self.flat)
        self.reducer = None
        self.crit = CrossEntropyLoss()
        self.scaler = None
        pool = args.pool
        x, y = synthetic_clips(pool * B, seed=1000 + rank, clip=30000 if model_name == "spec_bgru" else 32767)
        self.lab = torch.from_numpy(y).to(dev).view(pool, B)
        if model_name == "spec_bgru":
            # cfg5: int16 PCM + resident noise bank; the per-clip (file, offset, gain) draws of
            # dataset.py:190-193 are made up front (numpy); the mix runs on the device every step, inside
            # the spectrogram kernel's sample loads (features.NoisyClips -> srk_spec_noise_fwd, K4 fused)
            from speechrecognitionproject_amd.synthetic import synthetic_noise_bank, synthetic_noise_draws
            self.pcm16 = torch.from_numpy(x.astype(np.int16)).to(dev).view(pool, B, -1)
            self.bank = torch.from_numpy(synthetic_noise_bank()).to(dev)
            self.draws = [torch.from_numpy(a).to(dev).view(pool, B) for a in synthetic_noise_draws(pool * B, seed=2 + rank)]
            self.noisy = [features.NoisyClips(self.pcm16[j], self.bank, *[d[j] for d in self.draws])
                          for j in range(pool)]
        else:
            self.pcm = torch.from_numpy(x).to(dev).view(pool, B, -1)

    # ---- inputs
    def _inputs(self, srcs):
        return srcs[0]

    def _batch(self, i):
        j = i % self.args.pool
        if self.name == "spec_bgru":
            return [self.noisy[j]]
        return [self.pcm[j]]

    # ---- the step
    def _fwd_bwd(self, srcs, lab):
        self.opt.zero_grad()
        if self.reducer is not None:
            self.reducer.begin()
        out = self.model(self._inputs(srcs))
        loss = self.crit(out, lab)
        (self.scaler.scale(loss) if self.scaler is not None else loss).backward()
        return loss

    def _exchange_and_update(self):
        if self.reducer is not None:
            self.reducer.finish()        # bucketed all-reduces launched during backward
        else:
            parallel.allreduce_grads(self.flat)
        self.opt.step(scaler=self.scaler)

    def eager_step(self, i):
        loss = self._fwd_bwd(self._batch(i), self.lab[i % self.args.pool])
        self._exchange_and_update()
        return loss

    def _graph_body(self):
        j = self._slot
        loss = self._fwd_bwd(self._batch(j), self.lab[j])
        if self.world == 1:
            self.opt.step(scaler=self.scaler)
        elif self.exchange_in_graph:
            self._exchange_and_update()   # the bucketed RCCL all-reduces + Adam, captured with the step
        return loss

    def _capture(self, graph, warmup):
        """One GraphedStep per pre-staged batch slot, sharing one memory pool."""
        from speechrecognitionproject_amd.graphs import GraphedStep
        graphs = []
        mode = "thread_local" if self.exchange_in_graph else "global"
        for j in range(self.args.pool):
            self._slot = j
            graphs.append(GraphedStep(self._graph_body, warmup=max(2, warmup) if j == 0 else 0,
                                      pool=graphs[0].pool() if graphs else None, capture_error_mode=mode))
        return graphs

    def run(self, precision, steps, warmup, graph):
        """W warm-up + K timed steps at one matrix precision -> record dict (rank 0 uses it)."""
        args = self.args
        log("bench: %s %s B=%d, %d warm-up + %d timed steps%s" % (self.name, precision, self.B, warmup, steps,
                                                                   " (HIP graph)" if graph else ""))
        _lib.set_matmul_precision(precision)
        _lib.set_option("conv_fwd_fp32", 1 if self.conv_fwd_fp32 else 0)
        self.scaler = LossScaler(FP16_LOSS_SCALE, dynamic=False, device=self.dev) if precision == "fp16" else None
        self.opt.grad_scale = 1.0 / self.world
        # N > 1 with HIP graphs: the bucketed all-reduces are captured inside the step graph (forked where each
        # bucket's gradients are final, joined before Adam) on the capture-only process group;
        # --allreduce-outside-graph replays forward + backward and runs one flat all-reduce + Adam eagerly
        self.exchange_in_graph = (graph and self.world > 1 and args.overlap and not args.allreduce_outside_graph)
        if graph and self.world > 1:
            parallel.capture_group()   # before any capture: SyncBN's captured exchanges use it in every form
        self.reducer = (parallel.GradReducer(
            self.flat, bucket_mb=args.bucket_mb,
            capture_group=parallel.capture_group() if self.exchange_in_graph else None)
                        if (self.world > 1 and args.overlap and (self.exchange_in_graph or not graph)) else None)
        graphs = []
        if graph:
            # one graph per pre-staged batch slot, sharing one memory pool: each reads its own resident
            # batch (no per-step input copy); the first capture's warm-up covers the others
            failed = 0
            try:
                graphs = self._capture(graph, warmup)
            except Exception as e:   # noqa: BLE001 — every rank must take the same path below
                if not self.exchange_in_graph:
                    raise
                log("bench: capturing the all-reduces in the step graph failed (%s: %s); falling back to the "
                    "eager all-reduce after each replay" % (type(e).__name__, e))
                failed = 1
            if self.exchange_in_graph:
                flag = torch.tensor([failed], device=self.dev)
                torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX)
                if flag.item():
                    for g in graphs:
                        g.release()
                    torch.cuda.synchronize()
                    self.exchange_in_graph = False
                    if self.reducer is not None:
                        self.reducer.remove()
                    self.reducer = None
                    graphs = self._capture(graph, warmup)
            self.graph_allreduce = "in graph" if self.exchange_in_graph else "eager after replay"
            for g in graphs:
                loss = g.replay()    # one untimed replay of each: every captured step runs once before timing
        else:
            for i in range(warmup):
                loss = self.eager_step(i)
        torch.cuda.synchronize()
        if not torch.isfinite(loss).item():
            raise SystemExit("non-finite loss during warm-up")
        if self.world > 1:
            torch.distributed.barrier()
        prof = not args.no_prof and not graph
        if prof:
            _lib.prof_enable(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            if graphs:
                loss = graphs[i % args.pool].replay()
                if self.world > 1 and not self.exchange_in_graph:
                    self._exchange_and_update()
            else:
                loss = self.eager_step(i)
        torch.cuda.synchronize()
        if self.world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - t0
        if self.world > 1:
            t = torch.tensor([el], device=self.dev, dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        final_loss = float(loss.item())
        for g in graphs:
            g.release()
        del graphs
        eager_ms = None
        if not args.no_prof and graph:
            # kernel timers cannot run inside a graph: an eager pass of the same step, timed per kernel
            if self.reducer is not None:
                self.reducer.remove()
            self.reducer = None
            self.exchange_in_graph = False
            _lib.prof_enable(True)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for i in range(args.prof_steps):
                self.eager_step(i)
            torch.cuda.synchronize()
            eager_ms = (time.perf_counter() - t1) / args.prof_steps * 1e3
            prof = True
        kernels, singles = {}, []
        if prof:
            for name in MATRIX_KERNELS + OTHER_KERNELS:
                c, ms, w = _lib.prof_read(name)
                if c:
                    kernels[name] = {"launches": c, "ms_total": round(ms, 3), "work": w}
            singles = _lib.prof_kernels()
            _lib.prof_enable(False)
        torch.cuda.empty_cache()
        cmd = {"model": self.name, "batch": self.B, "world": self.world, "precision": precision,
               "sync_bn": bool(args.sync_bn), "conv_fwd_fp32": self.conv_fwd_fp32 and precision != "fp32"}
        _lib.set_option("conv_fwd_fp32", 0)
        skipped = self.scaler.overflows() if self.scaler is not None else None
        if self.reducer is not None:
            self.reducer.remove()
            self.reducer = None
        return {"el": el, "steps": steps, "warmup": warmup, "graph": bool(graph), "final_loss": final_loss,
                "exchange_in_graph": bool(graph and self.world > 1 and getattr(self, "graph_allreduce", "") == "in graph"),
                "fp16_skipped_steps": skipped,
                "kernels": kernels, "roofline": roofline(kernels, singles, cmd), "eager_ms": eager_ms,
                "prof_steps": args.prof_steps if (graph and prof) else steps}


def _workload_h2d(self, precision, steps, warmup):
    """The graphed step fed from pinned host memory: 2 device batch slots (graphs 0 / 1 read slot 0 /
    slot 1), host batches uploaded on a copy stream one step ahead.  The upload is the clips' int16 PCM
    (the WAV samples, 32 KB per clip; the feature kernel widens them in its load stage: the same values
    as the float32 items of Dataset).  Returns utt/s over the wall time of `steps` steps (uploads
    included) and the upload rate; plus the bare upload rate (copies only)."""
    assert self.name != "spec_bgru" and self.args.pool >= 2
    from speechrecognitionproject_amd.graphs import GraphedStep
    _lib.set_matmul_precision(precision)
    self.scaler = LossScaler(FP16_LOSS_SCALE, dynamic=False, device=self.dev) if precision == "fp16" else None
    self.opt.grad_scale = 1.0 / self.world
    n_host = 8
    x, _ = synthetic_clips(n_host * self.B, seed=4000 + self.rank)
    host = torch.from_numpy(x.astype(np.int16)).view(n_host, self.B, -1).pin_memory()
    staged, self.pcm = self.pcm, torch.empty((2, self.B, 16000), dtype=torch.int16, device=self.dev)
    # N > 1: the exchange as the main run settled it (in the graph, or eager after each replay)
    self.exchange_in_graph = self.world > 1 and getattr(self, "graph_allreduce", "") == "in graph"
    self.reducer = (parallel.GradReducer(self.flat, bucket_mb=self.args.bucket_mb, capture_group=parallel.capture_group())
                    if self.exchange_in_graph else None)
    graphs = []
    for j in range(2):
        self._slot = j
        graphs.append(GraphedStep(self._graph_body, warmup=max(2, warmup) if j == 0 else 0,
                                  pool=graphs[0].pool() if graphs else None,
                                  capture_error_mode="thread_local" if self.exchange_in_graph else "global"))
    cs = torch.cuda.Stream()
    cur = torch.cuda.current_stream()
    ev_copy = [torch.cuda.Event() for _ in range(2)]
    ev_done = [torch.cuda.Event() for _ in range(2)]
    for e in ev_done:
        e.record(cur)

    nocopy = os.environ.get("SRK_BENCH_H2D_NOCOPY", "0") == "1"   # diagnostic: the same loop without the copies

    def upload(i):
        j = i % 2
        cs.wait_event(ev_done[j])              # the step that last read slot j has finished
        with torch.cuda.stream(cs):
            if not nocopy:
                self.pcm[j].copy_(host[i % n_host], non_blocking=True)
            ev_copy[j].record(cs)

    def run(n, mark=None):
        upload(0)
        for i in range(n):
            j = i % 2
            cur.wait_event(ev_copy[j])
            graphs[j].replay()
            if self.world > 1 and not self.exchange_in_graph:
                self._exchange_and_update()
            ev_done[j].record(cur)
            if mark is not None and i == mark[0]:
                mark[1].record(cur)
            if i + 1 < n:
                upload(i + 1)

    run(4)
    torch.cuda.synchronize()
    # steady state: `skip` steps into an unbroken loop (the first batch's upload, which nothing can hide, and the
    # clock ramp after the synchronize behind), then `steps` steps timed by events on the compute stream; the
    # wall time of the whole loop (start-up included) is reported beside it
    skip = 4
    ev_a, ev_b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    run(skip + steps, mark=(skip - 1, ev_a))
    ev_b.record(cur)
    torch.cuda.synchronize()
    el_all = time.perf_counter() - t0
    el = ev_a.elapsed_time(ev_b) * 1e-3
    # the upload alone, same buffers and stream
    t1 = time.perf_counter()
    for i in range(steps):
        with torch.cuda.stream(cs):
            self.pcm[i % 2].copy_(host[i % n_host], non_blocking=True)
    cs.synchronize()
    el_copy = time.perf_counter() - t1
    for g in graphs:
        g.release()
    if self.reducer is not None:
        self.reducer.remove()
        self.reducer = None
    self.exchange_in_graph = False
    self.pcm = staged
    torch.cuda.empty_cache()
    step_bytes = self.B * 16000 * 2
    return {"value": round(self.B * steps / el, 2), "unit": "utt/s", "ms_per_step": round(el / steps * 1e3, 3),
            "timing": "steady state: %d steps after %d untimed ones of the same unbroken loop, HIP events on the "
                      "compute stream (every upload overlapped with the previous step)" % (steps, skip),
            "value_incl_startup": round(self.B * (skip + steps) / el_all, 2),
            "upload_bytes_per_step": step_bytes, "needed_gbs": round(step_bytes / (el / steps) / 1e9, 2),
            "upload_only_gbs": round(step_bytes * steps / el_copy / 1e9, 2), "steps": steps}


Workload.run_h2d = _workload_h2d


def roofline(kernels, singles, cmd):
    """The dominant matrix-core kernel CATEGORY of the profiled steps (e.g. gemm_f32 = every fp32 GEMM
    launch) — achieved algorithmic TFLOP/s over its launches vs the MFMA peak of its operand type —
    plus the largest SINGLE kernel (one kernel template at one shape) and the top 5 by time."""
    mm = {k: v for k, v in kernels.items() if k in MATRIX_KERNELS}
    if not mm:
        return None
    dom = max(mm, key=lambda k: mm[k]["ms_total"])
    k = mm[dom]
    tf = k["work"] / (k["ms_total"] * 1e-3) / 1e12
    peak = PEAK_LP_MFMA_TFLOPS if dom in LP_KERNELS else PEAK_FP32_MFMA_TFLOPS
    traffic, src = pmc_traffic(dom, cmd)
    # algorithmic HBM bytes of the category's launches (ProfScope::bytes: operands once + the output)
    alg = sum(r.get("bytes", 0.0) for r in singles if r["name"] == dom) / k["launches"]
    res = {"bound": "mfma", "kernel": dom, "achieved": round(tf, 2), "peak": peak,
           "unit": "TFLOP/s", "frac": round(tf / peak, 4),
           "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": src,
           "algorithmic_bytes_per_launch": round(alg) if alg else None,
           "traffic_ratio": round(traffic / alg, 3) if traffic and alg else None,
           "avg_launch_ms": round(k["ms_total"] / k["launches"], 5),
           "flops_per_launch": k["work"] / k["launches"]}
    mat = [r for r in singles if r["name"] in MATRIX_KERNELS and r["work"] > 0]
    if mat:
        big = max(mat, key=lambda r: r["ms_total"])
        btf = big["work"] / (big["ms_total"] * 1e-3) / 1e12
        bpeak = PEAK_LP_MFMA_TFLOPS if big["name"] in LP_KERNELS else PEAK_FP32_MFMA_TFLOPS
        res["largest_kernel"] = {"kernel": big["kernel"], "category": big["name"], "launches": big["launches"],
                                 "avg_launch_ms": round(big["ms_total"] / big["launches"], 5),
                                 "achieved": round(btf, 2), "peak": bpeak, "frac": round(btf / bpeak, 4)}
    res["top_kernels"] = [{"kernel": r["kernel"], "launches": r["launches"], "ms_total": round(r["ms_total"], 3)}
                          for r in sorted(singles, key=lambda r: -r["ms_total"])[:5]]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="clips per GPU per step (default per model)")
    ap.add_argument("--model", default=None, help="default: mfcc_bgru (cfg2) + the other configs under \"configs\"")
    ap.add_argument("--pool", type=int, default=4, help="distinct pre-staged batches per rank")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--precision", default="fp32", choices=sorted(_lib.PRECISIONS),
                    help="matrix-core operand precision (fp32 = the reference's arithmetic; bf16 / fp16 "
                         "operands with fp32 accumulation)")
    ap.add_argument("--no-lowprec", dest="lowprec", action="store_false",
                    help="skip the extra bf16 measurement reported under \"bf16\" on the same line")
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="time eager steps (one host launch per kernel) instead of HIP-graph replays")
    ap.add_argument("--prof-steps", type=int, default=5, help="eager steps of the per-kernel timing pass (graph mode)")
    ap.add_argument("--no-configs", dest="configs", action="store_false",
                    help="skip the cfg3 / cfg4 / cfg5 records of the default run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-h2d", dest="h2d", action="store_false",
                    help="skip the default run's \"h2d\" record (the cfg2 step fed from pinned host memory)")
    ap.add_argument("--no-prof", action="store_true")
    ap.add_argument("--no-feature-roofline", "--no-mfcc-roofline", dest="no_feature_roofline", action="store_true")
    ap.add_argument("--no-overlap", dest="overlap", action="store_false",
                    help="N > 1, eager: one blocking all-reduce after backward instead of bucketed all-reduces "
                         "overlapped with it (parallel.GradReducer)")
    ap.add_argument("--bucket-mb", type=float, default=8.0, help="gradient bucket size of the overlapped all-reduce")
    ap.add_argument("--allreduce-outside-graph", action="store_true",
                    help="N > 1, HIP graphs: replay forward + backward, then one flat all-reduce + Adam eagerly "
                         "(instead of the default: the bucketed all-reduces and Adam captured in the step graph, "
                         "overlapped with the backward, DESIGN.md §4)")
    ap.add_argument("--allreduce-in-graph", action="store_true",
                    help="accepted for compatibility: the captured exchange is the default")
    ap.add_argument("--conv-fwd-fp32", action="store_true",
                    help="16-bit modes: conv forwards on fp32 operands (the faithful 16-bit mode of the BatchNorm "
                         "models, srk option conv_fwd_fp32)")
    ap.add_argument("--sync-bn", action="store_true",
                    help="BatchNorm statistics over the global batch of all ranks (SyncBatchNorm1d; resnet_bgru, "
                         "cnn_bgru, mfrn_bgru)")
    ap.add_argument("--cpu-plumbing", action="store_true",
                    help="exercise the N-rank launch / timing / JSON path over gloo on CPU (no GPU; no measurement)")
    args = ap.parse_args()
    default_run = args.model is None
    args.model = args.model or "mfcc_bgru"
    if args.model not in DEFAULT_BATCH:
        raise SystemExit("unknown --model %s" % args.model)

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
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    B = args.batch or DEFAULT_BATCH[args.model]
    wl = Workload(args, args.model, B, rank, world, dev)
    main_rec = wl.run(args.precision, args.steps, args.warmup, args.graph)
    # the same step with 16-bit matrix-core operands (BASELINE.json cfg2 names bf16), same line
    lp_rec = None
    if args.lowprec and args.precision == "fp32":
        lp_rec = wl.run("bf16", args.steps, args.warmup, args.graph)
        _lib.set_matmul_precision(args.precision)
    h2d_rec = None
    if default_run and args.h2d:
        # SURVEY.md §8d's second figure: the same step fed from pinned host PCM (the reference's
        # DataLoader -> .to(DEVICE) crossing, training.py:77,86), the upload double-buffered
        h2d_rec = {"what": "cfg2 train step (HIP-graph replays) with each batch uploaded from pinned host memory "
                           "(int16 PCM, the WAV samples: K1 widens them to the float32 values Dataset yields) on a "
                           "copy stream, double-buffered: batch i+1 uploads while step i runs; value = clips / wall "
                           "time including every upload"}
        for prec in ("fp32", "bf16"):
            h2d_rec[prec] = wl.run_h2d(prec, args.steps, args.warmup)
        _lib.set_matmul_precision(args.precision)
    del wl
    extras = []
    if default_run and args.configs:
        for tag, name, prec, eb, esteps in EXTRA_CONFIGS:
            w2 = Workload(args, name, eb, rank, world, dev)
            w2.conv_fwd_fp32 = tag.endswith("-faithful")
            rec = w2.run(prec, esteps, 2, args.graph)
            rec.update(tag=tag, name=name, precision=prec, B=eb)
            extras.append(rec)
            del w2
            torch.cuda.empty_cache()
        _lib.set_matmul_precision(args.precision)

    # a persistent kernel that timed out invalidates every number above: fail loudly
    _lib.check_health(sync=True)
    if rank != 0:
        return
    el = main_rec["el"]
    value = world * B * args.steps / el
    kern = lambda ks: {k: {"launches": v["launches"], "ms_total": v["ms_total"]} for k, v in ks.items()}
    res = {
        "metric": "utterances/sec (1 s @16 kHz) MFCC+CNN-BiGRU train step",
        "value": round(value, 2), "unit": "utt/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.precision, "data": "synthetic (SURVEY.md §8d clip mix, pre-staged in HBM)",
        "config": {"workload": "%s, CE, backward, Adam (full training.py step), per-GPU batch %d"
                               % (CFG[args.model], B), "model": args.model,
                   "global_batch": world * B, "clip_samples": 16000, "parallelism": "dp%d" % world,
                   "step_execution": ("HIP graph replay" + (" of the whole step" if world == 1 or main_rec["exchange_in_graph"]
                                                            else " (forward + backward) + eager RCCL all-reduce + Adam")
                                      if args.graph else "eager"),
                   "allreduce": (None if world == 1 else
                                 "bucketed %.0f MB, captured in the step graph, overlapped with backward" % args.bucket_mb
                                 if main_rec["exchange_in_graph"] else
                                 "one flat buffer after backward" if (args.graph or not args.overlap)
                                 else "bucketed %.0f MB, overlapped with backward" % args.bucket_mb),
                   "sync_bn": bool(args.sync_bn)},
        "model_tflops": round(value * TRAIN_GFLOP_PER_UTT.get(args.model, 0) / 1e3, 2),
        "final_loss": round(main_rec["final_loss"], 5),
        "roofline": main_rec["roofline"],
        "kernels": kern(main_rec["kernels"]),
        "kernel_timing": ("eager pass of the same step, %d steps, HIP events on the launch stream; eager %.3f ms/step"
                          % (main_rec["prof_steps"], main_rec["eager_ms"])) if main_rec["eager_ms"] else
                         "the timed steps, HIP events on the launch stream",
    }
    if lp_rec is not None:
        res["bf16"] = {"dtype": "bf16", "value": round(world * B * args.steps / lp_rec["el"], 2),
                       "ms_per_step": round(lp_rec["el"] / args.steps * 1e3, 3),
                       "eager_ms_per_step": round(lp_rec["eager_ms"], 3) if lp_rec["eager_ms"] else None,
                       "final_loss": round(lp_rec["final_loss"], 5), "roofline": lp_rec["roofline"],
                       "kernels": kern(lp_rec["kernels"])}
    if main_rec["fp16_skipped_steps"] is not None:
        res["loss_scale"] = {"kind": "static", "scale": FP16_LOSS_SCALE, "skipped_steps": main_rec["fp16_skipped_steps"]}
    if main_rec["eager_ms"]:
        res["eager_ms_per_step"] = round(main_rec["eager_ms"], 3)
    if extras:
        res["configs"] = [{"config": r["tag"], "workload": CFG[r["name"]], "model": r["name"], "dtype": r["precision"],
                           "per_gpu_batch": r["B"], "global_batch": world * r["B"], "steps": r["steps"],
                           "value": round(world * r["B"] * r["steps"] / r["el"], 2), "unit": "utt/s",
                           "ms_per_step": round(r["el"] / r["steps"] * 1e3, 3),
                           "eager_ms_per_step": round(r["eager_ms"], 3) if r["eager_ms"] else None,
                           "final_loss": round(r["final_loss"], 5), "roofline": r["roofline"],
                           **({"gradients": GRADIENTS[r["tag"]]} if r["tag"] in GRADIENTS else {}),
                           **({"loss_scale": {"kind": "static", "scale": FP16_LOSS_SCALE,
                                              "skipped_steps": r["fp16_skipped_steps"]}}
                              if r["fp16_skipped_steps"] is not None else {})} for r in extras]
    if not args.no_feature_roofline and args.model in FEATURE:
        log("bench: feature roofline")
        res["feature_roofline"] = feature_roofline(args.model)
        if default_run:   # K2 / K3 (the fbank and spectrogram configs' feature kernels) on the same line
            res["feature_roofline_other"] = [feature_roofline(kernel=k) for k in ("fbank", "spec")]
    if h2d_rec is not None:
        res["h2d"] = h2d_rec
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.model, B, args.cpu_seconds)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
