"""The reference's ``training.py`` entry point (training.py:29-117), on the MI355X path.

    python training.py -key K -lr LR                               # reference CLI
    python training.py --model mfcc_bgru --synthetic 4096 --epochs 1 --batch-size 256
    python -m torch.distributed.run --nproc-per-node 8 training.py --synthetic 65536 ...

Same loop: Adam(lr) + CrossEntropyLoss, ExponentialLR(0.87) stepped once per epoch after epoch 5,
one ``str(loss)`` line per step appended to ``loss_<KEY>.txt``, per-epoch validation / training
accuracy lines via the plugin's ``accuracy`` (``val_<KEY>.txt``, ``train_<KEY>.txt``) and
``resample_unknown_class`` after each epoch.  Additions (all optional): ``--model`` selects the
plugin instead of editing an import line (training.py:39-46), ``--synthetic N`` trains on
synthetic clips when no Kaggle tree is available, ``--data-path/--output-path`` replace the
hard-coded paths (:21-24), ``--log-every`` batches loss lines to avoid a host sync per step,
``--loader device`` (default for WAV trees) replaces the per-item DataLoader with native batched
decode + one on-device augmentation launch per batch, and torchrun environments train
data-parallel (one process per GPU, RCCL all-reduce).  Full-size batches after the first two run as
replays of a HIP graph of the step (the batch is copied into the graph's static input first; a short
last batch runs eagerly; ``--no-graph`` disables it; data-parallel over RCCL the bucketed all-reduces
are captured in the graph too, DESIGN.md §4, with an eager fallback every rank agrees on if the
capture fails) — the same kernels in the
same order, so for models without dropout the same arithmetic bit for bit
(tests/test_graphs_gpu.py, tests/test_training_gpu.py); with dropout a replay draws its mask from
the device counter on top of the last eager seed, so masks (not the arithmetic) differ from
``--no-graph``.  ``--precision bf16|fp16`` runs the matrix cores on 16-bit operands (fp32
accumulation, fp32 parameters); fp16 trains with a loss scale (``--loss-scale``: dynamic by
default, or a fixed number) and skips any step whose gradients overflowed (optim.LossScaler).
"""
import argparse
import importlib
import os
import time

import torch
from torch.utils.data import DataLoader

from . import parallel
from . import _lib
from ._lib import check_health
from .nn import CrossEntropyLoss
from .optim import Adam, FlatParams, LossScaler

PLUGINS = ("mfcc_bgru", "fbanks_cnn", "spec_bgru", "resnet_bgru", "mfrn_bgru", "cnn_bgru", "spec_cnn")


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('-key', '--filekey', type=str, help='key for multiple trainings')
    p.add_argument('-lr', '--learning_rate', type=float, help='LEARNING_RATE')
    p.add_argument('--model', default='mfcc_bgru', choices=PLUGINS)
    p.add_argument('--data-path', default=None, help="parent of 'audio' and the *_list.txt files")
    p.add_argument('--output-path', default='.')
    p.add_argument('--epochs', type=int, default=1)
    p.add_argument('--batch-size', type=int, default=2)
    p.add_argument('--synthetic', type=int, default=0, help='train on N synthetic clips instead of WAV files')
    p.add_argument('--reduce', type=int, default=0, help='reduce_dataset(n) like training.py:66-67')
    p.add_argument('--log-every', type=int, default=1, help='write buffered loss lines every n steps')
    p.add_argument('--no-eval', action='store_true')
    p.add_argument('--mode', type=int, default=None,
                   help="Network(mode=...) for plugins that take it (resnet_bgru: 1 = the staged training's backend head)")
    p.add_argument('--sync-bn', action='store_true',
                   help='data-parallel: BatchNorm statistics over the global batch (SyncBatchNorm1d)')
    p.add_argument('--no-overlap', dest='overlap', action='store_false',
                   help='data-parallel: one all-reduce after backward instead of overlapped buckets')
    p.add_argument('--no-graph', dest='graph', action='store_false',
                   help='run every step eagerly instead of replaying a HIP graph of the step for full-size '
                        'batches (speechrecognitionproject_amd/graphs.py; single process)')
    p.add_argument('--no-dp-graph', dest='dp_graph', action='store_false',
                   help='data-parallel over RCCL: run every step eagerly instead of replaying HIP graphs of the '
                        'whole step with the bucketed all-reduces captured in them (DESIGN.md §4)')
    p.add_argument('--dp-graph', dest='dp_graph', action='store_true', help=argparse.SUPPRESS)
    p.add_argument('--loader', choices=('device', 'torch'), default='device',
                   help='WAV datasets: device = native batched decode + K10 on-device augmentation '
                        '(DeviceBatchLoader); torch = per-item Dataset.__getitem__ through DataLoader')
    p.add_argument('--precision', choices=('fp32', 'bf16', 'fp16'), default='fp32',
                   help='matrix-core operand precision (fp32 = the reference arithmetic; bf16 / fp16 operands with '
                        'fp32 accumulation)')
    p.add_argument('--conv-fwd-fp32', action='store_true',
                   help='16-bit precisions: convolution forwards on fp32 operands, their gradients on 16-bit ones '
                        '(the faithful 16-bit mode of the BatchNorm models: resnet_bgru gradients <= 2e-2 of float64 '
                        'instead of 4-39 %%, DESIGN.md)')
    p.add_argument('--loss-scale', default='dynamic',
                   help="fp16: 'dynamic' (start at 1024, halve on overflow, double after 2000 clean steps) or a "
                        "fixed scale; a step whose gradients are inf / NaN is skipped either way")
    p.add_argument('--save-model', action='store_true',
                   help="write model.state_dict() to OUTPUT/models/model_KEY.ckpt after training (the reference's "
                        "checkpoint path, training.py:104-107)")
    return p.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    saved = _lib.matmul_precision()
    try:
        _train(args)
    finally:
        _lib.set_matmul_precision(saved)      # process-wide: give the caller back its own mode
        _lib.set_option("conv_fwd_fp32", 0)


def _train(args):
    rank, world, local = parallel.init_from_env()
    key = args.filekey or ''
    lr = args.learning_rate if args.learning_rate is not None else 0.0001
    mod = importlib.import_module('speechrecognitionproject_amd.models.model_' + args.model)
    start = time.time()
    device = torch.device('cuda', local)
    _lib.set_matmul_precision(args.precision)
    _lib.set_option("conv_fwd_fp32", 1 if args.conv_fwd_fp32 else 0)

    if args.synthetic:
        from .dataset import SyntheticDataset
        data = SyntheticDataset(args.synthetic, seed=0)
        valset = SyntheticDataset(max(args.synthetic // 10, args.batch_size), seed=1)
    else:
        from .dataset import Dataset
        if not args.data_path:
            raise SystemExit("--data-path (Kaggle layout) or --synthetic N is required")
        data = Dataset(args.data_path + '/training_list.txt', args.data_path + '/audio')
        valset = Dataset(args.data_path + '/validation_list.txt', args.data_path + '/audio')
        if args.reduce:
            data.reduce_dataset(args.reduce)
            valset.reduce_dataset(args.reduce)

    torch.manual_seed(0)
    model = (mod.Network() if args.mode is None else mod.Network(mode=args.mode)).to(device)
    if args.sync_bn:
        from .nn import convert_sync_batchnorm
        model = convert_sync_batchnorm(model)
    flat = FlatParams(model.parameters())
    optimizer = Adam(model.parameters(), lr=lr, flat=flat)
    optimizer.grad_scale = 1.0 / world
    parallel.broadcast_flat(flat)
    # data-parallel steps are captured whole (the bucketed collectives included, on the capture-only
    # process group) over RCCL; gloo cannot be captured, and --no-dp-graph runs them eagerly
    use_graph = args.graph and (world == 1 or (args.dp_graph and torch.distributed.get_backend() == 'nccl'))
    # the capture-only group exists before any capture, for the bucketed reducer, the single flat
    # all-reduce of --no-overlap and SyncBatchNorm's statistics alike (parallel.group_for_now)
    cap_group = parallel.capture_group() if (use_graph and world > 1) else None
    reducer = parallel.GradReducer(flat, capture_group=cap_group) if (world > 1 and args.overlap) else None
    scheduler = torch.optim.lr_scheduler.ExponentialLR(optimizer, 0.87)
    criterion = CrossEntropyLoss()
    scaler = None
    if args.precision == 'fp16':
        if args.loss_scale == 'dynamic':
            scaler = LossScaler(1024.0, dynamic=True, device=device)
        else:
            scaler = LossScaler(float(args.loss_scale), dynamic=False, device=device)
    os.makedirs(args.output_path, exist_ok=True)
    loss_file = os.path.join(args.output_path, 'loss_' + key + '.txt')

    graphed = None          # GraphedStep of a full-batch step (captured after two eager full steps)
    static = {}
    full_eager = 0
    captures = 0
    side = None

    def eager_step(x, y):
        optimizer.zero_grad()
        if reducer is not None:
            reducer.begin()
        outputs = model(x)
        loss = criterion(outputs, y)
        (scaler.scale(loss) if scaler is not None else loss).backward()
        if reducer is not None:
            reducer.finish()
        else:
            parallel.allreduce_grads(flat)
        optimizer.step(scaler=scaler)
        return loss

    def graph_body():
        return eager_step(static['x'], static['y'])

    epoch = 0
    while epoch < args.epochs:
        if epoch > 4:
            scheduler.step()
            optimizer.sync_lr()     # a replayed step reads lr from the device
        sampler = None
        if world > 1:
            idx = parallel.shard_indices(len(data), rank, world, seed=0, epoch=epoch)
            sampler = torch.utils.data.SubsetRandomSampler(idx.tolist())
        if not args.synthetic and args.loader == 'device':
            from .dataset import DeviceBatchLoader
            loader = DeviceBatchLoader(data, batch_size=args.batch_size, shuffle=sampler is None, sampler=sampler,
                                       seed=rank)
        elif sampler is not None:
            loader = DataLoader(data, batch_size=args.batch_size, sampler=sampler, drop_last=False)
        else:
            loader = DataLoader(data, batch_size=args.batch_size, shuffle=True, drop_last=False)
        pending = []

        def flush():
            # every rank drains its buffered losses (and fails loudly on a persistent-kernel
            # timeout); only rank 0 writes the reference's loss file (training.py:94-95)
            nonlocal pending
            vals = torch.stack(pending).tolist() if pending else []
            check_health(sync=True)
            if rank == 0 and vals:
                with open(loss_file, 'a') as f:
                    for v in vals:
                        f.write(str(v) + '\n')
            pending = []

        for batch in loader:
            x, y = batch['audio'], batch['label'].to(device)
            full = x.shape[0] == args.batch_size
            if use_graph and full:
                if not static:
                    static['x'] = torch.empty(x.shape, dtype=torch.float32, device=device)
                    static['y'] = torch.empty(y.shape, dtype=y.dtype, device=device)
                if graphed is not None and not graphed.valid():
                    graphed, full_eager = None, 0      # a scratch buffer moved: warm up and capture again
                if graphed is None and full_eager < 2:
                    # the warm-up: real steps on real batches, on a side stream as a capture requires
                    if side is None:
                        side = torch.cuda.Stream()
                    side.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(side):
                        static['x'].copy_(x, non_blocking=True)
                        static['y'].copy_(y, non_blocking=True)
                        loss = graph_body()
                    torch.cuda.current_stream().wait_stream(side)
                    full_eager += 1
                else:
                    if graphed is None:
                        from .graphs import GraphedStep
                        # the last warm-up loss still holds its step's autograd graph (and with it the
                        # side stream's AccumulateGrad nodes): drop it before the capture
                        loss = None
                        failed = 0
                        try:   # warmed up by the side-stream steps
                            graphed = GraphedStep(graph_body, warmup=0,
                                                  capture_error_mode='thread_local' if world > 1 else 'global')
                        except Exception as e:   # noqa: BLE001 — a DP capture failure: every rank falls back
                            if world == 1 or captures:
                                raise
                            print('training: capturing the data-parallel step failed (%s: %s); running eagerly'
                                  % (type(e).__name__, e), flush=True)
                            failed = 1
                        if world > 1 and not captures:
                            # the first capture happens at the same batch on every rank: agree on the
                            # outcome (a later re-capture is rank-local — rank 0's evaluation can move a
                            # scratch buffer — and its collectives are captured, not run, so no exchange)
                            flag = torch.tensor([failed], device=device)
                            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX)
                            if flag.item():
                                graphed, use_graph = None, False
                        captures += 1
                    if graphed is None:   # the DP capture fell back: this batch eagerly
                        loss = eager_step(x, y)
                        pending.append(loss.detach())
                        if len(pending) >= args.log_every:
                            flush()
                        continue
                    static['x'].copy_(x, non_blocking=True)
                    static['y'].copy_(y, non_blocking=True)
                    loss = graphed.replay()
            else:
                loss = eager_step(x, y)
            pending.append(loss.detach().clone() if graphed is not None and loss is graphed.out else loss.detach())
            if len(pending) >= args.log_every:
                flush()
        flush()
        if not args.no_eval and rank == 0:
            mod.accuracy(model, valset, os.path.join(args.output_path, 'val_' + key + '.txt'), 4)
            mod.accuracy(model, data, os.path.join(args.output_path, 'train_' + key + '.txt'), 4)
            check_health(sync=True)
        if world > 1:
            parallel.barrier()    # the other ranks wait here (long timeout), not inside a collective
        epoch += 1
        if hasattr(data, 'resample_unknown_class'):
            data.resample_unknown_class()
    if args.save_model and rank == 0:
        os.makedirs(os.path.join(args.output_path, 'models'), exist_ok=True)
        torch.save(model.state_dict(), os.path.join(args.output_path, 'models', 'model_' + key + '.ckpt'))
    if scaler is not None and rank == 0:
        print('fp16 steps skipped (inf/NaN gradients): %d, final loss scale %g' % (scaler.overflows(), scaler.get_scale()))
    if rank == 0:
        print('key  ', key)
        print('time  ', time.time() - start)
        print('epochs  ', epoch)


if __name__ == '__main__':
    main()
