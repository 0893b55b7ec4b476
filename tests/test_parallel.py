"""Data-parallel plumbing (speechrecognitionproject_amd/parallel.py).

CPU (gloo, world_size 2): the flat-buffer all-reduce / broadcast and the sharding, and the DP
equivalence of the training step math on the CPU oracle (two ranks on half batches + summed
gradients / world == one rank on the full batch).
GPU (gloo over one device, world_size 2): the same equivalence through the HIP kernels.
"""
import os
import socket
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from speechrecognitionproject_amd import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker_plumbing(rank, world, port, q):
    _init(rank, world, port)
    try:
        flat = types.SimpleNamespace(data=torch.full((10,), float(rank + 1)), grad=torch.full((10,), float(rank + 1)))
        parallel.broadcast_flat(flat)
        parallel.allreduce_grads(flat)
        idx = parallel.shard_indices(11, rank, world, seed=3)
        q.put((rank, flat.data.tolist(), flat.grad.tolist(), idx.tolist()))
    finally:
        dist.destroy_process_group()


def test_flat_allreduce_broadcast_and_shards():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_plumbing, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for rank, data, grad, idx in res:
        assert data == [1.0] * 10                  # rank 0's parameters everywhere
        assert grad == [3.0] * 10                  # 1 + 2
    shards = [set(r[3]) for r in res]
    assert len(res[0][3]) == len(res[1][3]) == 6   # padded to equal length
    assert shards[0] | shards[1] == set(range(11))


def _worker_oracle_step(rank, world, port, q):
    _init(rank, world, port)
    try:
        from oracle import models as OM
        from speechrecognitionproject_amd.synthetic import synthetic_clips
        torch.manual_seed(0)
        net = OM.MfccBGRU(num_features=128)
        x, y = synthetic_clips(4, seed=9)
        xs, ys = torch.from_numpy(x[rank::world]), torch.from_numpy(y[rank::world])
        out = net(xs)
        loss = torch.nn.CrossEntropyLoss()(out, ys)
        loss.backward()
        g = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
        flat = types.SimpleNamespace(data=None, grad=g)
        parallel.allreduce_grads(flat)
        q.put((rank, (flat.grad / world).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
def test_dp_equivalence_cpu_oracle():
    from oracle import models as OM
    from speechrecognitionproject_amd.synthetic import synthetic_clips
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_oracle_step, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    torch.manual_seed(0)
    net = OM.MfccBGRU(num_features=128)
    x, y = synthetic_clips(4, seed=9)
    order = list(range(0, 4, 2)) + list(range(1, 4, 2))   # same clips, any order: CE is a mean
    loss = torch.nn.CrossEntropyLoss()(net(torch.from_numpy(x[order])), torch.from_numpy(y[order]))
    loss.backward()
    full = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
    for r in range(world):
        assert torch.allclose(torch.tensor(res[r]), full, atol=1e-6, rtol=1e-4)


def _worker_gpu_step(rank, world, port, q):
    _init(rank, world, port)
    try:
        from oracle import models as OM
        from speechrecognitionproject_amd import nn as snn
        from speechrecognitionproject_amd.models import model_mfcc_bgru
        from speechrecognitionproject_amd.optim import Adam, FlatParams
        from speechrecognitionproject_amd.synthetic import synthetic_clips
        torch.cuda.set_device(0)
        net = model_mfcc_bgru.Network().cuda()
        net.load_state_dict(OM.seeded_state_dict(OM.MfccBGRU(), 0))
        flat = FlatParams(net.parameters())
        opt = Adam(net.parameters(), lr=1e-4, flat=flat)
        opt.grad_scale = 1.0 / world
        parallel.broadcast_flat(flat)
        x, y = synthetic_clips(8, seed=9)
        opt.zero_grad()
        loss = snn.CrossEntropyLoss()(net(torch.from_numpy(x[rank::world])), torch.from_numpy(y[rank::world]).cuda())
        loss.backward()
        parallel.allreduce_grads(flat)      # gloo all-reduce of the device buffer
        opt.step()
        torch.cuda.synchronize()
        q.put((rank, flat.data.cpu()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_dp_equivalence_gpu_kernels(gpu):
    from oracle import models as OM
    from speechrecognitionproject_amd import nn as snn
    from speechrecognitionproject_amd.models import model_mfcc_bgru
    from speechrecognitionproject_amd.optim import Adam, FlatParams
    from speechrecognitionproject_amd.synthetic import synthetic_clips
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_gpu_step, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert torch.equal(res[0], res[1])                 # replicas stay identical
    net = model_mfcc_bgru.Network().cuda()
    net.load_state_dict(OM.seeded_state_dict(OM.MfccBGRU(), 0))
    flat = FlatParams(net.parameters())
    opt = Adam(net.parameters(), lr=1e-4, flat=flat)
    x, y = synthetic_clips(8, seed=9)
    order = list(range(0, 8, 2)) + list(range(1, 8, 2))
    opt.zero_grad()
    snn.CrossEntropyLoss()(net(torch.from_numpy(x[order])), torch.from_numpy(y[order]).cuda()).backward()
    opt.step()
    # one Adam step moves each weight by ~lr*sign(g); ranks' summed grads differ from the full
    # batch only by fp32 summation order
    diff = (res[0] - flat.data.cpu()).abs()
    assert (diff <= 2e-6).float().mean().item() >= 0.999


def test_bench_relaunches_itself_for_gpus_n():
    """`python bench.py --gpus 2` (no WORLD_SIZE) starts 2 ranks through torch.distributed.run and
    rank 0 prints one JSON line with n_gpus == 2 (CPU: --cpu-plumbing, gloo, no GPU work)."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--cpu-plumbing"], capture_output=True, text=True, timeout=300, env=env, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["config"]["parallelism"] == "dp2"


def test_bench_rejects_world_size_mismatch():
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--cpu-plumbing"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=repo)
    assert r.returncode != 0 and "process group has 1 ranks" in r.stderr


def _worker_syncbn(rank, world, port, q):
    _init(rank, world, port)
    try:
        from speechrecognitionproject_amd import nn as snn
        torch.cuda.set_device(0)
        g = torch.Generator().manual_seed(5)
        N, L, C = 6, 37, 64
        x = torch.randn(N, L, C, generator=g) * 3 + 2
        r = torch.randn(N, L, C, generator=g)
        dy = torch.randn(N, L, C, generator=g)
        sl = slice(rank * N // world, (rank + 1) * N // world)
        bn = snn.convert_sync_batchnorm(snn.BatchNorm1d(C)).cuda()
        assert isinstance(bn, snn.SyncBatchNorm1d)
        with torch.no_grad():
            bn.weight.copy_(torch.linspace(0.5, 1.5, C))
            bn.bias.copy_(torch.linspace(-0.3, 0.3, C))
        xm = x[sl].cuda().requires_grad_(True)
        rm = r[sl].cuda().requires_grad_(True)
        y = bn(xm, residual=rm, relu=True)
        (y * dy[sl].cuda()).sum().backward()
        torch.cuda.synchronize()
        q.put((rank, y.detach().cpu(), xm.grad.cpu(), rm.grad.cpu(), bn.weight.grad.cpu(), bn.bias.grad.cpu(),
               bn.running_mean.cpu(), bn.running_var.cpu()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sync_batchnorm_matches_global_batch(gpu):
    """SyncBatchNorm1d on 2 ranks x 3 clips == torch BatchNorm1d on the 6-clip batch (float64):
    outputs, input / residual gradients, summed dgamma / dbeta, running statistics
    (model_resnet_bgru.py:20,23,49 under data parallelism)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_syncbn, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((v[0], v[1:]) for v in (q.get(timeout=300) for _ in range(world)))
    for p in ps:
        p.join(timeout=60)
    g = torch.Generator().manual_seed(5)
    N, L, C = 6, 37, 64
    x = torch.randn(N, L, C, generator=g) * 3 + 2
    r = torch.randn(N, L, C, generator=g)
    dy = torch.randn(N, L, C, generator=g)
    ref = torch.nn.BatchNorm1d(C).double()
    with torch.no_grad():
        ref.weight.copy_(torch.linspace(0.5, 1.5, C))
        ref.bias.copy_(torch.linspace(-0.3, 0.3, C))
    xr = x.double().permute(0, 2, 1).requires_grad_(True)
    rr = r.double().permute(0, 2, 1).requires_grad_(True)
    yr = torch.relu(ref(xr) + rr)
    (yr * dy.double().permute(0, 2, 1)).sum().backward()
    y = torch.cat([res[0][0], res[1][0]]).double()
    dx = torch.cat([res[0][1], res[1][1]]).double()
    dr = torch.cat([res[0][2], res[1][2]]).double()
    close = lambda a, b, tol: (a - b).abs().max().item() <= tol * max(1.0, b.abs().max().item())
    assert close(y, yr.detach().permute(0, 2, 1), 1e-5)
    assert close(dx, xr.grad.permute(0, 2, 1), 1e-4)
    assert close(dr, rr.grad.permute(0, 2, 1), 1e-6)
    assert close(res[0][3].double() + res[1][3].double(), ref.weight.grad, 1e-4)
    assert close(res[0][4].double() + res[1][4].double(), ref.bias.grad, 1e-5)
    for k in (0, 1):   # identical statistics on both ranks
        assert close(res[k][5].double(), ref.running_mean, 1e-5) and close(res[k][6].double(), ref.running_var, 1e-5)


def _worker_reducer(rank, world, port, q):
    _init(rank, world, port)
    try:
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(40, 300), torch.nn.Tanh(), torch.nn.Linear(300, 200),
                                  torch.nn.Tanh(), torch.nn.Linear(200, 12))
        params = list(net.parameters())
        offs, n = [], 0
        for p in params:
            offs.append(n)
            n += (p.numel() + 63) // 64 * 64
        flat = types.SimpleNamespace(params=params, offsets=offs, numel=n, grad=torch.zeros(n))
        for p, o in zip(params, offs):
            p.grad = flat.grad[o:o + p.numel()].view_as(p)
        red = parallel.GradReducer(flat, bucket_mb=0.005)   # 1.3k floats: 3 buckets
        assert len(red.buckets) >= 3
        assert red.buckets[0][1] == n and red.buckets[-1][0] == 0
        assert all(red.buckets[i][0] == red.buckets[i + 1][1] for i in range(len(red.buckets) - 1))
        g = torch.Generator().manual_seed(10 + rank)
        x = torch.randn(16, 40, generator=g)
        red.begin()
        red.persistent_pending(1)                           # hold every bucket until "done"
        net(x).square().mean().backward()
        held = len(red.held)
        launched_before = len(red.works)
        red.persistent_done()
        launched_after = len(red.works)
        red.finish()
        mine = flat.grad.clone()
        # reference: this rank's gradient, summed over ranks in one plain all-reduce
        for p in params:
            p.grad = None
        net(x).square().mean().backward()
        ref = torch.cat([p.grad.reshape(-1) for p in params])
        dist.all_reduce(ref)
        got = torch.cat([mine[o:o + p.numel()] for p, o in zip(params, offs)])
        q.put((rank, held, launched_before, launched_after, float((got - ref).abs().max()), len(red.buckets)))
    finally:
        dist.destroy_process_group()


def test_grad_reducer_buckets_hold_and_sum():
    """parallel.GradReducer: contiguous buckets covering the flat buffer, launched by autograd's
    post-accumulate hooks, held while a persistent kernel is pending, and the summed result equals
    one plain all-reduce (gloo, world 2)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_reducer, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for rank, held, before, after, err, nb in res:
        assert held == nb and before == 0 and after == nb, (held, before, after, nb)
        assert err <= 1e-6


def _worker_gpu_resnet_syncbn(rank, world, port, q, mode):
    _init(rank, world, port)
    try:
        _resnet_syncbn_body(rank, world, q, mode)
    except BaseException as ex:   # report, do not leave the parent waiting on the queue
        import traceback
        q.put((rank, "error", traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def _resnet_syncbn_body(rank, world, q, mode):
    from oracle import models as OM
    from speechrecognitionproject_amd import nn as snn
    from speechrecognitionproject_amd.models import model_resnet_bgru
    from speechrecognitionproject_amd.optim import Adam, FlatParams
    from speechrecognitionproject_amd.synthetic import synthetic_clips
    torch.cuda.set_device(0)
    net = model_resnet_bgru.Network(mode=mode).cuda()
    net.load_state_dict(OM.seeded_state_dict(OM.ResnetBGRU(mode=mode), 0))
    net = snn.convert_sync_batchnorm(net)
    flat = FlatParams(net.parameters())
    opt = Adam(net.parameters(), lr=1e-4, flat=flat)
    opt.grad_scale = 1.0 / world
    parallel.broadcast_flat(flat)
    red = parallel.GradReducer(flat, bucket_mb=4.0)
    x, y = synthetic_clips(4, seed=21)
    opt.zero_grad()
    red.begin()
    loss = snn.CrossEntropyLoss()(net(torch.from_numpy(x[rank::world])), torch.from_numpy(y[rank::world]).cuda())
    loss.backward()
    launched_in_backward = len(red.works)
    red.finish()
    grad = flat.grad.cpu() / world
    opt.step()
    torch.cuda.synchronize()
    from speechrecognitionproject_amd import _lib
    _lib.check_health(sync=True)
    # numpy by value: torch CPU tensors would travel as shared-memory fds that this process takes
    # down with it when it exits before the parent has received them
    bufs = {n: b.cpu().numpy() for n, b in net.named_buffers()}
    q.put((rank, flat.data.cpu().numpy(), grad.numpy(), bufs, launched_in_backward, len(red.buckets)))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_dp_syncbn_overlap_matches_global_batch(gpu, mode):
    """resnet_bgru (BatchNorm in training mode) on 2 ranks x 2 clips with SyncBatchNorm1d and the
    bucketed all-reduce overlapped with backward == one process on the 4-clip batch
    (model_resnet_bgru.py:20,23,49): every gradient tensor norm-wise (<= 1e-3 in mode 0, 1e-2 in mode 1, or 3 x the reference's own
    fp32-vs-fp64 error on that tensor where BatchNorm over 4 clips makes that larger — see below; plus
    a gross element-wise bound), every parameter after one Adam step (<= 2e-6 wherever the gradient's
    sign is certain, |g| > 2 x the tensor's largest DP-vs-single difference; Adam's own 2 lr bound
    elsewhere) and every BatchNorm running
    statistic (<= 1e-5).  mode 1 runs the backend head's 250 / 125-channel BatchNorms on zero-padded
    float4 channel groups (model_resnet_bgru.py:57-71): their statistics must span the ranks too."""
    from oracle import models as OM
    from speechrecognitionproject_amd import nn as snn
    from speechrecognitionproject_amd.models import model_resnet_bgru
    from speechrecognitionproject_amd.optim import Adam, FlatParams
    from speechrecognitionproject_amd.synthetic import synthetic_clips
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker_gpu_resnet_syncbn, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((v[0], v[1:]) for v in (q.get(timeout=100) for _ in range(world)))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert not (len(res[r]) == 2 and isinstance(res[r][0], str) and res[r][0] == "error"), res[r][1]
        res[r] = (torch.from_numpy(res[r][0]), torch.from_numpy(res[r][1]),
                  {n: torch.from_numpy(b) for n, b in res[r][2].items()}) + tuple(res[r][3:])
    assert torch.equal(res[0][0], res[1][0])                 # replicas identical
    assert res[0][3] > 0 and res[0][4] > 1                  # buckets went out during backward
    net = model_resnet_bgru.Network(mode=mode).cuda()
    net.load_state_dict(OM.seeded_state_dict(OM.ResnetBGRU(mode=mode), 0))
    flat = FlatParams(net.parameters())
    opt = Adam(net.parameters(), lr=1e-4, flat=flat)
    x, y = synthetic_clips(4, seed=21)
    order = [0, 2, 1, 3]
    opt.zero_grad()
    snn.CrossEntropyLoss()(net(torch.from_numpy(x[order])), torch.from_numpy(y[order]).cuda()).backward()
    grad = flat.grad.cpu().clone()
    p0 = flat.data.cpu().clone()
    opt.step()
    p1 = flat.data.cpu()
    # The fp32 noise floor of these gradients, measured: the oracle's own float32 step vs its float64
    # step on the same 4 clips.  Training-mode BatchNorm over 4 clips (mode 1's BatchNorm1d(125)
    # normalizes each channel over 4 values) turns rounding into up to 3.5e-3 norm-wise / several %
    # element-wise error in the reference's OWN fp32 gradients; DP vs single process is held to
    # max(1e-3 norm-wise / 1e-2 element-wise, 3 x that floor) per tensor.  The statistics themselves
    # are checked at 1e-5 below, which a rank-local (unsynchronized) BatchNorm would miss by O(1).
    floor = {}
    for dt in (torch.float32, torch.float64):
        om = OM.ResnetBGRU(mode=mode)
        om.load_state_dict(OM.seeded_state_dict(OM.ResnetBGRU(mode=mode), 0))
        om = om.to(dt).train()
        xo = torch.from_numpy(x[order]).to(dt).unsqueeze(1)
        oo = om.resnet(xo) if mode == 1 else om.gru(om.resnet(xo))
        torch.nn.CrossEntropyLoss()(oo, torch.from_numpy(y[order])).backward()
        floor[dt] = {n: p.grad.double() for n, p in om.named_parameters() if p.grad is not None}
    ntol = 1e-3 if mode == 0 else 1e-2   # mode 1: measured 4e-3 (layer4.0.downsample.1) with a 3.5e-3 floor
    pname = {id(p): n for n, p in net.named_parameters()}
    for p, o in zip(flat.params, flat.offsets):
        n = pname[id(p)]
        sl = slice(o, o + p.numel())
        g1, g2 = grad[sl], res[0][1][sl]
        gmax = g1.abs().max().item()
        dg = (g2 - g1).abs()
        # norm-wise, and element-wise for all but a few elements: the stem conv's weight gradient sums
        # raw-PCM x dy terms (|x| up to 32767) under a training-mode BatchNorm — a cancellation whose
        # fp32 value depends on the summation order (measured 3e-4 of its largest element between
        # the 2 x 2 and the 4-clip orders) — and a ReLU input within rounding of 0 may fall on either
        # side and route one x * dy term or not (up to 3.6 % of the tensor's largest on a few layer2.0.conv1
        # elements in mode 1)
        fl = (floor[torch.float32][n] - floor[torch.float64][n]) if n in floor[torch.float64] else torch.zeros(1)
        assert dg.norm().item() <= max(ntol * g1.norm().item(), 3.0 * fl.norm().item()) + 1e-9, (n, dg.norm().item())
        # element-wise only a gross-error bound: one ReLU decision that flips at a position moves a whole
        # row of a 1x1 / k=15 conv's weight gradient (measured up to 3.6 % of the largest element, on
        # 139 elements of layer4.0.downsample in mode 1); a wrong sign or scale would exceed it
        assert dg.max().item() <= 0.2 * gmax + 3.0 * fl.abs().max().item() + 1e-9, (n, dg.max().item(), gmax)
        d = (res[0][0][sl] - p1[sl]).abs()
        # no sign flip possible, and |g| >> Adam's eps (1e-8), where its first step is lr * sign(g): at |g| ~ 1e-7 a
        # 2e-8 gradient difference alone moves lr g / (|g| + eps) by 2e-6 (r05h: layer3.1.conv2, g 8.9e-8 vs 7.2e-8)
        sure = g1.abs() > torch.clamp(2.0 * dg.max(), min=1e-6)
        if sure.any():
            k = int(torch.argmax(torch.where(sure, d, torch.zeros_like(d))))
            assert d[sure].max().item() <= 2e-6, (n, d[k].item(), g1[k].item(), g2[k].item(), dg.max().item())
        assert d.max().item() <= 2e-4 + 1e-6, n
        assert (p1[sl] - p0[sl]).abs().max().item() <= 1e-4 * 1.001 + 1e-7, n   # Adam's first step
    mine = {n: b.cpu() for n, b in net.named_buffers()}
    nstat = 0
    for n, b in mine.items():
        if n.endswith("running_mean") or n.endswith("running_var"):
            scale = max(1.0, b.abs().max().item())
            assert (res[0][2][n] - b).abs().max().item() <= 1e-5 * scale, n
            nstat += 1
        elif n.endswith("num_batches_tracked"):
            assert int(res[0][2][n]) == int(b), n
    assert nstat == 2 * 23


def test_grad_reducer_counts_in_place_params_once():
    """A layer that accumulates into .grad in place and calls mark_ready (nn.py: the GRU / Linear
    backward) still gets its post-accumulate hook run by autograd afterwards (with nothing to add).
    The reducer must count that parameter once: counted twice, a bucket shared with a parameter whose
    gradient comes later was declared complete and its all-reduce launched before that gradient
    existed (found at round 3 by the mode-1 SyncBN DP test: the fc1 / backend conv gradients came back
    zero over gloo).  Single process: the bucket's launch flag is what is checked."""
    torch.manual_seed(0)
    a = torch.nn.Parameter(torch.randn(6, 5))
    b = torch.nn.Parameter(torch.randn(4, 5))
    params = [b, a]
    offs = [0, 64]
    flat = types.SimpleNamespace(params=params, offsets=offs, numel=128, grad=torch.zeros(128))
    b.grad = flat.grad[0:20].view_as(b)
    a.grad = flat.grad[64:94].view_as(a)
    seen = []
    b.register_post_accumulate_grad_hook(lambda p: seen.append(red.launched[0]))   # runs before the reducer's hook
    red = parallel.GradReducer(flat, bucket_mb=1.0)
    assert len(red.buckets) == 1

    class InPlace(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            ctx.save_for_backward(x, w)
            return x @ w.t()

        @staticmethod
        def backward(ctx, dy):
            x, w = ctx.saved_tensors
            w.grad.add_(dy.t() @ x)          # in place, as the HIP GEMM epilogues do
            red.mark_ready([w])
            return dy @ w, None

    red.begin()
    x = torch.randn(3, 4)
    InPlace.apply(x @ b, a).sum().backward()
    assert seen == [False]                 # b's gradient arrived before the bucket was complete
    assert red.launched == [True]
