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
