"""HIP-graph replay of the train step (speechrecognitionproject_amd/graphs.py), as bench.py and
training.py --graph use it: the replayed step must be the eager step, bit for bit — the kernels are
deterministic, so K graph replays after the warm-up leave the same parameters, Adam moments and
BatchNorm statistics as the same number of eager steps on the same batches (training.py:83-95).
The per-step host values live on the device: the Adam step count advances per replay (bias
corrections of steps 1..K, not K copies of step 1), dropout draws a fresh mask per replay (the
eager reference steps draw theirs the same way under nn.dropout_replay_mode), the fp16 loss scale
and overflow check run inside the graph (optim.LossScaler).  The capture must not see a live
autograd graph of a warm-up step (torch's AccumulateGrad stream-mismatch warning)."""
import warnings

import pytest
import torch

from oracle import models as OM
from speechrecognitionproject_amd import _lib
from speechrecognitionproject_amd import nn as snn
from speechrecognitionproject_amd.graphs import GraphedStep
from speechrecognitionproject_amd.optim import Adam, FlatParams, LossScaler
from speechrecognitionproject_amd.synthetic import synthetic_clips

pytestmark = pytest.mark.gpu

OCLS = {"mfcc_bgru": OM.MfccBGRU, "fbanks_cnn": OM.FbanksCNN, "resnet_bgru": OM.ResnetBGRU, "spec_bgru": OM.SpecBGRU}


def _setup(name, B, seed):
    import importlib
    mod = importlib.import_module("speechrecognitionproject_amd.models.model_" + name)
    net = mod.Network().cuda()
    net.load_state_dict(OM.seeded_state_dict(OCLS[name](), 0))
    net.train()
    flat = FlatParams(net.parameters())
    opt = Adam(net.parameters(), lr=1e-4, flat=flat)
    x, y = synthetic_clips(3 * B, seed=seed)
    return net, flat, opt, torch.from_numpy(x).cuda().view(3, B, -1), torch.from_numpy(y).cuda().view(3, B)


def _stream_mismatch(ws):
    return [str(w.message)[:120] for w in ws if "AccumulateGrad" in str(w.message)]


@pytest.mark.parametrize("name,B,precision", [("mfcc_bgru", 64, "fp32"), ("mfcc_bgru", 64, "bf16"),
                                              ("resnet_bgru", 8, "fp32"), ("spec_bgru", 32, "fp16"),
                                              ("fbanks_cnn", 64, "fp32"), ("fbanks_cnn", 64, "bf16")])
def test_graph_replay_equals_eager_steps(gpu, name, B, precision):
    """fbanks_cnn runs with dropout on (train mode): the replays' masks come from the device counter,
    which the eager reference steps follow under nn.dropout_replay_mode."""
    K = 4
    try:
        _lib.set_matmul_precision(precision)
        states = []
        for graphed in (False, True):
            torch.manual_seed(0)
            net, flat, opt, pcm, lab = _setup(name, B, seed=17)
            crit = snn.CrossEntropyLoss()
            scaler = LossScaler(1024.0, dynamic=False) if precision == "fp16" else None
            sx, sy = pcm[0].clone(), lab[0].clone()

            def body():
                opt.zero_grad()
                loss = crit(net(sx), sy)
                (scaler.scale(loss) if scaler is not None else loss).backward()
                opt.step(scaler=scaler)
                return loss

            losses = []
            if graphed:
                with warnings.catch_warnings(record=True) as ws:
                    warnings.simplefilter("always")
                    g = GraphedStep(body, warmup=2)         # 2 eager steps on batch 0, then the capture
                    for i in range(K):
                        sx.copy_(pcm[(i + 1) % 3])
                        sy.copy_(lab[(i + 1) % 3])
                        losses.append(g.replay().item())
                assert not _stream_mismatch(ws), _stream_mismatch(ws)
                g.release()
            else:
                for i in range(2 + K):
                    if i >= 2:
                        sx.copy_(pcm[(i - 1) % 3])
                        sy.copy_(lab[(i - 1) % 3])
                        with snn.dropout_replay_mode():
                            loss = body()
                    else:
                        loss = body()
                    if i >= 2:
                        losses.append(loss.item())
            torch.cuda.synchronize()
            if scaler is not None:
                assert scaler.overflows() == 0
            bufs = [b.detach().clone() for n, b in net.named_buffers() if "running" in n]
            states.append((flat.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), opt.state_dev.clone(),
                           bufs, losses))
    finally:
        _lib.set_matmul_precision("fp32")
    (p0, m0, v0, s0, b0, l0), (p1, m1, v1, s1, b1, l1) = states
    assert int(s0[0]) == int(s1[0]) == 2 + K                    # the device step count advanced per replay
    assert l0 == l1
    assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1)
    assert all(torch.equal(a, b) for a, b in zip(b0, b1))
    assert _lib.spin_timeouts() == 0


def test_graph_dropout_fresh_mask_per_replay(gpu):
    d = snn.Dropout(0.5).cuda()
    x = torch.ones(1 << 16, device="cuda")
    g = GraphedStep(lambda: d(x), warmup=2)
    a = g.replay().clone()
    b = g.replay().clone()
    assert not torch.equal(a, b)
    assert abs((a != 0).float().mean().item() - 0.5) < 0.02 and abs((b != 0).float().mean().item() - 0.5) < 0.02
    g.release()


def test_dropout_leaves_cpu_generator_alone(gpu):
    """The reference's nn.Dropout on the GPU draws from the CUDA generator; the CPU stream (the
    DataLoader's shuffles, seeded by torch.manual_seed) must not move."""
    d = snn.Dropout(0.5).cuda()
    x = torch.ones(4096, device="cuda")
    torch.manual_seed(5)
    ref = torch.rand(4)
    torch.manual_seed(5)
    d(x)
    d(x)
    assert torch.equal(torch.rand(4), ref)


def test_graph_refuses_replay_after_scratch_regrowth(gpu):
    """A graph refers to the library's split-K scratch by address: once that buffer is reallocated
    (here: released, as a larger shape growing it would), replay must fail loudly instead of writing
    to freed memory; a fresh capture works again."""
    lin = snn.Linear(4096, 64).cuda()
    xb = torch.randn(256, 4096, device="cuda")

    def body():
        return lin(xb).sum()

    g = GraphedStep(body, warmup=2)
    want = g.replay().item()
    _lib.set_option("release_scratch", 1)
    assert not g.valid()
    with pytest.raises(_lib.SrkError):
        g.replay()
    g2 = GraphedStep(body, warmup=2)
    assert g2.replay().item() == want
