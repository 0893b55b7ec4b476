"""The 16-bit train steps bench.py times, at BASELINE.json's own shapes, against the fp32 CPU oracle
(SURVEY.md §8(a) A5 / A9, §8(d) configs[1] and configs[4]; VERDICT r03 "next" #1):

* cfg5 — int16 PCM + resident noise bank -> K4 noise mix (dataset.py:183-193) fused into the spectrogram
  [49 x 321] -> model_spec_bgru (model_spec_bgru.py:19-35), B = 512, fp16 matrix-core operands, the
  static loss scale of bench.py (1024) through optim.LossScaler, CE, backward, Adam;
* cfg2 — MFCC [51 x 39] -> model_mfcc_bgru (model_mfcc_bgru.py:21-37), B = 256, bf16 operands.

The other 16-bit mode of each model runs too.  Checked (tests/tolerances.py, "LP_*"): the mixed PCM
bit-exact; logits and loss <= 2e-2 relative; EVERY gradient tensor ||g - g_oracle||_2 /
||g_oracle||_2 <= 2e-2 (after unscaling); the parameters after the one Adam step (a) equal torch's
Adam formula applied to the HIP path's own unscaled gradient (<= 2e-7 absolute: the fused kernel's
arithmetic) and (b) move like the oracle's own Adam step: the update's disagreement with the
oracle's, weighted by |g_oracle|, <= 2e-2 (Adam's first step is lr * g / |g| per element, so an
element whose gradient is below the 16-bit noise floor may flip sign; weighting by |g| measures
what that costs).  No step may be skipped and no persistent recurrence may time out.

Plus the fp16 overflow path: a forced overflow (a loss scale of 3e38, then a NaN planted in the
gradient buffer) must skip the step — parameters, both Adam moments and the device step count
unchanged, the overflow counted, a dynamic scale halved — and the next clean step must run.
"""
import numpy as np
import pytest
import torch

from oracle import features as OF
from oracle import models as OM
from tolerances import LP_ADAM_ABS, LP_GRAD_REL, LP_UPDATE_WEIGHTED, LOGITS_REL_LOWPREC, rel_err
from speechrecognitionproject_amd import _lib
from speechrecognitionproject_amd import features as K
from speechrecognitionproject_amd import nn as snn
from speechrecognitionproject_amd.optim import Adam, FlatParams, LossScaler
from speechrecognitionproject_amd.synthetic import synthetic_clips, synthetic_noise_bank, synthetic_noise_draws

pytestmark = pytest.mark.gpu

LR = 1e-4
LOSS_SCALE = 1024.0      # bench.py FP16_LOSS_SCALE
OCLS = {"mfcc_bgru": OM.MfccBGRU, "spec_bgru": OM.SpecBGRU}
BATCH = {"mfcc_bgru": 256, "spec_bgru": 512}


def _inputs(name):
    B = BATCH[name]
    if name == "spec_bgru":
        x, y = synthetic_clips(B, seed=61, clip=30000)
        pcm16 = x.astype(np.int16)
        bank = synthetic_noise_bank()
        files, offs, gains = synthetic_noise_draws(B, seed=62)
        mixed = np.stack([OF.add_noise_uniform(pcm16[i], bank[files[i]], int(offs[i]), float(gains[i]))
                          for i in range(B)]).astype(np.float32)
        return {"pcm16": pcm16, "bank": bank, "draws": (files, offs, gains), "mixed": mixed, "labels": y}
    x, y = synthetic_clips(B, seed=63)
    return {"mixed": x, "labels": y}


@pytest.fixture(scope="module", params=["mfcc_bgru", "spec_bgru"])
def oracle_case(request):
    """One fp32 oracle train step per model (shared by both 16-bit modes)."""
    name = request.param
    inp = _inputs(name)
    sd = OM.seeded_state_dict(OCLS[name](), 0)
    ref = OCLS[name]()
    ref.load_state_dict(sd)
    ref.train()
    p0 = {n: p.detach().clone() for n, p in ref.named_parameters()}
    out, loss, _ = OM.train_step(ref, torch.from_numpy(inp["mixed"]), torch.from_numpy(inp["labels"]), lr=LR)
    grads = {n: p.grad.detach().clone() for n, p in ref.named_parameters()}
    p1 = {n: p.detach().clone() for n, p in ref.named_parameters()}
    return name, inp, sd, out.numpy(), float(loss), grads, p0, p1


def _torch_adam_first_step(p0, g):
    """torch.optim.Adam's first step in its operation order (fp32), on the HIP path's gradient."""
    m = (1 - 0.9) * g
    v = (1 - 0.999) * g * g
    denom = v.sqrt() / np.sqrt(1 - 0.999) + 1e-8
    return p0 - (LR / (1 - 0.9)) * (m / denom)


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_lowprec_train_step_at_config_shape(gpu, oracle_case, precision):
    import importlib
    name, inp, sd, want_out, want_loss, want_g, p0_ref, p1_ref = oracle_case
    mod = importlib.import_module("speechrecognitionproject_amd.models.model_" + name)
    net = mod.Network().cuda()
    net.load_state_dict(sd)
    net.train()
    flat = FlatParams(net.parameters())
    opt = Adam(net.parameters(), lr=LR, flat=flat)
    lab = torch.from_numpy(inp["labels"]).cuda()
    try:
        _lib.set_matmul_precision(precision)
        scaler = LossScaler(LOSS_SCALE, dynamic=False) if precision == "fp16" else None
        scale = LOSS_SCALE if scaler is not None else 1.0
        opt.zero_grad()
        if name == "spec_bgru":     # cfg5: the K4 mix inside the step (fused into K3's loads), as bench.py runs it
            files, offs, gains = inp["draws"]
            x = K.NoisyClips(torch.from_numpy(inp["pcm16"]).cuda(), torch.from_numpy(inp["bank"]).cuda(),
                             torch.from_numpy(files).cuda(), torch.from_numpy(offs).cuda(),
                             torch.from_numpy(gains).cuda())
            assert np.array_equal(x.mixed().cpu().numpy(), inp["mixed"])
        else:
            x = torch.from_numpy(inp["mixed"]).cuda()
        out = net(x)
        loss = snn.CrossEntropyLoss()(out, lab)
        (scaler.scale(loss) if scaler is not None else loss).backward()
        torch.cuda.synchronize()
        grads = {n: (p.grad.detach() / scale).cpu() for n, p in net.named_parameters()}
        p0 = {n: p.detach().cpu().clone() for n, p in net.named_parameters()}
        opt.step(scaler=scaler)
        torch.cuda.synchronize()
    finally:
        _lib.set_matmul_precision("fp32")
    assert _lib.spin_timeouts() == 0
    assert scaler is None or scaler.overflows() == 0
    assert opt.step_count == 1

    assert rel_err(out.detach().cpu().numpy(), want_out) <= LOGITS_REL_LOWPREC
    assert abs(loss.item() - want_loss) <= LOGITS_REL_LOWPREC * max(1.0, abs(want_loss))
    worst = {}
    for n, g in grads.items():
        gr = want_g[n].double()
        if gr.norm().item() == 0.0:
            # exactly-zero gradients stay exactly zero: the last layer's reverse W_hh only ever meets
            # h0 = 0 (the model reads out[:, -1, :], one reverse step)
            assert g.abs().max().item() == 0.0, n
            worst[n] = 0.0
            continue
        worst[n] = ((g.double() - gr).norm() / gr.norm()).item()
    bad = {n: e for n, e in worst.items() if not e <= LP_GRAD_REL}
    assert not bad, (bad, worst)

    for n, p in net.named_parameters():
        p1 = p.detach().cpu()
        assert torch.equal(p0[n], p0_ref[n]), n
        want_exact = _torch_adam_first_step(p0[n], grads[n])
        assert (p1 - want_exact).abs().max().item() <= LP_ADAM_ABS, n
        d_gpu = (p1 - p0[n]).double()
        d_ref = (p1_ref[n] - p0_ref[n]).double()
        w = want_g[n].double().abs()
        if w.sum().item() == 0.0:
            assert torch.equal(d_gpu, d_ref), n
            continue
        dis = ((w * (d_gpu - d_ref).abs()).sum() / (w * d_ref.abs()).sum()).item()
        assert dis <= LP_UPDATE_WEIGHTED, (n, dis)


def _small_step(net, opt, scaler, x, lab):
    opt.zero_grad()
    loss = snn.CrossEntropyLoss()(net(x), lab)
    scaler.scale(loss).backward()
    opt.step(scaler=scaler)
    return loss


def test_fp16_overflow_skips_the_step(gpu):
    """A step whose loss-scaled gradients overflow fp16 (or carry a NaN) changes nothing but the
    scaler's state; the next clean step updates normally (optim.LossScaler, srk_adam_step_scaled)."""
    from speechrecognitionproject_amd.models import model_mfcc_bgru
    torch.manual_seed(0)
    net = model_mfcc_bgru.Network().cuda()
    net.load_state_dict(OM.seeded_state_dict(OM.MfccBGRU(), 0))
    flat = FlatParams(net.parameters())
    opt = Adam(net.parameters(), lr=LR, flat=flat)
    x, y = synthetic_clips(16, seed=64)
    x, lab = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    try:
        _lib.set_matmul_precision("fp16")
        scaler = LossScaler(3e38, dynamic=True)          # the scaled loss overflows to inf
        opt.sync_lr()                                     # (the step writes lr into state_dev first)
        snap = (flat.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), opt.state_dev.clone())
        _small_step(net, opt, scaler, x, lab)
        torch.cuda.synchronize()
        assert not torch.isfinite(flat.grad).all()
        assert torch.equal(flat.data, snap[0]) and torch.equal(opt.exp_avg, snap[1])
        assert torch.equal(opt.exp_avg_sq, snap[2]) and torch.equal(opt.state_dev, snap[3])
        assert scaler.overflows() == 1 and scaler.get_scale() == np.float32(3e38) * np.float32(0.5)
        assert opt.step_count == 0

        # a NaN planted in an otherwise clean gradient: skipped too
        scaler2 = LossScaler(1024.0, dynamic=False)
        opt.zero_grad()
        snn.CrossEntropyLoss()(net(x), lab).backward()
        flat.grad[flat.numel // 2] = float("nan")
        opt.step(scaler=scaler2)
        torch.cuda.synchronize()
        assert torch.equal(flat.data, snap[0]) and scaler2.overflows() == 1 and scaler2.get_scale() == 1024.0

        # then a clean step runs and counts as step 1
        _small_step(net, opt, scaler2, x, lab)
        torch.cuda.synchronize()
        assert scaler2.overflows() == 1 and opt.step_count == 1
        assert not torch.equal(flat.data, snap[0]) and torch.isfinite(flat.data).all()
    finally:
        _lib.set_matmul_precision("fp32")


def test_dynamic_scale_grows_after_clean_steps(gpu):
    lin = snn.Linear(64, 12).cuda()
    flat = FlatParams(lin.parameters())
    opt = Adam(lin.parameters(), lr=LR, flat=flat)
    scaler = LossScaler(8.0, dynamic=True, growth_interval=3)
    x = torch.randn(32, 64, device="cuda")
    lab = torch.randint(0, 12, (32,), device="cuda")
    for _ in range(7):
        _small_step(lin, opt, scaler, x, lab)
    assert scaler.get_scale() == 32.0 and scaler.overflows() == 0 and opt.step_count == 7
