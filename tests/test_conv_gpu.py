"""K6 conv / pooling / dropout kernels vs plain PyTorch fp32 on the CPU, and the fbanks_cnn
plugin vs the reference golden."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden
from oracle import models as OM
from tolerances import LOGITS_REL, rel_err
from speechrecognitionproject_amd import _lib
from speechrecognitionproject_amd import nn as snn
from speechrecognitionproject_amd._lib import call
from speechrecognitionproject_amd.features import ptr, stream_ptr
from speechrecognitionproject_amd.models import model_fbanks_cnn
from speechrecognitionproject_amd.optim import Adam

pytestmark = pytest.mark.gpu

CONV2D = [  # N, H, W, Ci, Co, KH, KW, ph, pw   (model_fbanks_cnn.py:72-75 + odd sizes)
    (3, 98, 120, 1, 64, 7, 3, 3, 1),
    (2, 98, 40, 64, 128, 1, 7, 0, 3),
    (2, 98, 10, 128, 256, 1, 10, 0, 0),
    (3, 98, 1, 256, 512, 7, 1, 3, 0),
    (2, 9, 11, 5, 7, 3, 2, 1, 0),
    (24, 98, 40, 64, 128, 1, 7, 0, 3),   # many tiles + deep split-K weight gradient
    (4, 17, 13, 12, 36, 3, 3, 1, 1),     # N % 4 == 0 but odd tile edges
]


def _check_conv(N, H, W, Ci, Co, KH, KW, ph, pw, sh=1, sw=1):
    g = torch.Generator().manual_seed(N * 100 + Co)
    x = torch.randn(N, Ci, H, W, generator=g)
    w = torch.randn(Co, Ci, KH, KW, generator=g) / (Ci * KH * KW) ** 0.5
    b = torch.randn(Co, generator=g)
    xr, wr, br = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, br, stride=(sh, sw), padding=(ph, pw))
    gy = torch.randn(yr.shape, generator=g)
    (yr * gy).sum().backward()
    xm = x.permute(0, 2, 3, 1).contiguous().cuda().requires_grad_(True)
    wm, bm = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    ym = snn._Conv2dNHWCFn.apply(xm, wm, bm, (ph, pw), (sh, sw))
    (ym * gy.permute(0, 2, 3, 1).cuda()).sum().backward()
    y_nchw = ym.detach().permute(0, 3, 1, 2).cpu()
    assert y_nchw.shape == yr.shape
    assert rel_err(y_nchw.numpy(), yr.detach().numpy()) <= 1e-5
    assert rel_err(xm.grad.permute(0, 3, 1, 2).cpu().numpy(), xr.grad.numpy()) <= 1e-5
    assert rel_err(wm.grad.cpu().numpy(), wr.grad.numpy()) <= 1e-4
    assert rel_err(bm.grad.cpu().numpy(), br.grad.numpy()) <= 1e-5


@pytest.mark.parametrize("shape", CONV2D)
def test_conv2d_nhwc_vs_torch(gpu, shape):
    _check_conv(*shape)


@pytest.mark.parametrize("shape", [(64, 98, 40, 64, 128, 1, 7, 0, 3), (40, 98, 40, 64, 64, 1, 7, 0, 3),
                                   (96, 98, 1, 64, 128, 7, 1, 3, 0)])
def test_conv2d_tile256_vs_torch(gpu, shape):
    """srk option conv_tile = 256: the 256-row, 8-wave conv tiles (fp32) on tall convolutions."""
    from speechrecognitionproject_amd import _lib
    try:
        _lib.set_option("conv_tile", 256)
        _check_conv(*shape)
    finally:
        _lib.set_option("conv_tile", 128)


@pytest.mark.parametrize("shape", [(2, 98, 40, 64, 128, 1, 7, 0, 3), (3, 98, 1, 256, 512, 7, 1, 3, 0),
                                   (2, 98, 10, 128, 256, 1, 10, 0, 0), (4, 17, 13, 32, 128, 3, 3, 1, 1),
                                   (2, 1, 1000, 64, 128, 1, 15, 0, 7, 1, 2), (24, 98, 40, 64, 128, 1, 7, 0, 3)])
def test_conv2d_ring_vs_torch(gpu, shape):
    """srk option conv_ring: the fp32 LDS-DMA ring implicit GEMM (gemm_p32_kernel's structure with
    per-K-tile conv gathers, direct epilogue, fused bias sums) wherever the shape qualifies (channel
    counts % 16, >= 128 output columns, stride 1 for the data gradient); the rest as before."""
    from speechrecognitionproject_amd import _lib
    try:
        _lib.set_option("conv_ring", 0x87)   # every qualifying shape, any K
        _check_conv(*shape)
    finally:
        _lib.set_option("conv_ring", 0x77)


@pytest.mark.parametrize("shape", [  # 1-D strided convs of model_resnet_bgru.py:48,19-23 as H=1
    (2, 1, 16000, 1, 64, 1, 80, 0, 38, 1, 16), (2, 1, 1000, 64, 128, 1, 15, 0, 7, 1, 2),
    (2, 1, 1000, 64, 128, 1, 1, 0, 0, 1, 2), (3, 1, 125, 512, 512, 1, 15, 0, 7, 1, 1)])
def test_conv1d_strided_vs_torch(gpu, shape):
    _check_conv(*shape)


@pytest.mark.parametrize("N,H,W,C,kh,kw", [(2, 98, 120, 64, 1, 3), (2, 98, 40, 128, 1, 4), (3, 98, 1, 512, 98, 1),
                                           (2, 5, 7, 4, 2, 3)])
def test_maxpool_vs_torch(gpu, N, H, W, C, kh, kw):
    g = torch.Generator().manual_seed(H * W)
    x = torch.randn(N, C, H, W, generator=g)
    x[0, 0, 0, :3] = 1.0   # a tie: gradient goes to the first maximum, as in PyTorch
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, (kh, kw))
    gy = torch.randn(yr.shape, generator=g)
    (yr * gy).sum().backward()
    xm = x.permute(0, 2, 3, 1).contiguous().cuda().requires_grad_(True)
    ym = snn._MaxPoolNHWCFn.apply(xm, kh, kw)
    (ym * gy.permute(0, 2, 3, 1).cuda()).sum().backward()
    assert torch.equal(ym.detach().permute(0, 3, 1, 2).cpu(), yr.detach())
    assert torch.equal(xm.grad.permute(0, 3, 1, 2).cpu(), xr.grad)


@pytest.mark.parametrize("N,H,W,KH,KW,pool", [
    (3, 98, 120, 7, 3, 3), (2, 7, 9, 7, 3, 3), (1, 5, 31, 7, 3, 3),     # model_fbanks_cnn.py:72-73
    (3, 49, 321, 3, 7, 5), (2, 4, 13, 3, 7, 5)])                        # model_spec_cnn.py:24-25
def test_conv1_pool_fused_vs_torch(gpu, N, H, W, KH, KW, pool):
    """Fused conv1 + bias + maxpool (1,pool) vs torch conv2d + max_pool2d (floor mode: trailing
    columns dropped): pooled values, and dW / db through the pool (gradient routed by the argmax)."""
    g = torch.Generator().manual_seed(N * 7 + W)
    pad = (KH // 2, KW // 2)
    x = torch.randn(N, 1, H, W, generator=g) * 30.0
    w = torch.randn(64, 1, KH, KW, generator=g) * 0.2
    b = torch.randn(64, generator=g)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = F.max_pool2d(F.conv2d(x, wr, br, padding=pad), (1, pool))
    gy = torch.randn(yr.shape, generator=g)
    (yr * gy).sum().backward()
    wm, bm = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    ym = snn._Conv1PoolFn.apply(x[:, 0].cuda(), wm, bm, pad, pool)
    (ym * gy.permute(0, 2, 3, 1).cuda()).sum().backward()
    assert rel_err(ym.detach().permute(0, 3, 1, 2).cpu().numpy(), yr.detach().numpy()) <= 1e-5
    assert rel_err(wm.grad.cpu().numpy(), wr.grad.numpy()) <= 1e-4
    assert rel_err(bm.grad.cpu().numpy(), br.grad.numpy()) <= 1e-5


@pytest.mark.parametrize("prec", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("N,H,W,KH,KW,pool", [
    (3, 98, 120, 7, 3, 3), (2, 7, 9, 7, 3, 3), (1, 37, 31, 7, 3, 3), (3, 49, 321, 3, 7, 5), (2, 17, 13, 3, 7, 5)])
def test_conv1_pool_fwd16(gpu, prec, N, H, W, KH, KW, pool):
    """srk_conv1_pool_fwd16 (the fused conv1 + maxpool forward): pooled values vs torch fp32 conv2d +
    max_pool2d (1e-5), argmax bytes = the first maximum of each window wherever the window's top two
    values are apart, NaN windows (the maxpool rule: NaN wins), and the 16-bit copy == torch's RNE
    rounding of the fp32 output bit for bit; block row tails included."""
    import ctypes
    g = torch.Generator().manual_seed(N * 11 + W + KH)
    x = (torch.randn(N, H, W, generator=g) * 30.0)
    w = (torch.randn(64, 1, KH, KW, generator=g) * 0.2)
    b = torch.randn(64, generator=g)
    x[0, 0, :4] = float("nan")
    Wq = W // pool
    xd, wd, bd = x.cuda(), w.cuda(), b.cuda()
    try:
        _lib.set_matmul_precision(prec)
        y = torch.full((N, H, Wq, 64), 7.0, device="cuda")
        arg = torch.full((N, H, Wq, 64), 9, dtype=torch.uint8, device="cuda")
        y16 = torch.full((N * H * Wq * 64,), 3, dtype=torch.int16, device="cuda")
        wr = ctypes.c_int(-1)
        call("srk_conv1_pool_fwd16", ptr(xd), N, H, W, ptr(wd), ptr(bd), 64, KH, KW, KH // 2, KW // 2, pool, ptr(y),
             ptr(arg), ptr(y16), ctypes.byref(wr), stream_ptr())
        torch.cuda.synchronize()
    finally:
        _lib.set_matmul_precision("fp32")
    assert wr.value == (0 if prec == "fp32" else 1)
    dense = torch.nn.functional.conv2d(x.unsqueeze(1), w, b, padding=(KH // 2, KW // 2))   # [N, 64, H, W]
    win = dense[..., :Wq * pool].reshape(N, 64, H, Wq, pool).permute(0, 2, 3, 1, 4)      # [N, H, Wq, 64, pool]
    y, arg = y.cpu(), arg.cpu()
    nan_win = torch.isnan(win).any(-1)
    assert bool(nan_win.any()) and torch.equal(torch.isnan(y), nan_win)
    ref = win.nan_to_num(nan=-1e30).max(-1)
    ok = ~nan_win
    assert ((y[ok] - ref.values[ok]).abs().max() / ref.values[ok].abs().max()).item() <= 1e-5
    top2 = win.nan_to_num(nan=-1e30).topk(2, dim=-1).values
    clear = ok & ((top2[..., 0] - top2[..., 1]) > 1e-3 * (1 + top2[..., 0].abs()))
    assert torch.equal(arg[clear].long(), ref.indices[clear])
    assert bool((arg < pool).all())
    if wr.value:
        dt = torch.bfloat16 if prec == "bf16" else torch.float16
        got = y16.cpu().view(dt).reshape(N, H, Wq, 64)
        assert torch.equal(got[ok].view(torch.int16), y[ok].to(dt).view(torch.int16))


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("N,H,W,Ci,Co,KH,KW,ph,pw", [
    (2, 98, 40, 64, 128, 1, 7, 0, 3),      # conv2 of model_fbanks_cnn.py:74 (+ maxpool2 :75)
    (16, 98, 40, 64, 128, 1, 7, 0, 3),     # many tiles
    (2, 3, 8, 128, 64, 1, 7, 0, 3),        # a few rows, deep k: the split-K forward (dense, then pooled)
    (3, 5, 12, 8, 36, 3, 3, 1, 1),         # 3 x 3 taps, N not a tile multiple
])
@pytest.mark.parametrize("gather,ring", [(1, 0), (0, 0), (0, 6), (0, 0x87), (0, 0x77), (0, 0xf7)])
def test_conv_pool_fused_equals_separate(gpu, gather, ring, precision, N, H, W, Ci, Co, KH, KW, ph, pw):
    """conv + bias + MaxPool2d((1, 4)) in one launch (srk_conv2d_nhwc_fwd_pool: pooled epilogue and
    uint8 argmax; the backward unpools through the argmax) == the separate conv and maxpool kernels
    (bitwise: the same accumulators, the same first-maximum rule, the same gradient kernels), and
    vs torch's CPU fp32 conv + max_pool2d (fp32 mode).  gather = 1: the backward's gathers read the
    pooled gradient through the argmax (option conv_unpool_gather); 0: a dense scratch gradient."""
    from speechrecognitionproject_amd import _lib
    g = torch.Generator().manual_seed(N * 7 + Co)
    x = torch.randn(N, H, W, Ci, generator=g)
    w = torch.randn(Co, Ci, KH, KW, generator=g) / (Ci * KH * KW) ** 0.5
    b = torch.randn(Co, generator=g)
    Wo = W + 2 * pw - KW + 1
    gy = torch.randn(N, H + 2 * ph - KH + 1, Wo // 4, Co, generator=g)
    conv = snn.Conv2d(Ci, Co, (KH, KW), padding=(ph, pw)).cuda()
    pool = snn.MaxPool2d((1, 4))
    outs = []
    try:
        _lib.set_matmul_precision(precision)
        _lib.set_option("conv_unpool_gather", gather)
        _lib.set_option("conv_ring", ring)
        _lib.set_option("conv_row32", 0)   # the implicit-GEMM paths (row-staged: test_conv_row32_equals_gemm)
        for fused in (True, False):
            _lib.set_fused_conv_pool(fused)
            with torch.no_grad():
                conv.weight.copy_(w)
                conv.bias.copy_(b)
            conv.weight.grad = conv.bias.grad = None
            xm = x.cuda().requires_grad_(True)
            y = snn.conv_pool(xm, conv, pool)
            (y * gy.cuda()).sum().backward()
            torch.cuda.synchronize()
            outs.append([t.detach().cpu() for t in (y, xm.grad, conv.weight.grad, conv.bias.grad)])
    finally:
        _lib.set_option("conv_unpool_gather", 1)
        _lib.set_option("conv_ring", 0x77)
        _lib.set_option("conv_row32", 1)
        _lib.set_fused_conv_pool(True)
        _lib.set_matmul_precision("fp32")
    row_wgrad = (W, Ci, Co, KH, KW, ph, pw) == (40, 64, 128, 1, 7, 0, 3)   # fbanks_cnn conv2's shape
    for i, (a, c) in enumerate(zip(*outs)):
        if precision != "fp32" and (i == 3 or (i == 2 and row_wgrad)):
            # 16-bit modes (option conv_unpool16): the fused backward sums the bias gradient over the
            # pooled rows, the separate one over the dense dY (the same values and zeros, another order);
            # conv2's fused backward takes its weight gradient from the pooled gradient on the row-staged
            # conv_row16_wgrad_kernel (workgroup slabs reduced in order: another fp32 summation order)
            assert rel_err(a.numpy(), c.numpy()) <= 1e-5
        else:
            assert torch.equal(a, c)
    if precision == "fp32":
        xr, wr, br = (t.clone().requires_grad_(True) for t in (x.permute(0, 3, 1, 2), w, b))
        yr = F.max_pool2d(F.conv2d(xr, wr, br, padding=(ph, pw)), (1, 4))
        (yr * gy.permute(0, 3, 1, 2)).sum().backward()
        y, dx, dw, db = outs[0]
        assert rel_err(y.permute(0, 3, 1, 2).numpy(), yr.detach().numpy()) <= 1e-5
        assert rel_err(dx.permute(0, 3, 1, 2).numpy(), xr.grad.numpy()) <= 1e-5
        assert rel_err(dw.numpy(), wr.grad.numpy()) <= 1e-4
        assert rel_err(db.numpy(), br.grad.numpy()) <= 1e-5


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_conv_bias_grad_fused_into_wgrad(gpu, precision):
    """The conv bias gradient summed inside the weight-gradient kernel (option conv_fused_db, the
    unrounded fp32 dY values) vs the separate column-sum kernel: same to fp32 summation order, and
    every other gradient bitwise unchanged."""
    from speechrecognitionproject_amd import _lib
    g = torch.Generator().manual_seed(11)
    N, H, W, Ci, Co, KH, KW, ph, pw = 24, 98, 40, 64, 128, 1, 7, 0, 3
    x = torch.randn(N, H, W, Ci, generator=g).cuda()
    w = torch.randn(Co, Ci, KH, KW, generator=g).cuda() / (Ci * KW) ** 0.5
    b = torch.randn(Co, generator=g).cuda()
    gy = torch.randn(N, H, W, Co, generator=g).cuda()
    res = []
    try:
        _lib.set_matmul_precision(precision)
        for fused in (1, 0):
            _lib.set_option("conv_fused_db", fused)
            xm, wm, bm = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
            (snn._Conv2dNHWCFn.apply(xm, wm, bm, (ph, pw), (1, 1)) * gy).sum().backward()
            torch.cuda.synchronize()
            res.append((xm.grad.cpu(), wm.grad.cpu(), bm.grad.cpu()))
    finally:
        _lib.set_option("conv_fused_db", 1)
        _lib.set_matmul_precision("fp32")
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    want = gy.double().sum(dim=(0, 1, 2)).cpu()
    assert rel_err(res[0][2].numpy(), want.numpy()) <= 1e-5
    assert rel_err(res[1][2].numpy(), want.numpy()) <= 1e-5


def test_maxpool_rejects_unaligned_channels(gpu):
    from speechrecognitionproject_amd._lib import SrkError
    with pytest.raises(SrkError):
        snn._MaxPoolNHWCFn.apply(torch.zeros(1, 4, 6, 3, device="cuda"), 1, 3)


def test_dropout_mask(gpu):
    d = snn.Dropout(0.5).cuda()
    x = torch.ones(1 << 20, device="cuda", requires_grad=True)
    y = d(x)
    kept = (y != 0).float().mean().item()
    assert abs(kept - 0.5) < 0.01
    assert set(torch.unique(y).tolist()) <= {0.0, 2.0}
    y.sum().backward()
    assert torch.equal(x.grad, y.detach())
    y2 = d(x)
    assert not torch.equal(y, y2)          # a fresh mask per call
    d.eval()
    assert d(x) is x


def test_dropout_follows_torch_seed(gpu):
    d = snn.Dropout(0.5).cuda()
    x = torch.ones(4096, device="cuda")
    torch.manual_seed(3)
    a = d(x)
    torch.manual_seed(3)
    b = d(x)
    assert torch.equal(a, b)
    keep = (torch.arange(4096, device="cuda") % 3 == 0).to(torch.uint8)
    d.set_mask(keep)
    assert torch.equal(d(x), keep.float() * 2.0)
    assert not torch.equal(d(x), keep.float() * 2.0)     # the supplied mask is used once


@pytest.mark.parametrize("fixture", ["fbanks_cnn_golden.npz", "fbanks_cnn_train_golden.npz"])
def test_fbanks_cnn_vs_reference_golden(gpu, fixture):
    # the train-mode fixture replays the reference's dropout (model_fbanks_cnn.py:79,98) with the
    # keep mask it exported, through srk_dropout_apply
    g = golden(fixture)
    net = model_fbanks_cnn.Network().cuda()
    ref_sd = OM.seeded_state_dict(OM.FbanksCNN(), 0)
    assert list(net.state_dict().keys()) == list(ref_sd.keys())
    net.load_state_dict(ref_sd)
    net.train(bool(g["train_mode"]))
    if "dropout_keep" in g:
        assert net.training
        net.dropout.set_mask(torch.from_numpy(g["dropout_keep"]))
    params = dict(net.named_parameters())
    before = {k: v.detach().clone() for k, v in params.items()}
    opt = Adam(net.parameters(), lr=1e-4)
    opt.zero_grad()
    out = net(torch.from_numpy(g["pcm"]))
    loss = snn.CrossEntropyLoss()(out, torch.from_numpy(g["labels"]).cuda())
    loss.backward()
    grads = {k: v.grad.detach().clone() for k, v in params.items()}
    opt.step()
    assert rel_err(out.detach().cpu().numpy(), g["logits"]) <= LOGITS_REL
    assert abs(loss.item() - float(g["loss"])) <= 1e-4 * max(1.0, abs(float(g["loss"])))
    for k in g["names"]:
        gv = grads[k].reshape(-1).cpu().numpy()[g["gidx__" + k]]
        assert rel_err(gv, g["gval__" + k]) <= 2e-3, k
        dv = (params[k].detach() - before[k]).reshape(-1).cpu().numpy()[g["gidx__" + k]]
        assert np.mean(np.abs(dv - g["dval__" + k]) <= 2e-6) >= 0.98, k


@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("N,L,C,offset", [(3, 250, 256, 0.5), (48, 1000, 64, 40.0),
                                          (2, 254, 250, 0.5), (7, 1, 125, 1.0)])   # zero-padded channel groups
def test_batchnorm_vs_torch(gpu, training, relu, res, N, L, C, offset):
    """Also a many-chunk case with a large mean (the one-pass shifted-sum / Chan statistics)."""
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, C, L, generator=g) * 2 + offset
    r = torch.randn(N, C, L, generator=g)
    ref = torch.nn.BatchNorm1d(C)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.5, 0.5)
        ref.running_mean.uniform_(-0.1, 0.1)
        ref.running_var.uniform_(0.9, 1.1)
    mine = snn.BatchNorm1d(C).cuda()
    mine.load_state_dict(ref.state_dict())
    ref.train(training)
    mine.train(training)
    xr, rr = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
    yr = ref(xr)
    if res:
        yr = yr + rr
    gy = torch.randn(yr.shape, generator=g)
    if relu:
        # an element whose pre-activation is within fp32 rounding of 0 may fall on either side of
        # the relu mask (|x| ~ 40 leaves ~1e-5 absolute error in y): give those no gradient
        gy[yr.detach().abs() < 1e-4] = 0.0
        yr = torch.relu(yr)
    (yr * gy).sum().backward()
    xm = x.permute(0, 2, 1).contiguous().cuda().requires_grad_(True)
    rm = r.permute(0, 2, 1).contiguous().cuda().requires_grad_(True)
    ym = mine(xm, residual=rm if res else None, relu=relu)
    (ym * gy.permute(0, 2, 1).cuda()).sum().backward()
    assert rel_err(ym.detach().permute(0, 2, 1).cpu().numpy(), yr.detach().numpy()) <= 1e-5
    assert rel_err(xm.grad.permute(0, 2, 1).cpu().numpy(), xr.grad.numpy()) <= 1e-4
    if res:
        assert rel_err(rm.grad.permute(0, 2, 1).cpu().numpy(), rr.grad.numpy()) <= 1e-6
    assert rel_err(mine.weight.grad.cpu().numpy(), ref.weight.grad.numpy()) <= 1e-4
    assert rel_err(mine.bias.grad.cpu().numpy(), ref.bias.grad.numpy()) <= 1e-5
    assert rel_err(mine.running_mean.cpu().numpy(), ref.running_mean.numpy()) <= 1e-5
    assert rel_err(mine.running_var.cpu().numpy(), ref.running_var.numpy()) <= 1e-5


def test_resnet_bgru_vs_reference_golden(gpu):
    from speechrecognitionproject_amd.models import model_resnet_bgru
    g = golden("resnet_bgru_golden.npz")
    net = model_resnet_bgru.Network().cuda()
    net.load_state_dict(OM.seeded_state_dict(OM.ResnetBGRU(), 0))
    net.train(bool(g["train_mode"]))
    params = dict(net.named_parameters())
    opt = Adam([p for p in net.parameters() if p.requires_grad], lr=1e-4)
    opt.zero_grad()
    out = net(torch.from_numpy(g["pcm"]))
    loss = snn.CrossEntropyLoss()(out, torch.from_numpy(g["labels"]).cuda())
    loss.backward()
    assert rel_err(out.detach().cpu().numpy(), g["logits"]) <= LOGITS_REL
    assert abs(loss.item() - float(g["loss"])) <= 1e-4 * max(1.0, abs(float(g["loss"])))
    for k in g["names"]:
        gv = params[k].grad.reshape(-1).cpu().numpy()[g["gidx__" + k]]
        assert rel_err(gv, g["gval__" + k]) <= 5e-3, k


def test_resnet_bgru_mode1_vs_reference_golden(gpu):
    """The staged-training auxiliary head (model_resnet_bgru.py:57-71, 113-118, 147-149): the fc1
    output's time steps as the backend's channels, 250 / 125-channel BatchNorms on padded groups."""
    from speechrecognitionproject_amd.models import model_resnet_bgru
    g = golden("resnet_bgru_mode1_golden.npz")
    net = model_resnet_bgru.Network(mode=1).cuda()
    net.load_state_dict(OM.seeded_state_dict(OM.ResnetBGRU(mode=1), 0))
    net.train(bool(g["train_mode"]))
    params = dict(net.named_parameters())
    out = net(torch.from_numpy(g["pcm"]))
    assert out.shape == (len(g["pcm"]), 12)
    loss = snn.CrossEntropyLoss()(out, torch.from_numpy(g["labels"]).cuda())
    loss.backward()
    assert rel_err(out.detach().cpu().numpy(), g["logits"]) <= LOGITS_REL
    assert abs(loss.item() - float(g["loss"])) <= 1e-4 * max(1.0, abs(float(g["loss"])))
    assert all(p.grad is None for n, p in params.items() if n.startswith("gru."))   # the GRU is skipped
    for k in g["names"]:
        gv = params[k].grad.reshape(-1).cpu().numpy()[g["gidx__" + k]]
        if k == "resnet.backend_conv2.0.bias":
            # a bias feeding a training-mode BatchNorm has zero gradient (the batch mean absorbs it):
            # both sides hold rounding residue of size ~1e-7
            assert np.abs(gv).max() <= 1e-5 and np.abs(g["gval__" + k]).max() <= 1e-5, k
            continue
        assert rel_err(gv, g["gval__" + k]) <= 5e-3, k


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("N,H,W,Ci,Co,KH,KW,ph,pw", [(4, 98, 40, 64, 128, 1, 7, 0, 3), (2, 3, 8, 128, 64, 1, 7, 0, 3)])
def test_conv_pool_unpool16(gpu, prec, N, H, W, Ci, Co, KH, KW, ph, pw):
    """16-bit modes: the pooled conv's backward writing the dense dY straight as its 16-bit operand copy
    (option conv_unpool16 = 1: no dense fp32 dY, bias gradient from the pooled gradient) == the dense
    fp32 dY + 16-bit conversion path (0): the same rounded operands, so dx bitwise; db to fp32 summation
    order, and dW too for fbanks_cnn conv2's shape (its weight gradient on the row-staged
    conv_row16_wgrad_kernel from the pooled gradient: workgroup slabs reduced in order), bitwise otherwise."""
    from speechrecognitionproject_amd import _lib
    g = torch.Generator().manual_seed(N * 5 + Co + Ci)
    x = torch.randn(N, H, W, Ci, generator=g)
    w = torch.randn(Co, Ci, KH, KW, generator=g) / (Ci * KH * KW) ** 0.5
    b = torch.randn(Co, generator=g)
    Wo = W + 2 * pw - KW + 1
    gy = torch.randn(N, H + 2 * ph - KH + 1, Wo // 4, Co, generator=g).cuda()
    conv = snn.Conv2d(Ci, Co, (KH, KW), padding=(ph, pw)).cuda()
    pool = snn.MaxPool2d((1, 4))
    outs = []
    try:
        _lib.set_matmul_precision(prec)
        for u16 in (1, 0):
            _lib.set_option("conv_unpool16", u16)
            with torch.no_grad():
                conv.weight.copy_(w)
                conv.bias.copy_(b)
            conv.weight.grad = conv.bias.grad = None
            xm = x.cuda().requires_grad_(True)
            y = snn.conv_pool(xm, conv, pool)
            (y * gy).sum().backward()
            torch.cuda.synchronize()
            outs.append([t.detach().cpu() for t in (y, xm.grad, conv.weight.grad, conv.bias.grad)])
    finally:
        _lib.set_option("conv_unpool16", 1)
        _lib.set_matmul_precision("fp32")
    row_wgrad = (W, Ci, Co, KH, KW, ph, pw) == (40, 64, 128, 1, 7, 0, 3)
    for i, (a, c) in enumerate(zip(*outs)):
        assert torch.isfinite(a).all()
        if i == 3 or (i == 2 and row_wgrad):
            assert rel_err(a.numpy(), c.numpy()) <= 1e-5
        else:
            assert torch.equal(a, c), i


@pytest.mark.parametrize("N", [3, 32])
def test_conv_row32_equals_gemm(gpu, N):
    """Option conv_row32: fbanks_cnn conv2 + maxpool2 (Conv2d(64, 128, (1, 7), padding (0, 3)) over W = 40, then
    MaxPool2d((1, 4)), model_fbanks_cnn.py:74-75) on fp32 operands on the row-staged kernel — image rows staged
    once per tile, the weights streamed per tap, the taps as shifted reads — equals the implicit-GEMM kernel bit for
    bit: the same k-permuted 8-deep blocks of 32x32x2 MFMAs in the same (kw, ci) order, the same pooled epilogue.
    N = 3: a partial last tile (294 rows); N = 32: more tiles than CUs (the persistent tile loop).  NaN windows
    follow the pool rule."""
    from speechrecognitionproject_amd import nn as snn
    H, W, Ci, Co = 98, 40, 64, 128
    g = torch.Generator().manual_seed(N + 303)
    x = torch.randn(N, H, W, Ci, generator=g).cuda()
    w = (torch.randn(Co, Ci, 1, 7, generator=g) / (Ci * 7) ** 0.5).cuda()
    b = torch.randn(Co, generator=g).cuda()
    x[0, 0, :8] = float("nan")
    outs = []
    try:
        for row in (1, 0):
            _lib.set_option("conv_row32", row)
            _lib.prof_enable(True)
            with torch.no_grad():
                y = snn._ConvPoolNHWCFn.apply(x, w, b, (0, 3), 4)
            torch.cuda.synchronize()
            used = any("conv_row32" in e["kernel"] for e in _lib.prof_kernels())
            _lib.prof_enable(False)
            outs.append((y, used))
    finally:
        _lib.set_option("conv_row32", 1)
        _lib.prof_enable(False)
    (y1, u1), (y0, u0) = outs
    assert u1 and not u0
    nan = torch.isnan(y1)
    assert bool(nan.any()) and torch.equal(nan, torch.isnan(y0))
    assert torch.equal(y1[~nan], y0[~nan])
    # the backward (finite input): the argmax the gradients route through is the implicit GEMM's (weight and bias
    # gradients, on the same kernels either way, bitwise); the data gradient on the row-staged kernel
    # (conv_row32_dgrad_kernel: the pooled gradient unpooled at staging, k order (half, kw, co)) within 1e-5 of
    # the implicit GEMM's and of float64
    x[0, 0, :8] = 0.5
    gy = torch.randn(N, H, W // 4, Co, generator=g).cuda()
    grads = []
    try:
        for row in (1, 0):
            _lib.set_option("conv_row32", row)
            _lib.prof_enable(True)
            xm, wm, bm = (t.clone().requires_grad_(True) for t in (x, w, b))
            (snn._ConvPoolNHWCFn.apply(xm, wm, bm, (0, 3), 4) * gy).sum().backward()
            torch.cuda.synchronize()
            ks = [e["kernel"] for e in _lib.prof_kernels()]
            used = any("conv_row32_dgrad" in k for k in ks) and any("conv_row32_wgrad" in k for k in ks)
            _lib.prof_enable(False)
            grads.append((xm.grad, wm.grad, bm.grad, used))
    finally:
        _lib.set_option("conv_row32", 1)
        _lib.prof_enable(False)
    assert grads[0][3] and not grads[1][3]
    # every gradient on the row-staged kernels (data: conv_row32_dgrad_kernel; weight and bias:
    # conv_row32_wgrad_kernel, k = (workgroup's tiles, row, pixel pair), one slab per workgroup reduced in
    # order) within 1e-5 of the implicit GEMM's (another fp32 summation order) and of float64 below
    for a_, c_ in zip(grads[0][:3], grads[1][:3]):
        a_, c_ = a_.double(), c_.double()
        assert torch.isfinite(a_).all()
        assert ((a_ - c_).abs().max() / c_.abs().max()).item() <= 1e-5
    dx1, dx0 = grads[0][0].double(), grads[1][0].double()
    # float64 reference of the data gradient: unpool through the argmax, then conv_transpose
    with torch.no_grad():
        xd = x.double().permute(0, 3, 1, 2)
        wd = w.double()
        yd = torch.nn.functional.conv2d(xd, wd, b.double(), padding=(0, 3))     # [N, Co, H, W]
        win = yd.reshape(N, Co, H, W // 4, 4)
        am = win.argmax(-1, keepdim=True)
        dyd = torch.zeros_like(win).scatter_(-1, am, gy.double().permute(0, 3, 1, 2).unsqueeze(-1)).reshape(N, Co, H, W)
        dx64 = torch.nn.grad.conv2d_input(xd.shape, wd, dyd, padding=(0, 3)).permute(0, 2, 3, 1)
        dw64 = torch.nn.grad.conv2d_weight(xd, wd.shape, dyd, padding=(0, 3))
        db64 = dyd.sum((0, 2, 3))
    assert ((dx1 - dx64).abs().max() / dx64.abs().max()).item() <= 1e-5
    for got, ref in ((grads[0][1].double(), dw64), (grads[0][2].double(), db64)):
        assert ((got - ref).abs().max() / ref.abs().max()).item() <= 1e-5
    # deterministic: the same inputs give the same bits (fixed tile -> workgroup map, slabs reduced in order)
    xm, wm, bm = (t.clone().requires_grad_(True) for t in (x, w, b))
    (snn._ConvPoolNHWCFn.apply(xm, wm, bm, (0, 3), 4) * gy).sum().backward()
    assert torch.equal(wm.grad, grads[0][1]) and torch.equal(bm.grad, grads[0][2])


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("N", [3, 512])
def test_conv_full_width_fwd_gemm(gpu, prec, N):
    """fbanks_cnn conv3 (Conv2d(128, 256, (1, 10)) over width 10, model_fbanks_cnn.py:76): a full-width "valid" conv,
    whose forward runs as the plain GEMM x[(n, h)][(kw, ci)] . Wt + bias (option conv_fw_gemm) — within 1e-5 of the
    implicit GEMM (the same operands, rounded alike in bf16; another fp32 summation order) and, in fp32, of float64.
    N = 512: the cfg3 batch."""
    H, W, Ci, Co = 98, 10, 128, 256
    g = torch.Generator().manual_seed(N + 77)
    x = torch.randn(N, H, W, Ci, generator=g).cuda()
    w = (torch.randn(Co, Ci, 1, W, generator=g) / (Ci * W) ** 0.5).cuda()
    b = torch.randn(Co, generator=g).cuda()
    ys = []
    _lib.set_matmul_precision(prec)
    try:
        for on in (1, 0):
            _lib.set_option("conv_fw_gemm", on)
            _lib.prof_enable(True)
            with torch.no_grad():
                y = snn._Conv2dNHWCFn.apply(x, w, b, (0, 0), (1, 1))
            torch.cuda.synchronize()
            # the plain GEMM's launch (innermost profiling scope: M x N x K = N H x Co x W Ci)
            used = any(e["kernel"].startswith("gemm_") and "%dx%dx%d" % (N * H, Co, W * Ci) in e["kernel"]
                       for e in _lib.prof_kernels())
            _lib.prof_enable(False)
            ys.append((y.double(), used))
    finally:
        _lib.set_option("conv_fw_gemm", 1)
        _lib.set_matmul_precision("fp32")
        _lib.prof_enable(False)
    (y1, u1), (y0, u0) = ys
    assert u1 and not u0 and y1.shape == (N, H, 1, Co)
    assert torch.isfinite(y1).all()
    assert ((y1 - y0).abs().max() / y0.abs().max()).item() <= 1e-5
    if prec == "fp32":
        ref = F.conv2d(x.double().permute(0, 3, 1, 2), w.double(), b.double()).permute(0, 2, 3, 1)
        assert ((y1 - ref).abs().max() / ref.abs().max()).item() <= 1e-5
