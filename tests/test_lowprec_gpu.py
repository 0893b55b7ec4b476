"""Reduced-precision matrix-core mode (srk_set_option "matmul_precision" = bf16 / fp16;
BASELINE.json cfg2 "bf16", cfg5 "fp16 MFMA").

The kernels round their fp32 operands to bf16 / fp16 (nearest-even) on chip and accumulate in fp32,
so the oracle for ONE GEMM is exact: the same rounding done by torch on the host, then a float64
product.  Whole models are checked against the fp32 reference with the bf16/fp16 tolerance of
SURVEY.md Appendix A (logits <= 2e-2 relative), stated in tests/tolerances.py.
"""
import numpy as np
import pytest
import torch

from speechrecognitionproject_amd import _lib
from speechrecognitionproject_amd._lib import call
from speechrecognitionproject_amd.features import ptr, stream_ptr

pytestmark = pytest.mark.gpu

TORCH_DT = {"bf16": torch.bfloat16, "fp16": torch.float16}


@pytest.fixture(params=["bf16", "fp16"])
def prec(request, gpu):
    _lib.set_matmul_precision(request.param)
    yield request.param
    _lib.set_matmul_precision("fp32")


def _rounded(t, prec):
    return t.to(TORCH_DT[prec]).double()


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 29, 39), (130, 260, 70), (300, 129, 1024), (12, 1024, 4),
                                   (256, 128, 8192), (640, 384, 200)])
def test_gemm_lowprec_exact_rounding(prec, ta, tb, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g)
    opA = _rounded(A.T if ta else A, prec)
    opB = _rounded(B.T if tb else B, prec)
    ref = 0.5 * (opA @ opB) + 2.0 * C0.double() + bias.double()
    Ad, Bd, Cd, bd = A.cuda(), B.cuda(), C0.clone().cuda(), bias.cuda()
    call("srk_gemm_f32", ta, tb, M, N, K, 0.5, ptr(Ad), Ad.shape[1], ptr(Bd), Bd.shape[1], 2.0, ptr(Cd), N,
         ptr(bd), 1, stream_ptr())
    out = Cd.cpu().double()
    # only the fp32 accumulation order differs from the oracle
    scale = (opA.abs() @ opB.abs()).max().item()
    assert (out - ref).abs().max().item() <= 2e-6 * (1 + scale)


@pytest.mark.parametrize("M,N,K", [(12, 1024, 256), (1536, 512, 4000), (3072, 39, 13056)])
def test_gemm_lowprec_rowsum_is_fp32(prec, M, N, K):
    """dW = dY^T X with the bias gradient fused: the row sums come from the fp32 operand."""
    g = torch.Generator().manual_seed(K)
    dY = torch.randn(K, M, generator=g)          # stored [K][M] (trans_a)
    X = torch.randn(K, N, generator=g)
    dYd, Xd = dY.cuda(), X.cuda()
    dW = torch.empty(M, N, device="cuda")
    rs = torch.empty(M, device="cuda")
    call("srk_gemm_rowsum_f32", 1, 0, M, N, K, 1.0, ptr(dYd), M, ptr(Xd), N, 0.0, ptr(dW), N, ptr(rs), stream_ptr())
    ref = _rounded(dY.T, prec) @ _rounded(X, prec)
    scale = (_rounded(dY.T, prec).abs() @ _rounded(X, prec).abs()).max().item()
    assert (dW.cpu().double() - ref).abs().max().item() <= 2e-6 * (1 + scale)
    rref = dY.double().sum(0)
    assert (rs.cpu().double() - rref).abs().max().item() <= 1e-5 * (1 + dY.abs().sum(0).max().item())


def test_precision_option_validation(gpu):
    with pytest.raises(ValueError):
        _lib.set_matmul_precision("fp8")
    with pytest.raises(_lib.SrkError):
        _lib.set_option("matmul_precision", 3)
    assert _lib.matmul_precision() == "fp32"


# ----------------------------------------------------------------------------- GRU recurrence
def _emulate_bigru(x, sd, H, L, prec):
    """float64 BiGRU with the kernels' rounding: every matmul operand (x, W_ih, h_{t-1}, W_hh)
    rounded to `prec`; gates, cell update and outputs exact."""
    r = lambda t: _rounded(t, prec)
    h_in = x.double()
    B, T, _ = x.shape
    for layer in range(L):
        outs = []
        for sfx in ("", "_reverse"):
            w_ih, w_hh = sd["weight_ih_l%d%s" % (layer, sfx)], sd["weight_hh_l%d%s" % (layer, sfx)]
            b_ih, b_hh = sd["bias_ih_l%d%s" % (layer, sfx)].double(), sd["bias_hh_l%d%s" % (layer, sfx)].double()
            gi = r(h_in) @ r(w_ih).T + b_ih
            h = torch.zeros(B, H, dtype=torch.float64)
            ys = [None] * T
            for t in (range(T) if sfx == "" else reversed(range(T))):
                gh = r(h) @ r(w_hh).T + b_hh
                rg = torch.sigmoid(gi[:, t, :H] + gh[:, :H])
                zg = torch.sigmoid(gi[:, t, H:2 * H] + gh[:, H:2 * H])
                ng = torch.tanh(gi[:, t, 2 * H:] + rg * gh[:, 2 * H:])
                h = (1 - zg) * ng + zg * h
                ys[t] = h
            outs.append(torch.stack(ys, 1))
        h_in = torch.cat(outs, -1)
    return h_in


# B = 300 / 512: more rows than one persistent launch holds (256), so the recurrence runs as two
# batch-chunk launches (b_begin > 0) — the path cfg4 / cfg5 take at their per-GPU batch of 512
@pytest.mark.parametrize("B,T,IN,L", [(70, 9, 39, 2), (256, 6, 321, 1), (300, 5, 39, 2), (512, 4, 321, 1)])
def test_bigru_lowprec_forward_matches_emulation(prec, B, T, IN, L):
    from tolerances import GRU_LOWPREC_EMU_ABS
    from speechrecognitionproject_amd import nn as snn
    H = 512
    torch.manual_seed(3)
    ref = torch.nn.GRU(IN, H, num_layers=L, bidirectional=True, batch_first=True)
    sd = ref.state_dict()
    mine = snn.BiGRU(IN, H, num_layers=L).cuda()
    mine.load_state_dict(sd)
    x = torch.randn(B, T, IN)
    _lib.prof_enable(1)
    y, _ = mine(x.cuda())
    torch.cuda.synchronize()
    n_lp = _lib.prof_read("gru_fwd_seq_lp")[0]
    _lib.prof_enable(0)
    assert n_lp >= L, "the bf16/fp16 persistent recurrence did not run"
    emu = _emulate_bigru(x, sd, H, L, prec)
    err = (y.detach().cpu().double() - emu).abs().max().item()
    assert err <= GRU_LOWPREC_EMU_ABS, err
    assert _lib.spin_timeouts() == 0


@pytest.mark.parametrize("B", [96, 512])
def test_bigru_lowprec_grads_close_to_fp32(prec, B):
    from speechrecognitionproject_amd import nn as snn
    T, IN, H, L = 8, 39, 512, 2
    torch.manual_seed(4)
    ref = torch.nn.GRU(IN, H, num_layers=L, bidirectional=True, batch_first=True)
    mine = snn.BiGRU(IN, H, num_layers=L).cuda()
    mine.load_state_dict(ref.state_dict())
    x = torch.randn(B, T, IN)
    w = torch.randn(B, T, 2 * H)
    xr = x.clone().requires_grad_(True)
    (ref(xr)[0] * w).sum().backward()
    _lib.prof_enable(1)
    xm = x.cuda().requires_grad_(True)
    (mine(xm)[0] * w.cuda()).sum().backward()
    torch.cuda.synchronize()
    n_lp = _lib.prof_read("gru_bwd_seq_lp")[0]
    _lib.prof_enable(0)
    assert n_lp >= L
    refp = dict(ref.named_parameters())
    for n, p in mine.named_parameters():
        gr = refp[n].grad.double()
        err = ((p.grad.cpu().double() - gr).norm() / gr.norm()).item()
        assert err <= 2e-2, (n, err)
    gx = xr.grad.double()
    assert ((xm.grad.cpu().double() - gx).norm() / gx.norm()).item() <= 2e-2
    assert _lib.spin_timeouts() == 0


# ----------------------------------------------------------------------------- whole models
@pytest.mark.parametrize("name", ["mfcc_bgru", "spec_bgru", "fbanks_cnn", "resnet_bgru", "spec_cnn", "cnn_bgru",
                                  "mfrn_bgru"])
def test_model_lowprec_logits_vs_reference_golden(prec, name):
    import importlib
    from conftest import golden
    from oracle import models as OM
    from tolerances import LOGITS_REL_LOWPREC, rel_err
    from speechrecognitionproject_amd import nn as snn
    ocls = {"mfcc_bgru": OM.MfccBGRU, "spec_bgru": OM.SpecBGRU, "fbanks_cnn": OM.FbanksCNN,
            "resnet_bgru": OM.ResnetBGRU, "spec_cnn": OM.SpecCNN, "cnn_bgru": OM.CnnBGRU, "mfrn_bgru": OM.MfrnBGRU}[name]
    mod = importlib.import_module("speechrecognitionproject_amd.models.model_" + name)
    g = golden(name + "_golden.npz")
    net = mod.Network().cuda()
    net.load_state_dict(OM.seeded_state_dict(ocls(), 0))
    net.train(bool(g["train_mode"]))
    out = net(torch.from_numpy(g["pcm"]))
    loss = snn.CrossEntropyLoss()(out, torch.from_numpy(g["labels"]).cuda())
    loss.backward()
    assert rel_err(out.detach().cpu().numpy(), g["logits"]) <= LOGITS_REL_LOWPREC
    assert abs(loss.item() - float(g["loss"])) <= LOGITS_REL_LOWPREC * max(1.0, abs(float(g["loss"])))
    for p in net.parameters():
        assert p.grad is None or torch.isfinite(p.grad).all()


@pytest.mark.parametrize("name,precision,B", [("mfcc_bgru", "bf16", 256), ("spec_bgru", "fp16", 512),
                                              ("fbanks_cnn", "bf16", 512), ("spec_bgru", "bf16", 300)])
def test_model_lowprec_at_config_batch(gpu, name, precision, B):
    """BASELINE.json's configs at their own per-GPU batch (cfg2 bf16 B=256, cfg5 fp16 B=512, cfg3 in
    bf16 at B=512): logits of the 16-bit mode vs the fp32 CPU oracle (<= 2e-2) and vs the fp32 HIP
    path on the same clips; the fp32 HIP path vs the oracle per clip (tolerances.logits_ok: 1e-4,
    widened only by the reference's own float32 spread on spectrogram-fed clips); the persistent
    recurrence must not have timed out."""
    import importlib
    from oracle import models as OM
    from tolerances import LOGITS_REL_LOWPREC, logits_ok, rel_err, spec_reference_spread
    from speechrecognitionproject_amd.synthetic import synthetic_clips
    ocls = {"mfcc_bgru": OM.MfccBGRU, "spec_bgru": OM.SpecBGRU, "fbanks_cnn": OM.FbanksCNN}[name]
    mod = importlib.import_module("speechrecognitionproject_amd.models.model_" + name)
    sd = OM.seeded_state_dict(ocls(), 0)
    x, _ = synthetic_clips(B, seed=31, clip=30000)
    net = mod.Network().cuda().eval()
    net.load_state_dict(sd)
    ref = ocls()
    ref.load_state_dict(sd)
    with torch.no_grad():
        want = ref.eval()(torch.from_numpy(x)).numpy()
        xd = torch.from_numpy(x).cuda()
        fp32 = net(xd).cpu().numpy()
        try:
            _lib.set_matmul_precision(precision)
            lp = net(xd).cpu().numpy()
        finally:
            _lib.set_matmul_precision("fp32")
    spread = None
    if name.startswith("spec"):
        # the model half exactly: the oracle model fed the GPU's own spectrogram (each clip's
        # features are held to spec_ok by test_features_gpu.py) == the HIP logits at 1e-4
        from speechrecognitionproject_amd import features as K
        from tolerances import LOGITS_REL
        with torch.no_grad():
            gpu_feats = K.spec(xd).cpu()
            out, _ = ref.gru(gpu_feats.transpose(1, 2))
            model_only = ref.fc(out[:, -1, :]).numpy()
        assert rel_err(fp32, model_only) <= LOGITS_REL, rel_err(fp32, model_only)
        spread = spec_reference_spread(ref, x, want)
    ok, worst = logits_ok(fp32, want, spread)
    assert ok, worst
    assert rel_err(lp, want) <= LOGITS_REL_LOWPREC, rel_err(lp, want)
    assert rel_err(lp, fp32) <= LOGITS_REL_LOWPREC
    assert _lib.spin_timeouts() == 0


# ----------------------------------------------------------------------------- convolutions
CONV_LP = [  # N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw  (fbanks_cnn layers, resnet 1-D strided, odd edges)
    (2, 98, 40, 64, 128, 1, 7, 0, 3, 1, 1),
    (2, 98, 10, 128, 256, 1, 10, 0, 0, 1, 1),
    (3, 98, 1, 256, 512, 7, 1, 3, 0, 1, 1),
    (2, 9, 11, 5, 7, 3, 2, 1, 0, 1, 1),
    (4, 17, 13, 12, 36, 3, 3, 1, 1, 1, 1),
    (2, 1, 1000, 64, 128, 1, 15, 0, 7, 1, 2),
    (2, 1, 16000, 1, 64, 1, 80, 0, 38, 1, 16),
]


@pytest.mark.parametrize("shape", CONV_LP)
def test_conv_lowprec_exact_rounding(prec, shape):
    """Implicit-GEMM conv fwd / dgrad / wgrad with 16-bit operands == the float64 convolution of
    the host-rounded operands (x, w for fwd; dy, w for dgrad; x, dy for wgrad)."""
    import torch.nn.functional as F
    from speechrecognitionproject_amd import nn as snn
    N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw = shape
    g = torch.Generator().manual_seed(N * 100 + Co + KW)
    x = torch.randn(N, Ci, H, W, generator=g)
    w = torch.randn(Co, Ci, KH, KW, generator=g) / (Ci * KH * KW) ** 0.5
    b = torch.randn(Co, generator=g)
    xm = x.permute(0, 2, 3, 1).contiguous().cuda().requires_grad_(True)
    wm, bm = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    _lib.prof_enable(1)
    ym = snn._Conv2dNHWCFn.apply(xm, wm, bm, (ph, pw), (sh, sw))
    gy = torch.randn(ym.permute(0, 3, 1, 2).shape, generator=g)
    (ym * gy.permute(0, 2, 3, 1).cuda()).sum().backward()
    torch.cuda.synchronize()
    # (a full-width conv's forward runs as the plain 16-bit GEMM: profiled under its GEMM category)
    n_lp = sum(_lib.prof_read(c)[0] for c in ("conv_fwd_lp", "conv_wgrad_lp", "gemm_bf16", "gemm_f16"))
    _lib.prof_enable(0)
    assert n_lp >= 2, "the 16-bit conv kernels did not run"
    xr, wr, gr = _rounded(x, prec), _rounded(w, prec), _rounded(gy, prec)
    y_ref = F.conv2d(xr, wr, b.double(), stride=(sh, sw), padding=(ph, pw))
    dx_ref = torch.nn.grad.conv2d_input(x.shape, wr, gr, stride=(sh, sw), padding=(ph, pw))
    dw_ref = torch.nn.grad.conv2d_weight(xr, w.shape, gr, stride=(sh, sw), padding=(ph, pw))
    K = Ci * KH * KW

    def close(out, ref, k):
        # fp32 accumulation of k rounded products; only the summation order differs
        return (out.double() - ref).abs().max().item() <= 1e-5 * (1 + ref.abs().max().item()) * max(1.0, (k / 256) ** 0.5)

    assert close(ym.detach().permute(0, 3, 1, 2).cpu(), y_ref, K)
    assert close(xm.grad.permute(0, 3, 1, 2).cpu(), dx_ref, Co * KH * KW)
    assert close(wm.grad.cpu(), dw_ref, N * y_ref.shape[2] * y_ref.shape[3])


CONV_S16 = [  # 8-aligned channel counts: the pre-rounded 16-bit source path (option conv16_sources)
    (2, 98, 40, 64, 128, 1, 7, 0, 3, 1, 1),
    (3, 98, 1, 256, 512, 7, 1, 3, 0, 1, 1),
    (2, 1, 1000, 64, 128, 1, 15, 0, 7, 1, 2),   # strided: dgrad taps with no exact source
    (8, 1, 1000, 64, 64, 1, 15, 0, 7, 1, 1),    # wgrad K = 8000 pixels: split-K slabs
    (3, 1, 125, 512, 512, 1, 15, 0, 7, 1, 1),
    (2, 5, 7, 8, 24, 3, 3, 1, 1, 1, 1),         # partial 64-row / -column tiles
    (2, 1, 500, 128, 256, 1, 1, 0, 0, 1, 2),    # 1x1 downsample
]


@pytest.mark.parametrize("shape", CONV_S16)
def test_conv_16bit_sources_bit_identical(prec, shape):
    """bf16 / fp16 convs gathering from the pre-rounded 16-bit copy (conv16_sources = 1) give the
    SAME bits as rounding the fp32 gathers at LDS-store time (0): same rounding, same MFMA order.
    The bias gradient is the exception by design: the fp32-gather path sums it inside the
    weight-gradient kernel (conv_fused_db), the 16-bit-source path with the column-sum kernel — the
    same fp32 values in another order (1e-5).  (The 16-bit LDS-DMA ring kernels, conv_ring bits 4-6, read
    the 16-bit copies only: test_conv_16bit_ring holds them to these kernels.)"""
    from speechrecognitionproject_amd import nn as snn
    N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw = shape
    g = torch.Generator().manual_seed(N * 31 + Co + KW)
    x = torch.randn(N, H, W, Ci, generator=g).cuda()
    w = (torch.randn(Co, Ci, KH, KW, generator=g) / (Ci * KH * KW) ** 0.5).cuda()
    b = torch.randn(Co, generator=g).cuda()
    Ho, Wo = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
    gy = torch.randn(N, Ho, Wo, Co, generator=g).cuda()
    outs = []
    try:
        _lib.set_option("conv_ring", 6)   # the register-staged 16-bit kernels on both sides (no 16-bit ring)
        for on in (0, 1):
            _lib.set_option("conv16_sources", on)
            xm, wm, bm = (t.clone().requires_grad_(True) for t in (x, w, b))
            _lib.prof_enable(1)
            ym = snn._Conv2dNHWCFn.apply(xm, wm, bm, (ph, pw), (sh, sw))
            (ym * gy).sum().backward()
            torch.cuda.synchronize()
            assert (_lib.prof_read("conv_to16")[0] > 0) == bool(on)
            _lib.prof_enable(0)
            outs.append((ym.detach(), xm.grad, wm.grad, bm.grad))
    finally:
        _lib.set_option("conv16_sources", 1)
        _lib.set_option("conv_ring", 0x77)
        _lib.prof_enable(0)
    for a, c in zip(outs[0][:3], outs[1][:3]):
        assert torch.equal(a, c)
    db0, db1 = outs[0][3].double(), outs[1][3].double()
    assert ((db0 - db1).abs().max() / db1.abs().max()).item() <= 1e-5


@pytest.mark.parametrize("shape", CONV_S16[:4])
def test_conv_kept_16bit_copy_matches_plain_abi(prec, shape):
    """srk_conv2d_nhwc_fwd16 / bwd16 (the autograd path: the forward's 16-bit copy of x kept for the
    backward) == the plain srk_conv2d_nhwc_fwd / bwd pair called through the C ABI, bitwise; the
    backward rounds only dY (and the weights) once the copy is kept."""
    import ctypes
    N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw = shape
    g = torch.Generator().manual_seed(N * 7 + Ci + KH)
    x = torch.randn(N, H, W, Ci, generator=g).cuda()
    w = (torch.randn(Co, Ci, KH, KW, generator=g) / (Ci * KH * KW) ** 0.5).cuda()
    Ho, Wo = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
    dy = torch.randn(N, Ho, Wo, Co, generator=g).cuda()
    ws = torch.empty(Ci * Co * KH * KW, device="cuda")
    y0, dx0, dw0 = torch.empty_like(dy), torch.empty_like(x), torch.empty_like(w)
    call("srk_conv2d_nhwc_fwd", ptr(x), N, H, W, Ci, ptr(w), None, Co, KH, KW, ph, pw, sh, sw, ptr(y0), ptr(ws),
         stream_ptr())
    call("srk_conv2d_nhwc_bwd", ptr(x), N, H, W, Ci, ptr(w), Co, KH, KW, ph, pw, sh, sw, ptr(dy), ptr(dx0), ptr(dw0),
         None, ptr(ws), stream_ptr())
    x16 = torch.empty(x.numel(), device="cuda", dtype=torch.int16)
    written = ctypes.c_int(-1)
    y1, dx1, dw1 = torch.empty_like(dy), torch.empty_like(x), torch.empty_like(w)
    call("srk_conv2d_nhwc_fwd16", ptr(x), N, H, W, Ci, ptr(w), None, Co, KH, KW, ph, pw, sh, sw, ptr(y1), ptr(ws),
         ptr(x16), ctypes.byref(written), stream_ptr())
    assert written.value == 1
    x16_expect = x.reshape(-1).to(TORCH_DT[prec]).view(torch.int16)
    assert torch.equal(x16, x16_expect)   # round-to-nearest-even, as torch's cast
    _lib.prof_enable(1)
    call("srk_conv2d_nhwc_bwd16", ptr(x), N, H, W, Ci, ptr(w), Co, KH, KW, ph, pw, sh, sw, ptr(dy), ptr(dx1),
         ptr(dw1), None, ptr(ws), ptr(x16), stream_ptr())
    torch.cuda.synchronize()
    bytes_to16 = _lib.prof_read("conv_to16")[2]
    _lib.prof_enable(0)
    assert bytes_to16 == 6.0 * (dy.numel() + w.numel())   # dY and the dgrad weights; x not again
    for a, b in ((y0, y1), (dx0, dx1), (dw0, dw1)):
        assert torch.equal(a, b)


# ----------------------------------------------------------------------------- 16-bit operands in memory
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(8, 8, 8), (40, 24, 72), (136, 264, 200), (304, 128, 1024), (256, 128, 8192),
                                   (1000, 520, 64)])
def test_gemm_16bit_operands(prec, ta, tb, M, N, K):
    """srk_gemm_16: operands already bf16 / fp16 in memory == float64 product of those values."""
    g = torch.Generator().manual_seed(M * 5 + N * 3 + K)
    dt = TORCH_DT[prec]
    A = torch.randn((K, M) if ta else (M, K), generator=g).to(dt)
    B = torch.randn((N, K) if tb else (K, N), generator=g).to(dt)
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g)
    opA = (A.T if ta else A).double()
    opB = (B.T if tb else B).double()
    ref = 0.5 * (opA @ opB) + 2.0 * C0.double() + bias.double()
    Ad, Bd, Cd, bd = A.cuda(), B.cuda(), C0.clone().cuda(), bias.cuda()
    _lib.prof_enable(1)
    call("srk_gemm_16", ta, tb, M, N, K, 0.5, ptr(Ad), Ad.shape[1], ptr(Bd), Bd.shape[1], 2.0, ptr(Cd), N,
         ptr(bd), 1, stream_ptr())
    torch.cuda.synchronize()
    assert _lib.prof_read("gemm_f16" if prec == "fp16" else "gemm_bf16")[0] == 1
    _lib.prof_enable(0)
    scale = (opA.abs() @ opB.abs()).max().item()
    assert (Cd.cpu().double() - ref).abs().max().item() <= 2e-6 * (1 + scale)


@pytest.mark.parametrize("kernel", [1, 2])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0)])
@pytest.mark.parametrize("M,N,K", [(1288, 776, 1352), (1032, 264, 4104), (2048, 512, 64), (1536, 1024, 1000)])
def test_gemm_16bit_kernels_at_tile_edges(prec, kernel, ta, tb, M, N, K):
    """Both 16-bit-operand GEMM kernels (register-staged / LDS-DMA ping-pong, srk option
    gemm16_kernel) on shapes with partial 256-row / -column tiles, k tails (K % 64 != 0),
    split-K and a single K-tile == float64 product of the 16-bit values."""
    g = torch.Generator().manual_seed(M + 7 * N + 11 * K + ta)
    dt = TORCH_DT[prec]
    A = torch.randn((K, M) if ta else (M, K), generator=g).to(dt)
    B = torch.randn((N, K) if tb else (K, N), generator=g).to(dt)
    C0 = torch.randn(M, N, generator=g)
    opA = (A.T if ta else A).double()
    opB = (B.T if tb else B).double()
    ref = opA @ opB + C0.double()
    Ad, Bd, Cd = A.cuda(), B.cuda(), C0.clone().cuda()
    _lib.set_option("gemm16_kernel", kernel)
    try:
        call("srk_gemm_16", ta, tb, M, N, K, 1.0, ptr(Ad), Ad.shape[1], ptr(Bd), Bd.shape[1], 1.0, ptr(Cd), N,
             None, 0, stream_ptr())
        torch.cuda.synchronize()
    finally:
        _lib.set_option("gemm16_kernel", 0)
    scale = (opA.abs() @ opB.abs()).max().item()
    assert (Cd.cpu().double() - ref).abs().max().item() <= 2e-6 * (1 + scale)


@pytest.mark.parametrize("ta,tb", [(1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("M,N,K,batch", [(1536, 512, 4095, 2), (264, 136, 1032, 3), (1024, 256, 64, 2)])
def test_gemm_16bit_batched(prec, ta, tb, M, N, K, batch):
    """srk_gemm_16_batched (the BiGRU backward's batch-2 dW_hh launch; split-K slabs per batch) ==
    float64 product of the 16-bit values, batch by batch, on strided views of one buffer."""
    if (not ta or tb) and K % 8:   # a k-contiguous operand needs rows of 8-element multiples
        K += 8 - K % 8
    g = torch.Generator().manual_seed(M + 3 * N + 5 * K + batch)
    dt = TORCH_DT[prec]
    ra, ca = (K, M) if ta else (M, K)
    rb, cb = (N, K) if tb else (K, N)
    sA, sB, sC = ra * ca + 24, rb * cb + 8, M * N + 4     # padded strides (multiples of 8 / 4)
    A = torch.randn(batch * sA, generator=g).to(dt)
    B = torch.randn(batch * sB, generator=g).to(dt)
    C0 = torch.randn(batch * sC, generator=g)
    Ad, Bd, Cd = A.cuda(), B.cuda(), C0.clone().cuda()
    call("srk_gemm_16_batched", ta, tb, M, N, K, 1.0, ptr(Ad), ca, sA, ptr(Bd), cb, sB, 1.0, ptr(Cd), N, sC, batch,
         stream_ptr())
    torch.cuda.synchronize()
    out = Cd.cpu().double()
    for z in range(batch):
        a = A[z * sA:z * sA + ra * ca].view(ra, ca).double()
        b = B[z * sB:z * sB + rb * cb].view(rb, cb).double()
        opA, opB = (a.T if ta else a), (b.T if tb else b)
        ref = opA @ opB + C0[z * sC:z * sC + M * N].view(M, N).double()
        scale = (opA.abs() @ opB.abs()).max().item()
        assert (out[z * sC:z * sC + M * N].view(M, N) - ref).abs().max().item() <= 2e-6 * (1 + scale), z
        assert torch.equal(out[z * sC + M * N:(z + 1) * sC], C0[z * sC + M * N:(z + 1) * sC].double())  # gaps


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16"])
def test_bigru_batched_dwhh_matches_per_direction(gpu, precision):
    """The batch-2 dW_hh launch (option gru_dwhh_batched, default; fp32: the ping-pong kernel with the
    fused bias-gradient row sums per batch) == one launch per direction up to fp32 split-K summation
    order; every other gradient is bitwise identical."""
    from speechrecognitionproject_amd import nn as snn
    _lib.set_matmul_precision(precision)
    try:
        _batched_dwhh_case(snn)
    finally:
        _lib.set_matmul_precision("fp32")


def _batched_dwhh_case(snn):
    B, T, IN, H = 256, 20, 39, 512
    torch.manual_seed(7)
    mine = snn.BiGRU(IN, H, num_layers=2).cuda()
    x = torch.randn(B, T, IN, device="cuda")
    w = torch.randn(B, T, 2 * H, device="cuda")
    grads = []
    for batched in (1, 0):
        _lib.set_option("gru_dwhh_batched", batched)
        try:
            for p in mine.parameters():
                p.grad = None
            (mine(x)[0] * w).sum().backward()
            torch.cuda.synchronize()
        finally:
            _lib.set_option("gru_dwhh_batched", 1)
        grads.append({n: p.grad.detach().clone() for n, p in mine.named_parameters()})
    for n in grads[0]:
        a, b = grads[0][n], grads[1][n]
        if "_hh" in n:   # weight_hh (split order) and bias_hh (the fp32 path's fused row sums)
            assert ((a - b).norm() / b.norm()).item() <= 1e-5, n
        else:
            assert torch.equal(a, b), n
    assert _lib.spin_timeouts() == 0


def test_gemm_16bit_rejects_misaligned(prec):
    A = torch.zeros(16, 12, dtype=TORCH_DT[prec], device="cuda")
    C = torch.zeros(16, 16, device="cuda")
    with pytest.raises(_lib.SrkError):
        call("srk_gemm_16", 0, 1, 16, 16, 12, 1.0, ptr(A), 12, ptr(A), 12, 0.0, ptr(C), 16, None, 0, stream_ptr())


@pytest.mark.parametrize("precision,H,opts", [("bf16", 128, {}), ("fp16", 128, {}), ("bf16", 512, {"gru_persistent": 0}),
                                              ("fp32", 128, {"gemm32_kernel": 1})])
def test_bigru_backward_when_batched_dwhh_is_unavailable(gpu, precision, H, opts):
    """the batched dW_hh launch (both directions in one GEMM with fused row sums) exists
    only on the fp32-operand ping-pong kernel.  The fp32-operand GRU backward that 16-bit mode takes
    without the persistent kernels (H != 512, gru_persistent=0), and fp32 with the register-staged
    kernel forced, must fall back to per-direction launches: same gradients as gru_dwhh_batched=0."""
    from speechrecognitionproject_amd import nn as snn
    B, T, IN, L = 24, 7, 39, 2
    torch.manual_seed(5)
    ref = torch.nn.GRU(IN, H, num_layers=L, bidirectional=True, batch_first=True)
    x = torch.randn(B, T, IN, device="cuda")
    w = torch.randn(B, T, 2 * H, device="cuda")
    grads = []
    try:
        _lib.set_matmul_precision(precision)
        for k, v in opts.items():
            _lib.set_option(k, v)
        for batched in (1, 0):
            _lib.set_option("gru_dwhh_batched", batched)
            mine = snn.BiGRU(IN, H, num_layers=L).cuda()
            mine.load_state_dict(ref.state_dict())
            (mine(x)[0] * w).sum().backward()
            torch.cuda.synchronize()
            grads.append({n: p.grad.detach().clone() for n, p in mine.named_parameters()})
    finally:
        _lib.set_option("gru_dwhh_batched", 1)
        _lib.set_option("gru_persistent", 1)
        _lib.set_option("gemm32_kernel", 0)
        _lib.set_matmul_precision("fp32")
    for n in grads[0]:
        assert torch.isfinite(grads[0][n]).all(), n
        assert torch.equal(grads[0][n], grads[1][n]), n


@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0)])
@pytest.mark.parametrize("M,N,K,beta", [(5120, 3328, 520, 0.0), (1304, 712, 2056, 2.0), (2560, 2560, 8, 0.0),
                                        (5120, 3328, 512, 1.0)])
def test_gemm16_pingpong(prec, ta, tb, M, N, K, beta):
    """The 16-bit ping-pong GEMM (gemm16_kernel = 2) == float64 of the 16-bit values (k tails: 520, 8;
    row / column edges: 1304 x 712; split-K: 2056; more than one round of tiles: 5120 x 3328) and == the
    register-staged 16-bit kernel up to the fp32 summation order."""
    g = torch.Generator().manual_seed(M + 3 * N + K + tb)
    dt = TORCH_DT[prec]
    A = torch.randn((K, M) if ta else (M, K), generator=g).to(dt)
    B = torch.randn((N, K) if tb else (K, N), generator=g).to(dt)
    C0 = torch.randn(M, N, generator=g)
    opA = (A.T if ta else A).double()
    opB = (B.T if tb else B).double()
    ref = 0.5 * (opA @ opB) + beta * C0.double()
    Ad, Bd = A.cuda(), B.cuda()
    outs = []
    try:
        for kern in (2, 1):
            _lib.set_option("gemm16_kernel", kern)
            Cd = C0.clone().cuda()
            call("srk_gemm_16", ta, tb, M, N, K, 0.5, ptr(Ad), Ad.shape[1], ptr(Bd), Bd.shape[1], beta, ptr(Cd), N,
                 None, 0, stream_ptr())
            outs.append(Cd.cpu().double())
    finally:
        _lib.set_option("gemm16_kernel", 0)
    scale = (opA.abs() @ opB.abs()).max().item()
    assert (outs[0] - ref).abs().max().item() <= 2e-6 * (1 + scale)
    assert (outs[0] - outs[1]).abs().max().item() <= 2e-6 * (1 + scale)


@pytest.mark.parametrize("shape", [(2, 98, 40, 64, 128, 1, 7, 0, 3), (3, 98, 1, 256, 512, 7, 1, 3, 0),
                                   (2, 1, 1000, 64, 128, 1, 15, 0, 7, 1, 2), (4, 17, 13, 32, 256, 3, 3, 1, 1),
                                   # more tiles than CUs (fwd 256 x 128; fwd + dgrad 256 x 256)
                                   (32, 98, 40, 64, 128, 1, 7, 0, 3), (68, 1, 500, 256, 512, 1, 15, 0, 7)])
def test_conv_16bit_ring(prec, shape):
    """srk option conv_ring bits 4-6: the 16-bit LDS-DMA ring convolutions (gemm_g16_kernel's
    structure, per-K-tile conv gathers of the 16-bit operand copies) == the register-staged 16-bit
    conv kernels on the same rounded operands up to the fp32 summation order, forward and backward."""
    from speechrecognitionproject_amd import nn as snn
    N, H, W, Ci, Co, KH, KW, ph, pw = shape[:9]
    sh, sw = (shape[9], shape[10]) if len(shape) > 9 else (1, 1)
    g = torch.Generator().manual_seed(N * 13 + Co + KW)
    x = torch.randn(N, H, W, Ci, generator=g).cuda()
    w = (torch.randn(Co, Ci, KH, KW, generator=g) / (Ci * KH * KW) ** 0.5).cuda()
    b = torch.randn(Co, generator=g).cuda()
    Ho, Wo = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
    gy = torch.randn(N, Ho, Wo, Co, generator=g).cuda()
    outs = []
    try:
        # ring (one k-step per MFMA section), ring with whole K-tiles per section (conv_ring_qs, every width),
        # register-staged
        for mask, qs in ((0x70 | 6, 0), (0x70 | 6, 7), (6, 0)):
            _lib.set_option("conv_ring", mask)
            _lib.set_option("conv_ring_qs", qs)
            xm, wm, bm = (t.clone().requires_grad_(True) for t in (x, w, b))
            ym = snn._Conv2dNHWCFn.apply(xm, wm, bm, (ph, pw), (sh, sw))
            (ym * gy).sum().backward()
            torch.cuda.synchronize()
            outs.append([t.detach().double() for t in (ym, xm.grad, wm.grad, bm.grad)])
    finally:
        _lib.set_option("conv_ring", 0x77)
        _lib.set_option("conv_ring_qs", 6)
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)   # the same MFMA order per accumulator
    for a, c in zip(outs[0], outs[2]):
        assert ((a - c).abs().max() / c.abs().max()).item() <= 1e-5


@pytest.mark.parametrize("B,T,IN,wide", [(256, 51, 39, 1), (256, 9, 1024, 1), (200, 6, 39, 1), (300, 5, 1024, 0),
                                         (64, 2, 24, 1)])
def test_bigru_dwhh_fused_matches_gemm(prec, B, T, IN, wide):
    """Option gru_dwhh_fused: the 16-bit backward recurrence kernel accumulates dW_hh itself (4 extra
    worker waves, dg_t^T h_prev on the matrix cores after each step's publish, per-(chunk, row group)
    partials summed in order) instead of the batched GEMM over dgh16 / y16.  Same rounded operands, other
    fp32 summation order: dW_hh within 1e-5 of the GEMM path norm-wise, every
    other gradient and the output unchanged.  Shapes: the cfg2 layer-0 (fused projection) and layer-1
    inputs, a partial last row group, two 256-row chunks (64-row workgroups off), T = 2."""
    from speechrecognitionproject_amd import nn as snn
    H = 512
    torch.manual_seed(11)
    mine = snn.BiGRU(IN, H, num_layers=1).cuda()
    x = torch.randn(B, T, IN, device="cuda")
    w = torch.randn(B, T, 2 * H, device="cuda")
    res = []
    try:
        _lib.set_matmul_precision(prec)
        _lib.set_option("gru_lp_wide", wide)
        for fused in (1, 0, 3, 5, 7):   # 3 / 5 / 7: the h_prev fetch / priority timing variants, bitwise mode 1
            _lib.set_option("gru_dwhh_fused", fused)
            mine.zero_grad()
            xm = x.clone().requires_grad_(True)
            _lib.prof_enable(True)
            ym, _ = mine(xm)
            (ym * w).sum().backward()
            torch.cuda.synchronize()
            kinds = [k["kernel"] for k in _lib.prof_kernels()]
            _lib.prof_enable(False)
            if fused:   # the fused kernel ran and no dW_hh GEMM did
                assert any("_lp2dw" in k for k in kinds), kinds
                assert not any("1536x512" in k for k in kinds), kinds
            res.append({"y": ym.detach().clone(), "dx": xm.grad.clone(),
                        **{n: p.grad.detach().clone() for n, p in mine.named_parameters()}})
    finally:
        _lib.set_option("gru_dwhh_fused", 1)
        _lib.set_option("gru_lp_wide", 1)
        _lib.set_matmul_precision("fp32")
    assert _lib.spin_timeouts() == 0
    for v in res[2:]:
        for n in res[0]:
            assert torch.equal(res[0][n], v[n]), n
    for n in res[0]:
        a, b = res[0][n], res[1][n]
        assert torch.isfinite(a).all(), n
        if "weight_hh" in n:
            # two fp32 summation orders of up to B (T - 1) = 12.8k products of either sign (GEMM: 32-deep
            # k-tiles in 10 split-K slabs; fused: 32-row MFMA k-steps accumulated over T, then 8 row-group
            # partials); element-wise the cancellation amplifies that (measured up to 3.3e-5 of the largest
            # element, fp16 at B = 200, T = 6), so the bound is norm-wise; a missing or doubled row group /
            # step would be O(1e-1)
            err = float((a - b).norm() / b.norm())
            assert err <= 1e-5, (n, err)
        else:
            assert torch.equal(a, b), n


@pytest.mark.parametrize("B,T,IN", [(256, 51, 39), (256, 9, 1024), (200, 6, 1024), (96, 3, 39), (64, 2, 1024), (32, 1, 1024)])
def test_bigru_fwd_worker(prec, B, T, IN):
    """Option gru_fwd_worker: the 16-bit forward recurrence with 4 worker waves that store y / y16 / the
    gates from LDS after each publish and (no fused projection) fetch gi two steps ahead by LDS-DMA,
    against the kernel without them.  The same source arithmetic in a separately compiled instantiation
    (the compiler's multiply-add contraction in the cell may differ, as between the 64- and 32-row
    kernels, test_bigru_lowprec_wide_matches_chunked): step 0 of each direction bitwise, outputs within
    5e-4, gradients 2e-3 norm-wise (the backward reads the gates / y16 the workers wrote), each mode
    bitwise reproducible.  Shapes: the cfg2 layer-0 (fused projection) and layer-1 inputs, a partial row
    group, and T = 1..3 (the workers' DMA / wait counts at the sequence edges)."""
    from speechrecognitionproject_amd import nn as snn
    H = 512
    torch.manual_seed(12)
    mine = snn.BiGRU(IN, H, num_layers=1).cuda()
    x = torch.randn(B, T, IN, device="cuda")
    w = torch.randn(B, T, 2 * H, device="cuda")
    res = []
    try:
        _lib.set_matmul_precision(prec)
        for ow in (1, 1, 0):
            _lib.set_option("gru_fwd_worker", ow)
            mine.zero_grad()
            xm = x.clone().requires_grad_(True)
            _lib.prof_enable(True)
            ym, _ = mine(xm)
            (ym * w).sum().backward()
            torch.cuda.synchronize()
            kinds = [k["kernel"] for k in _lib.prof_kernels()]
            _lib.prof_enable(False)
            assert any("_lp2ow" in k for k in kinds) == bool(ow), kinds
            res.append({"y": ym.detach().clone(), "dx": xm.grad.clone(),
                        **{n: p.grad.detach().clone() for n, p in mine.named_parameters()}})
    finally:
        _lib.set_option("gru_fwd_worker", 0)
        _lib.set_matmul_precision("fp32")
    assert _lib.spin_timeouts() == 0
    a, a2, c = res
    for n in a:
        assert torch.isfinite(a[n]).all(), n
        assert torch.equal(a[n], a2[n]), n
    assert torch.equal(a["y"][:, 0, :H], c["y"][:, 0, :H]) and torch.equal(a["y"][:, -1, H:], c["y"][:, -1, H:])
    assert float((a["y"] - c["y"]).abs().max()) <= 5e-4
    for n in a:
        if n == "y":
            continue
        if float(c[n].norm()) == 0.0:   # T = 1: h_prev = 0, so dW_hh is exactly zero on both paths
            assert torch.equal(a[n], c[n]), n
            continue
        err = float((a[n] - c[n]).norm() / c[n].norm())
        assert err <= 2e-3, (n, err)


@pytest.mark.parametrize("shape", CONV_S16 + [(3, 17, 24, 128, 64, 3, 3, 1, 1, 1, 1), (5, 98, 40, 64, 128, 1, 7, 0, 3, 1, 1)])
@pytest.mark.parametrize("pooled", [False, True])
def test_conv_fast16_gathers_bitwise(prec, shape, pooled):
    """Option conv_fast16: the register-staged 16-bit-source convs gathering one uniform tap per K-tile
    (channels a multiple of the 64-deep K-tile) through per-row base offsets and zero-filling buffer loads ==
    the generic gathers (per-unit tap splits, masks at LDS-store time), bit for bit — forward (plain and with the
    fused (1, 4) max pool), data and weight gradients; the register-staged kernels on both sides (no ring)."""
    from speechrecognitionproject_amd import nn as snn
    N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw = shape
    Ho, Wo = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
    if pooled and (sh != 1 or sw != 1 or Wo % 4):
        pytest.skip("the fused pool needs stride 1 and Wo % 4 == 0")
    g = torch.Generator().manual_seed(N * 29 + Co + KW + int(pooled))
    x = torch.randn(N, H, W, Ci, generator=g).cuda()
    w = (torch.randn(Co, Ci, KH, KW, generator=g) / (Ci * KH * KW) ** 0.5).cuda()
    b = torch.randn(Co, generator=g).cuda()
    gy = torch.randn(N, Ho, Wo // 4 if pooled else Wo, Co, generator=g).cuda()
    outs = []
    try:
        _lib.set_option("conv_ring", 6)
        for fast in (1, 0):
            _lib.set_option("conv_fast16", fast)
            xm, wm, bm = (t.clone().requires_grad_(True) for t in (x, w, b))
            if pooled:
                ym = snn._ConvPoolNHWCFn.apply(xm, wm, bm, (ph, pw), 4)
            else:
                ym = snn._Conv2dNHWCFn.apply(xm, wm, bm, (ph, pw), (sh, sw))
            (ym * gy).sum().backward()
            torch.cuda.synchronize()
            outs.append((ym.detach(), xm.grad, wm.grad, bm.grad))
    finally:
        _lib.set_option("conv_fast16", 1)
        _lib.set_option("conv_ring", 0x77)
    for a, c in zip(*outs):
        assert torch.isfinite(a).all()
        assert torch.equal(a, c)


@pytest.mark.parametrize("N", [3, 32])
@pytest.mark.parametrize("form", [1, 2])   # 8 waves / 4 waves (forward); the data gradient's two splits with them
def test_conv_row16_equals_gemm(prec, N, form):
    """Option conv_row16: fbanks_cnn conv2 + maxpool2 (Conv2d(64, 128, (1, 7), padding (0, 3)) over W = 40, then
    MaxPool2d((1, 4)), model_fbanks_cnn.py:74-75) on the row-staged kernel — weights resident in LDS, image rows
    staged once per tile, the taps as shifted reads — equals the implicit-GEMM kernels bit for bit: the same
    16-bit operands in the same k order.  N = 3: a partial last tile (294 rows); N = 32: more tiles than CUs
    (the persistent loop with the register prefetch of the next tile)."""
    from speechrecognitionproject_amd import nn as snn
    H, W, Ci, Co = 98, 40, 64, 128
    g = torch.Generator().manual_seed(N + 101)
    x = torch.randn(N, H, W, Ci, generator=g).cuda()
    w = (torch.randn(Co, Ci, 1, 7, generator=g) / (Ci * 7) ** 0.5).cuda()
    b = torch.randn(Co, generator=g).cuda()
    x[0, 0, :8] = float("nan")   # NaN windows: the pool rule
    outs = []
    try:
        for row in (form, 0):
            _lib.set_option("conv_row16", row)
            _lib.prof_enable(True)
            with torch.no_grad():
                y = snn._ConvPoolNHWCFn.apply(x, w, b, (0, 3), 4)
            torch.cuda.synchronize()
            used = any("conv_row16" in e["kernel"] for e in _lib.prof_kernels())
            _lib.prof_enable(False)
            outs.append((y, used))
    finally:
        _lib.set_option("conv_row16", 1)
        _lib.prof_enable(False)
    (y1, u1), (y0, u0) = outs
    assert u1 and not u0
    nan = torch.isnan(y1)
    assert bool(nan.any()) and torch.equal(nan, torch.isnan(y0))
    assert torch.equal(y1[~nan], y0[~nan])
    # the argmax the backward routes through: every gradient equal too (finite input), the data gradient on the
    # row-staged kernel (option conv_row16_dgrad) against the implicit GEMM's; then the plain conv's backward
    # with a dense dY through the same hook
    x[0, 0, :8] = 0.5
    gy = torch.randn(N, H, W // 4, Co, generator=g).cuda()
    gd = torch.randn(N, H, W, Co, generator=g).cuda()
    grads, dense = [], []
    try:
        for row in (form, 0):
            _lib.set_option("conv_row16", row)
            _lib.set_option("conv_row16_dgrad", form if row else 0)
            _lib.prof_enable(True)
            xm, wm, bm = (t.clone().requires_grad_(True) for t in (x, w, b))
            (snn._ConvPoolNHWCFn.apply(xm, wm, bm, (0, 3), 4) * gy).sum().backward()
            torch.cuda.synchronize()
            ks = [e["kernel"] for e in _lib.prof_kernels()]
            grads.append((xm.grad, wm.grad, bm.grad, any("conv_row16_dgrad" in k for k in ks),
                          any("conv_row16_wgrad" in k for k in ks)))
            _lib.prof_enable(False)
            xm, wm, bm = (t.clone().requires_grad_(True) for t in (x, w, b))
            (snn._Conv2dNHWCFn.apply(xm, wm, bm, (0, 3), (1, 1)) * gd).sum().backward()
            torch.cuda.synchronize()
            dense.append((xm.grad, wm.grad, bm.grad))
    finally:
        _lib.set_option("conv_row16", 1)
        _lib.set_option("conv_row16_dgrad", 2)
        _lib.prof_enable(False)
    assert grads[0][3] and not grads[1][3] and grads[0][4] and not grads[1][4]
    # the data gradient and the dense-dY conv's gradients bitwise; the pooled conv's weight and bias gradients on
    # the row-staged conv_row16_wgrad_kernel (the same 16-bit operands — x's copy, dY unpooled and rounded at
    # staging — in another fp32 summation order: workgroup slabs reduced in order) within 1e-5 of the implicit GEMM's
    for a_, c_ in [(grads[0][0], grads[1][0])] + list(zip(*dense)):
        assert torch.isfinite(a_).all() and torch.equal(a_, c_)
    for a_, c_ in zip(grads[0][1:3], grads[1][1:3]):
        a_, c_ = a_.double(), c_.double()
        assert torch.isfinite(a_).all()
        assert ((a_ - c_).abs().max() / c_.abs().max()).item() <= 1e-5
