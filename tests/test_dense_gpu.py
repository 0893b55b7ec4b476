"""GEMM / GRU / Linear / cross-entropy / Adam kernels vs plain PyTorch fp32 (CPU) references."""
import numpy as np
import pytest
import torch

from speechrecognitionproject_amd import nn as snn
from speechrecognitionproject_amd._lib import call
from speechrecognitionproject_amd.features import ptr, stream_ptr
from speechrecognitionproject_amd.optim import Adam, FlatParams

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 29, 39), (130, 260, 70), (300, 129, 1024), (12, 1024, 4)])
def test_gemm_f32(gpu, ta, tb, M, N, K):
    g = torch.Generator().manual_seed(M * 1000 + N + K)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g)
    ref = 0.5 * ((A.T if ta else A).double() @ (B.T if tb else B).double()) + 2.0 * C0.double() + bias.double()
    Ad, Bd, Cd, bd = A.cuda(), B.cuda(), C0.clone().cuda(), bias.cuda()
    call("srk_gemm_f32", ta, tb, M, N, K, 0.5, ptr(Ad), Ad.shape[1], ptr(Bd), Bd.shape[1], 2.0, ptr(Cd), N,
         ptr(bd), 1, stream_ptr())
    out = Cd.cpu().double()
    assert (out - ref).abs().max() <= 1e-5 * (1 + (A.abs().max() * B.abs().max() * K).item())


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("ta,tb,M,N,K", [
    (0, 1, 256, 12, 1024), (0, 0, 256, 12, 1024), (0, 1, 5, 1, 3), (0, 0, 1000, 16, 4097),   # N <= 16, A k-contiguous
    (1, 0, 12, 1024, 256), (0, 0, 16, 777, 300), (1, 0, 1, 5, 1),                            # M <= 16, B row-contiguous
    (0, 0, 256, 1024, 12), (1, 0, 300, 515, 16), (0, 0, 70, 9, 1),                           # K <= 16
    # every model's 12-class classifier at the configs' batches (forward, dW + db, dx):
    # fbanks_cnn fc2 (in 256) and the BiGRU heads (in 1024) at B = 512
    (0, 1, 512, 12, 256), (1, 0, 12, 256, 512), (0, 0, 512, 256, 12),
    (0, 1, 512, 12, 1024), (1, 0, 12, 1024, 512), (0, 0, 512, 1024, 12)])
def test_gemm_skinny(gpu, precision, ta, tb, M, N, K):
    """GEMMs with a dimension <= 16 (the output layers' fc GEMMs) on the VALU skinny kernels (option
    gemm_skinny): == float64 product of the (rounded, in bf16 / fp16 mode) operands with alpha, beta,
    bias, and the fused row sums of the UNROUNDED op(A); == the matrix-core tile path within fp32
    summation order."""
    from speechrecognitionproject_amd import _lib
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K + ta)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g)
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[precision]
    opA, opB = (A.T if ta else A), (B.T if tb else B)
    ref = 0.5 * (opA.to(dt).double() @ opB.to(dt).double()) + 2.0 * C0.double() + bias.double()
    tol = 2e-6 * (1 + (opA.abs().double() @ opB.abs().double()).max().item())
    Ad, Bd = A.cuda(), B.cuda()
    _lib.set_matmul_precision(precision)
    outs = []
    try:
        for skinny in (1, 0):
            _lib.set_option("gemm_skinny", skinny)
            _lib.prof_enable(1)
            Cd = C0.clone().cuda()
            call("srk_gemm_f32", ta, tb, M, N, K, 0.5, ptr(Ad), Ad.shape[1], ptr(Bd), Bd.shape[1], 2.0, ptr(Cd), N,
                 ptr(bias.cuda()), 1, stream_ptr())
            rs = torch.full((M,), 3.0, device="cuda")
            Cr = torch.zeros(M, N, device="cuda")
            call("srk_gemm_rowsum_f32", ta, tb, M, N, K, 1.0, ptr(Ad), Ad.shape[1], ptr(Bd), Bd.shape[1], 0.0,
                 ptr(Cr), N, ptr(rs), stream_ptr())
            torch.cuda.synchronize()
            kinds = [k["kernel"] for k in _lib.prof_kernels()]
            _lib.prof_enable(0)
            assert all(("skinny" in k) == bool(skinny) for k in kinds), kinds
            outs.append((Cd.cpu().double(), rs.cpu().double()))
    finally:
        _lib.set_option("gemm_skinny", 1)
        _lib.set_matmul_precision("fp32")
    for c, r in outs:
        assert (c - ref).abs().max().item() <= tol
        assert (r - opA.double().sum(1)).abs().max().item() <= 1e-4 * (1 + K ** 0.5)   # beta 0: rs overwritten
    assert (outs[0][0] - outs[1][0]).abs().max().item() <= 2 * tol


def _ref_gru(IN, H, L):
    return torch.nn.GRU(IN, H, num_layers=L, bidirectional=True, batch_first=True)


@pytest.mark.parametrize("B,T,IN,H,L", [(5, 7, 39, 128, 2), (33, 3, 20, 128, 1), (70, 5, 16, 256, 1), (4, 51, 39, 512, 2)])
def test_bigru_fwd_bwd_vs_torch(gpu, B, T, IN, H, L):
    torch.manual_seed(0)
    ref = _ref_gru(IN, H, L)
    mine = snn.BiGRU(IN, H, num_layers=L).cuda()
    mine.load_state_dict(ref.state_dict())
    x = torch.randn(B, T, IN)
    w = torch.randn(B, T, 2 * H)
    xr = x.clone().requires_grad_(True)
    yr, hr = ref(xr)
    (yr * w).sum().backward()
    xm = x.cuda().requires_grad_(True)
    ym, hm = mine(xm)
    (ym * w.cuda()).sum().backward()
    tol = 2e-5 * max(1.0, T / 10)
    assert (ym.detach().cpu() - yr.detach()).abs().max() <= tol
    assert (hm.detach().cpu() - hr.detach()).abs().max() <= tol
    assert (xm.grad.cpu() - xr.grad).abs().max() <= 50 * tol * (1 + xr.grad.abs().max())
    refp = dict(ref.named_parameters())
    for n, p in mine.named_parameters():
        gr = refp[n].grad
        err = (p.grad.cpu() - gr).abs().max() / (gr.abs().max() + 1e-12)
        assert err <= 1e-4, (n, float(err))


def test_linear_strided_and_ce(gpu):
    torch.manual_seed(1)
    ref = torch.nn.Linear(1024, 12)
    mine = snn.Linear(1024, 12).cuda()
    mine.load_state_dict(ref.state_dict())
    h = torch.randn(6, 5, 1024)
    labels = torch.tensor([0, 3, 11, 5, 5, 2])
    hr = h.clone().requires_grad_(True)
    lr_ = torch.nn.CrossEntropyLoss()(ref(hr[:, -1, :]), labels)
    lr_.backward()
    hm = h.cuda().requires_grad_(True)
    lm = snn.CrossEntropyLoss()(mine(hm[:, -1, :]), labels.cuda())
    lm.backward()
    assert abs(lm.item() - lr_.item()) <= 1e-5 * max(1, abs(lr_.item()))
    assert (hm.grad.cpu() - hr.grad).abs().max() <= 1e-6
    assert (mine.weight.grad.cpu() - ref.weight.grad).abs().max() <= 1e-6
    assert (mine.bias.grad.cpu() - ref.bias.grad).abs().max() <= 1e-6


def test_ce_bad_label_is_nan(gpu):
    loss = snn.CrossEntropyLoss()(torch.zeros(2, 12, device="cuda"), torch.tensor([0, 12], device="cuda"))
    assert torch.isnan(loss).item()


def test_adam_matches_torch(gpu):
    torch.manual_seed(2)
    ref = torch.nn.Linear(37, 5)
    mine = torch.nn.Linear(37, 5).cuda()
    mine.load_state_dict(ref.state_dict())
    fp = FlatParams(mine.parameters())
    opt_m = Adam(mine.parameters(), lr=1e-2, flat=fp)
    opt_r = torch.optim.Adam(ref.parameters(), lr=1e-2)
    for it in range(5):
        x = torch.randn(8, 37)
        opt_r.zero_grad()
        ref(x).pow(2).sum().backward()
        opt_r.step()
        opt_m.zero_grad()
        mine(x.cuda()).pow(2).sum().backward()
        opt_m.step()
    for (n, a), (_, b) in zip(ref.named_parameters(), mine.named_parameters()):
        assert (a.detach() - b.detach().cpu()).abs().max() <= 1e-5, n


@pytest.mark.parametrize("kernel", [1, 2])
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1288, 776, 1352), (1032, 264, 4100), (2048, 512, 16), (1536, 516, 13056)])
def test_gemm_f32_kernels_at_tile_edges(gpu, kernel, ta, tb, M, N, K):
    """Both fp32 GEMM kernels (register-staged / LDS-DMA ping-pong, srk option gemm32_kernel) on
    shapes with partial 256-row / -column tiles, k tails (K % 16 != 0), a single K-tile and split-K,
    with alpha, beta and a bias, and the fused row sums of op(A) (the dW GEMMs' bias gradient)."""
    from speechrecognitionproject_amd import _lib
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K + 11 * ta + 13 * tb)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn((N, K) if tb else (K, N), generator=g)
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g)
    opA, opB = (A.T if ta else A).double(), (B.T if tb else B).double()
    ref = 0.5 * (opA @ opB) + 2.0 * C0.double() + bias.double()
    tol = 1e-5 * (1 + (opA.abs() @ opB.abs()).max().item())
    Ad, Bd = A.cuda(), B.cuda()
    _lib.set_option("gemm32_kernel", kernel)
    try:
        Cd = C0.clone().cuda()
        call("srk_gemm_f32", ta, tb, M, N, K, 0.5, ptr(Ad), Ad.shape[1], ptr(Bd), Bd.shape[1], 2.0, ptr(Cd), N,
             ptr(bias.cuda()), 1, stream_ptr())
        Cr = torch.zeros(M, N, device="cuda")
        rs = torch.full((M,), 3.0, device="cuda")
        call("srk_gemm_rowsum_f32", ta, tb, M, N, K, 1.0, ptr(Ad), Ad.shape[1], ptr(Bd), Bd.shape[1], 1.0, ptr(Cr),
             N, ptr(rs), stream_ptr())   # beta = 1 on C (zero-initialised below) and on the row sums
        torch.cuda.synchronize()
    finally:
        _lib.set_option("gemm32_kernel", 0)
    assert (Cd.cpu().double() - ref).abs().max().item() <= tol
    assert (rs.cpu().double() - (3.0 + opA.sum(1))).abs().max().item() <= 1e-3 * (1 + K ** 0.5)


@pytest.mark.parametrize("ta", [0, 1])
@pytest.mark.parametrize("M,N,K", [(96, 64, 13056), (3072, 39, 4999), (12, 1024, 256)])
def test_gemm_rowsum_splitk(gpu, ta, M, N, K):
    # the weight-gradient shape class: tall K (split over K), fused row sums of op(A) (= db)
    g = torch.Generator().manual_seed(K)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn(K, N, generator=g)
    opA = (A.T if ta else A).double()
    ref = opA @ B.double()
    ref_rs = opA.sum(1)
    Ad, Bd = A.cuda(), B.cuda()
    C = torch.empty(M, N, device="cuda")
    rs = torch.empty(M, device="cuda")
    for _ in range(2):   # deterministic: two launches are bitwise equal
        call("srk_gemm_rowsum_f32", ta, 0, M, N, K, 1.0, ptr(Ad), Ad.shape[1], ptr(Bd), N, 0.0, ptr(C), N, ptr(rs),
             stream_ptr())
        c1, r1 = C.clone(), rs.clone()
    assert torch.equal(c1, C) and torch.equal(r1, rs)
    assert (C.cpu().double() - ref).abs().max() <= 1e-5 * (1 + 4 * K ** 0.5 * 16)
    assert (rs.cpu().double() - ref_rs).abs().max() <= 1e-3


def test_colsum_large(gpu):
    X = torch.randn(13056, 3072)
    out = torch.empty(3072, device="cuda")
    call("srk_colsum_f32", ptr(X.cuda()), 13056, 3072, 3072, ptr(out), 0.0, stream_ptr())
    assert (out.cpu().double() - X.double().sum(0)).abs().max() <= 1e-3


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,T,IN", [(256, 51, 24), (512, 19, 1024), (200, 9, 24)])
def test_bigru_xcd_local_handoff_is_bitwise_identical(gpu, prec, B, T, IN):
    """The persistent recurrence with the XCD-local hand-off (census of HW_REG_XCC_ID, plain stores
    kept in the XCD's L2; option gru_xcd_local, default on) produces bitwise the same outputs and
    gradients as the placement-independent write-through protocol: each (direction, group, slice)
    does the same arithmetic in the same order, only which workgroup runs it changes.  B = 512 runs
    two 256-row chunk launches (census per launch); B = 200 has a partial grid (no census: fallback)."""
    from speechrecognitionproject_amd import _lib
    H = 512
    torch.manual_seed(11)
    mine = snn.BiGRU(IN, H, num_layers=1).cuda()
    x = torch.randn(B, T, IN)
    w = torch.randn(B, T, 2 * H)
    outs = {}
    try:
        _lib.set_matmul_precision(prec)
        for mode in (1, 0):
            _lib.set_option("gru_xcd_local", mode)
            for _ in range(2):   # twice: the census and the flags must reset between launches
                mine.zero_grad()
                xm = x.cuda().requires_grad_(True)
                ym, _ = mine(xm)
                (ym * w.cuda()).sum().backward()
            outs[mode] = [ym.detach().cpu(), xm.grad.cpu()] + [p.grad.cpu() for p in mine.parameters()]
    finally:
        _lib.set_option("gru_xcd_local", 1)
        _lib.set_matmul_precision("fp32")
    assert _lib.spin_timeouts() == 0
    for i, (a, b) in enumerate(zip(outs[1], outs[0])):
        assert torch.equal(a, b), i


@pytest.mark.parametrize("B,T", [(1, 6), (67, 13), (256, 51), (300, 7)])
def test_bigru_persistent_matches_per_step_and_torch(gpu, B, T):
    """The one-launch persistent recurrence (H = 512) agrees with the per-step kernels (same cell
    math; each workgroup walks the recurrent k sum in its own rotated order, so fp32 rounding
    differs: 2e-5 relative) and matches torch's CPU GRU; B = 300 exercises the 256-row chunking,
    B = 1 / 67 the clamped partial 64-row groups."""
    from speechrecognitionproject_amd import _lib
    IN, H = 24, 512
    torch.manual_seed(3)
    ref = _ref_gru(IN, H, 1)
    mine = snn.BiGRU(IN, H, num_layers=1).cuda()
    mine.load_state_dict(ref.state_dict())
    x = torch.randn(B, T, IN)
    w = torch.randn(B, T, 2 * H)
    outs = {}
    try:
        for mode in (1, 0):
            _lib.set_option("gru_persistent", mode)
            mine.zero_grad()
            xm = x.cuda().requires_grad_(True)
            ym, _ = mine(xm)
            (ym * w.cuda()).sum().backward()
            outs[mode] = [ym.detach().cpu(), xm.grad.cpu()] + [p.grad.cpu() for p in mine.parameters()]
    finally:
        _lib.set_option("gru_persistent", 1)
    assert _lib.spin_timeouts() == 0
    for i, (a, b) in enumerate(zip(outs[1], outs[0])):
        err = float((a - b).abs().max() / (b.abs().max() + 1e-30))
        assert err <= 2e-5, (i, err)
    if B * T <= 4000:
        xr = x.clone().requires_grad_(True)
        yr, _ = ref(xr)
        (yr * w).sum().backward()
        assert (outs[1][0] - yr.detach()).abs().max() <= 2e-5 * max(1.0, T / 10)
        gr = ref.weight_hh_l0.grad
        gm = dict(mine.named_parameters())["weight_hh_l0"].grad.cpu()
        assert (gm - gr).abs().max() / gr.abs().max() <= 1e-4


def test_flat_grads_accumulate_in_place(gpu):
    """FlatParams lays each BiGRU direction pair out back to back, so the layer sees the stacked
    weights as one tensor and the backward ADDS into the .grad views (beta = 1 epilogues) instead
    of handing autograd fresh gradients: two backward passes must give exactly twice one pass,
    and the result must equal the returned-gradient path of a module without FlatParams."""
    torch.manual_seed(7)
    B, T, IN, H = 40, 5, 39, 512
    ref = _ref_gru(IN, H, 2)
    plain = snn.BiGRU(IN, H, num_layers=2).cuda()
    plain.load_state_dict(ref.state_dict())
    fc_plain = snn.Linear(2 * H, 12).cuda()
    flat_net = torch.nn.ModuleDict({"gru": snn.BiGRU(IN, H, num_layers=2), "fc": snn.Linear(2 * H, 12)}).cuda()
    flat_net["gru"].load_state_dict(ref.state_dict())
    flat_net["fc"].load_state_dict(fc_plain.state_dict())
    flat = FlatParams(flat_net.parameters())
    g = flat_net["gru"]
    assert g.weight_ih_l0_reverse.data_ptr() == g.weight_ih_l0.data_ptr() + g.weight_ih_l0.numel() * 4
    x = torch.randn(B, T, IN, device="cuda")
    lab = torch.randint(0, 12, (B,), device="cuda")

    def loss_of(gru, fc):
        y, _ = gru(x)
        return snn.CrossEntropyLoss()(fc(y[:, -1, :]), lab)

    loss_of(plain, fc_plain).backward()
    flat.zero_grad()
    loss_of(flat_net["gru"], flat_net["fc"]).backward()
    one = flat.grad.clone()
    loss_of(flat_net["gru"], flat_net["fc"]).backward()
    assert torch.allclose(flat.grad, 2 * one, rtol=1e-5, atol=1e-9)
    named = dict(flat_net["gru"].named_parameters())
    for n, p in plain.named_parameters():
        d = (named[n].grad - 2 * p.grad).abs().max().item()
        assert d <= 1e-5 * (1 + p.grad.abs().max().item()), n
    assert (flat_net["fc"].weight.grad - 2 * fc_plain.weight.grad).abs().max().item() <= 1e-6
    assert (flat_net["fc"].bias.grad - 2 * fc_plain.bias.grad).abs().max().item() <= 1e-6


def test_plain_autograd_gets_gradients_without_flatparams(gpu):
    """Without FlatParams the layers return their gradients to autograd (no in-place .grad
    writes): torch.autograd.grad sees them and leaves .grad untouched, AccumulateGrad hooks fire,
    and a torch optimizer's zero_grad(set_to_none=False) + two backward passes sum."""
    from speechrecognitionproject_amd import nn as snn
    torch.manual_seed(0)
    gru = snn.BiGRU(39, 512, num_layers=1).cuda()
    fc = snn.Linear(1024, 12).cuda()
    params = list(gru.parameters()) + list(fc.parameters())
    x = torch.randn(8, 5, 39, device="cuda")

    def loss_fn():
        return fc(gru(x)[0][:, -1, :]).square().sum()

    grads = torch.autograd.grad(loss_fn(), params)
    assert all(g is not None and torch.isfinite(g).all() for g in grads)
    assert all(p.grad is None for p in params)
    fired = []
    fc.weight.register_post_accumulate_grad_hook(lambda p: fired.append(1))
    opt = torch.optim.SGD(params, lr=0.0)
    opt.zero_grad(set_to_none=False)
    loss_fn().backward()
    loss_fn().backward()
    assert len(fired) == 2
    for p, g in zip(params, grads):
        assert torch.allclose(p.grad, 2 * g, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,T,IN", [(256, 51, 39), (256, 13, 1024), (512, 9, 24), (300, 7, 24), (67, 11, 1024), (1, 5, 39)])
def test_bigru_fp32_dual_chain_matches_four_wave(gpu, B, T, IN):
    """The fp32 two-chain recurrence kernels, forward and backward (8 waves, k halves combined through
    LDS, per-wave flags, a 3-slot hand-off ring; option gru_fp32_dual_chain, default on) against the
    4-wave kernels: the same cell math with the recurrent k sum split in two halves (2e-5 relative), the fused layer-0
    projection (IN <= 64) and the gi-GEMM path, full / partial / chunked (B = 300, 512) grids; and
    run twice — bitwise the same both times (deterministic order, flags and ring reset per launch), and
    with either chain at static priority (option gru_dc_prio) — bitwise the same again."""
    from speechrecognitionproject_amd import _lib
    H = 512
    torch.manual_seed(5)
    mine = snn.BiGRU(IN, H, num_layers=1).cuda()
    x = torch.randn(B, T, IN)
    w = torch.randn(B, T, 2 * H)
    outs = {}
    try:
        # (two-chain, static chain priority): the priority (option gru_dc_prio) changes timing only
        for mode, prio in ((1, 0), (1, 0), (0, 0), (1, 1), (1, 2)):
            _lib.set_option("gru_fp32_dual_chain", mode)
            _lib.set_option("gru_dc_prio", prio)
            mine.zero_grad()
            xm = x.cuda().requires_grad_(True)
            ym, _ = mine(xm)
            (ym * w.cuda()).sum().backward()
            outs.setdefault(mode, []).append([ym.detach().cpu(), xm.grad.cpu()] + [p.grad.cpu() for p in mine.parameters()])
    finally:
        _lib.set_option("gru_fp32_dual_chain", 1)
        _lib.set_option("gru_dc_prio", 0)
    assert _lib.spin_timeouts() == 0
    for k in (1, 2, 3):
        for a, b in zip(outs[1][0], outs[1][k]):
            assert torch.equal(a, b)
    for i, (a, b) in enumerate(zip(outs[1][0], outs[0][0])):
        err = float((a - b).abs().max() / (b.abs().max() + 1e-30))
        assert err <= 2e-5, (i, err)



@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("B,T,IN", [(512, 9, 39), (512, 6, 1024), (300, 7, 39), (1024, 5, 48), (448, 5, 24)])
def test_bigru_lowprec_wide_matches_chunked(gpu, prec, B, T, IN):
    """16-bit recurrence over more than 256 rows: the 64-row workgroup kernels (8 waves, one launch of
    up to 512 rows; option gru_lp_wide, default on) against the 32-row kernels run as 256-row chunks
    one after the other.  Each row runs the same source arithmetic, but the two instantiations are
    compiled separately and the compiler's multiply-add contraction in the cell is free to differ:
    step 0 (h_prev = 0) is bitwise equal, later steps differ at fp32 rounding level, amplified by the
    16-bit hand-off (measured <= 1.3e-4 on outputs of magnitude <= 1).  Bounds: outputs 5e-4 absolute,
    gradients 2e-3 relative (norm-wise), and each mode bitwise reproducible run to run.  IN = 48 keeps
    the fused forward on the chunked kernel (the wide one fuses inputs of <= 40) while the backward
    runs wide; B = 1024 is two wide launches (bias partials of chunk 1); B = 448 a partial grid."""
    from speechrecognitionproject_amd import _lib
    H = 512
    torch.manual_seed(12)
    mine = snn.BiGRU(IN, H, num_layers=1).cuda()
    x = torch.randn(B, T, IN)
    w = torch.randn(B, T, 2 * H)
    outs = {}
    try:
        _lib.set_matmul_precision(prec)
        for mode in (1, 1, 0):
            _lib.set_option("gru_lp_wide", mode)
            _lib.prof_enable(True)
            mine.zero_grad()
            xm = x.cuda().requires_grad_(True)
            ym, _ = mine(xm)
            (ym * w.cuda()).sum().backward()
            torch.cuda.synchronize()
            kinds = {r["kernel"].split(" ")[0] for r in _lib.prof_kernels() if r["name"].startswith("gru_")}
            _lib.prof_enable(False)
            outs.setdefault(mode, []).append(([ym.detach().cpu(), xm.grad.cpu()],
                                              dict((n, p.grad.cpu()) for n, p in mine.named_parameters()), kinds))
    finally:
        _lib.set_option("gru_lp_wide", 1)
        _lib.set_matmul_precision("fp32")
    assert _lib.spin_timeouts() == 0
    assert "gru_bwd_persistent_lp2w_kernel" in outs[1][0][2] and "gru_bwd_persistent_lp2w_kernel" not in outs[0][0][2]
    assert ("gru_fwd_persistent_lp2w_kernel" in outs[1][0][2]) == (IN != 48)
    (a0, g0, _), (a1, g1, _) = outs[1]
    (c0, h0, _), = outs[0]
    for a, b in zip(a0, a1):
        assert torch.equal(a, b)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), n
    if IN != 48:   # step 0 of each direction: no recurrent term, bitwise equal
        assert torch.equal(a0[0][:, 0, :H], c0[0][:, 0, :H]) and torch.equal(a0[0][:, -1, H:], c0[0][:, -1, H:])
    assert float((a0[0] - c0[0]).abs().max()) <= 5e-4
    for a, b in [(a0[1], c0[1])] + [(g0[n], h0[n]) for n in g0]:
        err = float((a - b).norm() / b.norm())
        assert err <= 2e-3, err


@pytest.mark.parametrize("M,N,K,ta,beta,bias", [(13056, 1024, 3072, 0, 0.0, 0), (8000, 1024, 777, 0, 1.5, 1),
                                                (7000, 1100, 2048, 1, 0.0, 2)])
def test_gemm_streamk(gpu, M, N, K, ta, beta, bias):
    """srk option gemm_streamk: the fp32 ping-pong GEMM over a grid of 1/2 .. 1 round of 256 x 256
    tiles (the BiGRU layers' dx: 204 tiles on 256 CUs) split into equal runs of K-tiles, partial tiles
    summed by the fixup kernel — vs float64 and vs the one-run-per-tile launch."""
    from speechrecognitionproject_amd import _lib
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn((K, M) if ta else (M, K), generator=g)
    B = torch.randn(K, N, generator=g)
    C0 = torch.randn(M, N, generator=g)
    bv = torch.randn(M if bias == 2 else N, generator=g)
    ref = 0.5 * ((A.T if ta else A).double() @ B.double()) + beta * C0.double()
    if bias == 1:
        ref += bv.double()
    elif bias == 2:
        ref += bv.double()[:, None]
    Ad, Bd, bd = A.cuda(), B.cuda(), bv.cuda()
    outs = []
    try:
        for sk in (1, 0):
            _lib.set_option("gemm_streamk", sk)
            Cd = C0.clone().cuda()
            call("srk_gemm_f32", ta, 0, M, N, K, 0.5, ptr(Ad), Ad.shape[1], ptr(Bd), N, beta, ptr(Cd), N,
                 ptr(bd) if bias else None, bias, stream_ptr())
            outs.append(Cd.cpu().double())
    finally:
        _lib.set_option("gemm_streamk", 1)
    tol = 1e-5 * (1 + (A.abs().max() * B.abs().max() * K).item())
    assert (outs[0] - ref).abs().max() <= tol
    assert (outs[0] - outs[1]).abs().max() <= tol
