"""Autograd modules over libsrk.so: the drop-in replacements for the torch.nn layers the
reference models use (nn.GRU, nn.Linear, nn.CrossEntropyLoss).  Parameter names and shapes are
torch's, so reference ``state_dict`` checkpoints load unchanged.

Every forward/backward runs a HIP kernel through the C ABI; there is no CPU or torch-kernel
fallback (the GPU and the library are required).
"""
import ctypes
import os

import torch
import torch.nn as tnn

from . import _lib
from ._lib import call
from .features import ptr, require_gpu, stream_ptr


def _check_cuda(*ts):
    for t in ts:
        if t is not None and (t.device.type != "cuda" or t.dtype != torch.float32):
            raise _lib.SrkError("libsrk ops need float32 CUDA tensors, got %s %s" % (t.device, t.dtype))


# ----------------------------------------------------------------------------- GRU
def _adjacent(a, b):
    """b starts right where a ends in one storage (FlatParams lays BiGRU twins out this way)."""
    return (a.is_contiguous() and b.is_contiguous() and a.dtype == b.dtype and a.shape == b.shape
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
            and b.data_ptr() == a.data_ptr() + a.numel() * a.element_size())


def _dir_pair(a, b):
    """The [2, ...] stacked tensor of a direction pair: a view when adjacent, else a copy."""
    if _adjacent(a, b):
        return a.as_strided((2,) + tuple(a.shape), (a.numel(),) + tuple(a.stride()))
    return torch.stack([a, b])


# conv weight / BatchNorm parameter gradients added into FlatParams-owned .grad by their kernels (A/B switch:
# 0 = returned to autograd; the GRU's in-place pairs are not affected)
INPLACE_GRADS = os.environ.get("SRK_INPLACE_GRADS", "1") != "0"


def _flat_grad(p):
    """p.grad when p is owned by a FlatParams (optim.py) and its .grad is still that buffer's view:
    the one case where a backward may accumulate into .grad in place (beta = 1 in the GEMM
    epilogue) and hand autograd None.  Any other parameter (plain torch optimizers, DDP,
    torch.autograd.grad) gets its gradient returned to autograd as usual, so AccumulateGrad and
    its hooks run."""
    flat = getattr(p, "_srk_flat", None)
    g = p.grad
    if flat is None or g is None or not flat.owns_grad(p):
        return None
    return g


def _reducer_of(p):
    """The overlapped gradient all-reduce (parallel.GradReducer) attached to p's FlatParams, if any."""
    flat = getattr(p, "_srk_flat", None)
    return getattr(flat, "reducer", None) if flat is not None else None


def _grad_pair(a, b):
    """The stacked .grad of a FlatParams-owned direction pair to ACCUMULATE into in place
    (autograd's own accumulation, fused into the kernels' epilogues), or None (then the gradient
    is returned to autograd as usual)."""
    ga, gb = _flat_grad(a), _flat_grad(b)
    if ga is None or gb is None or not _adjacent(ga, gb):
        return None
    return _dir_pair(ga, gb)


class _GRULayerFn(torch.autograd.Function):
    """One bidirectional GRU layer (srk_gru_layer_fwd / srk_gru_layer_bwd) over the direction
    pairs (weight_ih_lN, weight_ih_lN_reverse), ... of the parameters themselves."""

    @staticmethod
    def forward(ctx, x, grad_on, w_ih_f, w_ih_r, w_hh_f, w_hh_r, b_ih_f, b_ih_r, b_hh_f, b_hh_r):
        # grad_on: torch.is_grad_enabled() at the call (inside forward it is always off, and
        # needs_input_grad ignores it): an evaluation pass under no_grad must not register copies
        B, T, IN = x.shape
        H = w_hh_f.shape[-1]
        x = x.contiguous()
        w_ih, w_hh = _dir_pair(w_ih_f, w_ih_r), _dir_pair(w_hh_f, w_hh_r)
        b_ih, b_hh = _dir_pair(b_ih_f, b_ih_r), _dir_pair(b_hh_f, b_hh_r)
        _check_cuda(x, w_ih, w_hh, b_ih, b_hh)
        y = torch.empty((B, T, 2 * H), device=x.device, dtype=torch.float32)
        ws = torch.empty(int(_lib.lib().srk_gru_workspace_floats(B, T, IN, H, 0)), device=x.device)
        # 16-bit modes: the previous layer's own 16-bit copy of h is this layer's x16 (module note at
        # _copies16); this layer's copy of its output goes to the next layer
        x16 = _copy16_get(x) if IN % 8 == 0 else None
        call("srk_gru_layer_fwd_x16", ptr(x), ptr(x16) if x16 is not None else None, B, T, IN, H, ptr(w_ih),
             ptr(w_hh), ptr(b_ih), ptr(b_hh), ptr(y), ptr(ws), stream_ptr())
        ctx.x16 = x16
        off = int(_lib.lib().srk_gru_y16_offset(B, T, IN, H)) if _copy16_wanted(2 * H) else -1
        if off >= 0 and grad_on and any(ctx.needs_input_grad):
            _copy16_put(y, ws[off:].view(torch.int16)[:y.numel()])
        ctx.save_for_backward(x, w_ih, w_hh, y, ws)
        ctx.dims = (B, T, IN, H)
        ctx.params = (w_ih_f, w_ih_r, w_hh_f, w_hh_r, b_ih_f, b_ih_r, b_hh_f, b_hh_r)
        ctx.prec = _lib.matmul_precision()   # the backward runs at its forward's precision
        red = _reducer_of(w_ih_f)
        if red is not None and grad_on and any(ctx.needs_input_grad):
            red.persistent_pending(1)      # collectives wait until this layer's recurrence is enqueued
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_ih, w_hh, y, ws = ctx.saved_tensors
        B, T, IN, H = ctx.dims
        P = ctx.params
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        targets = [_grad_pair(P[2 * i], P[2 * i + 1]) for i in range(4)]
        acc = all(t is not None for t in targets) and all(ctx.needs_input_grad[2:])
        if acc:   # accumulate straight into the parameters' .grad (FlatParams)
            dw_ih, dw_hh, db_ih, db_hh = targets
        else:
            dw_ih, dw_hh = torch.empty_like(w_ih), torch.empty_like(w_hh)
            db_ih = torch.empty((2, 3 * H), device=x.device)
            db_hh = torch.empty((2, 3 * H), device=x.device)
        ws2 = torch.empty(int(_lib.lib().srk_gru_workspace_floats(B, T, IN, H, 1)), device=x.device)
        _copy16_drop(y)   # the next layer's backward has run
        x16, ctx.x16 = ctx.x16, None
        with _lib.precision_scope(ctx.prec):
            call("srk_gru_layer_bwd_x16", ptr(x), ptr(x16) if x16 is not None else None, B, T, IN, H, ptr(w_ih),
                 ptr(w_hh), ptr(y), ptr(ws), ptr(dy), ptr(dx) if dx is not None else None, ptr(dw_ih), ptr(dw_hh),
                 ptr(db_ih), ptr(db_hh), int(acc), ptr(ws2), stream_ptr())
        red = _reducer_of(P[0])
        if red is not None:
            red.persistent_done()
            if acc:
                red.mark_ready(P)
        if acc:
            return (dx, None) + (None,) * 8
        return (dx, None, dw_ih[0], dw_ih[1], dw_hh[0], dw_hh[1], db_ih[0], db_ih[1], db_hh[0], db_hh[1])


class BiGRU(tnn.Module):
    """Drop-in for ``nn.GRU(input_size, hidden_size, num_layers, bidirectional=True,
    batch_first=True)`` (h0 = 0, no inter-layer dropout).  ``forward(x) -> (output, h_n)``."""

    def __init__(self, input_size, hidden_size, num_layers=1, bidirectional=True, batch_first=True):
        super().__init__()
        if not (bidirectional and batch_first):
            raise ValueError("BiGRU implements bidirectional=True, batch_first=True (the reference's config)")
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.bidirectional, self.batch_first = True, True
        H = hidden_size
        k = 1.0 / H ** 0.5
        for layer in range(num_layers):
            inp = input_size if layer == 0 else 2 * H
            for sfx in ("", "_reverse"):
                for name, shape in (("weight_ih", (3 * H, inp)), ("weight_hh", (3 * H, H)),
                                    ("bias_ih", (3 * H,)), ("bias_hh", (3 * H,))):
                    p = tnn.Parameter(torch.empty(shape).uniform_(-k, k))
                    setattr(self, "%s_l%d%s" % (name, layer, sfx), p)
            for name in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):   # FlatParams layout hint
                getattr(self, "%s_l%d" % (name, layer))._srk_pair = getattr(self, "%s_l%d_reverse" % (name, layer))

    def _pairs(self, layer):
        return [getattr(self, "%s_l%d%s" % (name, layer, sfx))
                for name in ("weight_ih", "weight_hh", "bias_ih", "bias_hh") for sfx in ("", "_reverse")]

    def forward(self, x):
        require_gpu()
        h = x
        finals = []
        for layer in range(self.num_layers):
            h = _GRULayerFn.apply(h, torch.is_grad_enabled(), *self._pairs(layer))
            H = self.hidden_size
            finals += [h[:, -1, :H], h[:, 0, H:]]
        return h, torch.stack(finals)


class _LastStepFn(torch.autograd.Function):
    """``x[:, -1, :]`` of a [B, T, C] sequence — the models' last-step select before their fc layer
    (model_mfcc_bgru.py:37 and the other BiGRU plugins).  The forward is the same strided view (the Linear
    GEMM reads it by row stride); the backward writes the [B, T, C] gradient, zeros and the last step, in
    one pad kernel instead of autograd's zero fill followed by a slice copy (one launch less per step)."""

    @staticmethod
    def forward(ctx, x):
        ctx.T = x.shape[1]
        return x[:, -1, :]

    @staticmethod
    def backward(ctx, g):
        return tnn.functional.pad(g.unsqueeze(1), (0, 0, ctx.T - 1, 0))


def last_step(x):
    """``x[:, -1, :]`` with a one-kernel backward (``_LastStepFn``)."""
    return _LastStepFn.apply(x)


# ----------------------------------------------------------------------------- Linear
class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        # x may be a row-strided 2-D view (e.g. out[:, -1, :]); the GEMM takes its row stride
        if x.dim() != 2 or x.stride(1) != 1:
            x = x.contiguous()
        _check_cuda(x, w, b)
        w_param = w
        w = w.contiguous()
        M, K = x.shape
        N = w.shape[0]
        y = torch.empty((M, N), device=x.device)
        call("srk_gemm_f32", 0, 1, M, N, K, 1.0, ptr(x), x.stride(0), ptr(w), K, 0.0, ptr(y), N,
             ptr(b) if b is not None else None, 1 if b is not None else 0, stream_ptr())
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        ctx.params = (w_param, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        M, K = x.shape
        N = w.shape[0]
        dx = dw = db = None
        s = stream_ptr()
        if ctx.needs_input_grad[0]:
            dx = torch.empty((M, K), device=x.device)
            call("srk_gemm_f32", 0, 0, M, K, N, 1.0, ptr(dy), N, ptr(w), K, 0.0, ptr(dx), K, None, 0, s)
        want_db = ctx.has_bias and ctx.needs_input_grad[2]
        # accumulate straight into the parameters' existing .grad buffers (beta = 1, fused into the
        # GEMM epilogue) instead of returning a fresh gradient for autograd to add
        wp, bp = ctx.params
        gw = _flat_grad(wp)
        gb = _flat_grad(bp) if bp is not None else None
        acc = gw is not None and (not want_db or gb is not None)
        if ctx.needs_input_grad[1]:
            dw = gw if acc else torch.empty((N, K), device=x.device)
            beta = 1.0 if acc else 0.0
            if want_db:   # dW = dy^T x with db = row sums of dy^T fused into the same kernel
                db = gb if acc else torch.empty((N,), device=x.device)
                call("srk_gemm_rowsum_f32", 1, 0, N, K, M, 1.0, ptr(dy), N, ptr(x), x.stride(0), beta, ptr(dw), K,
                     ptr(db), s)
            else:
                call("srk_gemm_f32", 1, 0, N, K, M, 1.0, ptr(dy), N, ptr(x), x.stride(0), beta, ptr(dw), K, None, 0,
                     s)
        else:
            acc = False
        if want_db and db is None:
            db = torch.empty((N,), device=x.device)
            call("srk_colsum_f32", ptr(dy), M, N, N, ptr(db), 0.0, s)
        if acc:
            red = _reducer_of(wp)
            if red is not None:
                red.mark_ready([wp] + ([bp] if bp is not None else []))
            return dx, None, None
        return dx, dw, db


class Linear(tnn.Module):
    """Drop-in for ``nn.Linear`` (same parameter names/shapes/init)."""

    def __init__(self, in_features, out_features, bias=True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = tnn.Parameter(torch.empty(out_features, in_features))
        self.bias = tnn.Parameter(torch.empty(out_features)) if bias else None
        ref = tnn.Linear(in_features, out_features, bias)     # torch's own init distribution
        with torch.no_grad():
            self.weight.copy_(ref.weight)
            if bias:
                self.bias.copy_(ref.bias)

    def forward(self, x):
        require_gpu()
        lead = x.shape[:-1]
        y = _LinearFn.apply(x.reshape(-1, x.shape[-1]) if x.dim() != 2 else x, self.weight, self.bias)
        return y.reshape(*lead, self.out_features)


# ----------------------------------------------------------------------------- loss
class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        logits = logits.contiguous()
        _check_cuda(logits)
        B, C = logits.shape
        labels = labels.to(device=logits.device, dtype=torch.int64).contiguous()
        loss = torch.empty((), device=logits.device)
        dlogits = torch.empty_like(logits) if ctx.needs_input_grad[0] else None
        ws = torch.empty(B + 1, device=logits.device)
        call("srk_cross_entropy", ptr(logits), ptr(labels), B, C, ptr(loss),
             ptr(dlogits) if dlogits is not None else None, ptr(ws), stream_ptr())
        ctx.save_for_backward(dlogits)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dlogits,) = ctx.saved_tensors
        return dlogits * g, None


class CrossEntropyLoss(tnn.Module):
    """Drop-in for ``nn.CrossEntropyLoss()`` (mean reduction), training.py:73."""

    def forward(self, logits, labels):
        require_gpu()
        return _CrossEntropyFn.apply(logits, labels)


# ----------------------------------------------------------------------------- 16-bit operand copies
# At bf16 / fp16 matmul precision the convolutions read 16-bit copies of x and dY.  In resnet_bgru every
# conv input is a BatchNorm output and every conv dY is a BatchNorm dx (model_resnet_bgru.py:19-39), so
# BatchNorm writes the copy beside its fp32 output (srk_batchnorm_fwd16 / _bwd16, the same rounding) and
# the conv takes it instead of re-reading the fp32 tensor to round it.  The hand-over is keyed by the
# tensor's address and checked against its identity: the entry holds the fp32 tensor itself (so the
# address cannot be reused while the entry lives), its version counter (any in-place write since
# invalidates it), element count and precision.  Forward copies are made in training steps only (training
# mode, autograd on); the producing BatchNorm's backward drops its forward entry, the conv backward pops the
# dY entry it consumes, and the table is bounded (a step's worth of entries).
COPIES16 = os.environ.get("SRK_BN_COPY16", "1") != "0"   # A/B switch (tests flip it)
RELU_MASK = os.environ.get("SRK_BN_RELU_MASK", "1") != "0"   # BatchNorm ReLU bits for the backward (A/B switch)
_copies16 = {}
_COPIES16_MAX = 32   # > the live entries of one resnet_bgru / mfrn_bgru step (about 22)


def _copy16_wanted(C):
    return COPIES16 and _lib.matmul_precision() != "fp32" and C % 8 == 0


def _copy16_put(t, t16):
    _copies16.pop(t.data_ptr(), None)
    while len(_copies16) >= _COPIES16_MAX:
        _copies16.pop(next(iter(_copies16)))
    _copies16[t.data_ptr()] = (t, t._version, t.numel(), _lib.matmul_precision(), t16)


def _copy16_get(t, pop=False):
    """The producer's 16-bit copy of t (a float32 contiguous CUDA tensor) at the current precision, or None."""
    e = _copies16.get(t.data_ptr())
    if e is None:
        return None
    src, ver, n, prec, t16 = e
    ok = (t.dtype == torch.float32 and t.is_contiguous() and t.numel() == n and t._version == ver
          and src.data_ptr() == t.data_ptr() and prec == _lib.matmul_precision())
    if pop or not ok:
        _copies16.pop(t.data_ptr(), None)
    return t16 if ok else None


def _copy16_drop(t):
    _copies16.pop(t.data_ptr(), None)   # t is alive (saved for backward), so the entry at its address is its own


# ----------------------------------------------------------------------------- conv / pool (NHWC)
def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class _Conv2dNHWCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, padding, stride):
        # w: the Conv2d weight [Co, Ci, KH, KW], or a Conv1d weight [Co, Ci, K] taken as [Co, Ci, 1, K] (the
        # parameter itself either way, so the backward can accumulate into its .grad)
        x = x.contiguous()
        w_param = w
        w = w.contiguous()
        if w.dim() == 3:
            w = w.unsqueeze(2)
        _check_cuda(x, w, b)
        N, H, W, Ci = x.shape
        Co, Ci2, KH, KW = w.shape
        if Ci2 != Ci:
            raise _lib.SrkError("conv: input has %d channels, weight expects %d" % (Ci, Ci2))
        ph, pw = padding
        sh, sw = stride
        Ho, Wo = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
        y = torch.empty((N, Ho, Wo, Co), device=x.device)
        ws = torch.empty(int(_lib.lib().srk_conv2d_workspace_floats(Ci, Co, KH, KW)), device=x.device)
        # 16-bit matmul precision with 8-aligned channels: keep the forward's 16-bit copy of x for the
        # backward's gathers (srk_conv2d_nhwc_fwd16; the library reports whether it wrote it)
        x16, written = None, ctypes.c_int(0)
        if _lib.matmul_precision() != "fp32" and Ci % 8 == 0 and Co % 8 == 0:
            x16 = _copy16_get(x)   # the producing BatchNorm's copy (written = 2: ready)
            if x16 is not None:
                written.value = 2
            elif ctx.needs_input_grad[1]:
                x16 = torch.empty(x.numel(), device=x.device, dtype=torch.int16)
        call("srk_conv2d_nhwc_fwd16", ptr(x), N, H, W, Ci, ptr(w), ptr(b) if b is not None else None, Co, KH, KW,
             ph, pw, sh, sw, ptr(y), ptr(ws), ptr(x16) if x16 is not None else None, ctypes.byref(written),
             stream_ptr())
        ctx.x16 = x16 if written.value else None
        ctx.prec = _lib.matmul_precision()
        ctx.save_for_backward(x, w)
        ctx.w_param = w_param
        ctx.geom = (padding, stride, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        (ph, pw), (sh, sw), has_b = ctx.geom
        N, H, W, Ci = x.shape
        Co, _, KH, KW = w.shape
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        # the weight gradient ADDED to a FlatParams-owned .grad in the layout kernel (no autograd add kernel)
        gw = _flat_grad(ctx.w_param) if ctx.needs_input_grad[1] and INPLACE_GRADS else None
        dw = gw if gw is not None else torch.empty_like(w)
        db = torch.empty((Co,), device=x.device) if has_b else None
        ws = torch.empty(int(_lib.lib().srk_conv2d_workspace_floats(Ci, Co, KH, KW)), device=x.device)
        x16 = ctx.x16 if ctx.prec == _lib.matmul_precision() else None   # a copy in this precision only
        ctx.x16 = None
        dy16 = _copy16_get(dy, pop=True)   # the producing BatchNorm backward's copy of dY
        call("srk_conv2d_nhwc_bwd16_acc", ptr(x), N, H, W, Ci, ptr(w), Co, KH, KW, ph, pw, sh, sw, ptr(dy),
             ptr(dy16) if dy16 is not None else None, ptr(dx) if dx is not None else None, ptr(dw),
             ptr(db) if db is not None else None, ptr(ws), ptr(x16) if x16 is not None else None,
             1 if gw is not None else 0, stream_ptr())
        if gw is not None:
            red = _reducer_of(ctx.w_param)
            if red is not None:
                red.mark_ready([ctx.w_param])
            dw = None
        else:
            dw = dw.view(ctx.w_param.shape)
        return dx, dw, db, None, None


class Conv2d(tnn.Module):
    """nn.Conv2d-compatible parameters (weight [Co, Ci, KH, KW], bias [Co], torch init) applied to
    CHANNELS-LAST input [N, H, W, Ci] -> [N, Ho, Wo, Co] (the models keep activations NHWC)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True):
        super().__init__()
        ref = tnn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, padding=padding, bias=bias)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = ref.kernel_size, ref.stride, ref.padding
        self.weight = tnn.Parameter(ref.weight.detach().clone())
        self.bias = tnn.Parameter(ref.bias.detach().clone()) if bias else None

    def forward(self, x):
        require_gpu()
        return _Conv2dNHWCFn.apply(x, self.weight, self.bias, self.padding, self.stride)


class Conv1d(tnn.Module):
    """nn.Conv1d-compatible parameters (weight [Co, Ci, K]) on channels-last input [N, L, Ci]."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, bias=True):
        super().__init__()
        ref = tnn.Conv1d(in_channels, out_channels, kernel_size, stride=stride, padding=padding, bias=bias)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = ref.kernel_size, ref.stride, ref.padding
        self.weight = tnn.Parameter(ref.weight.detach().clone())
        self.bias = tnn.Parameter(ref.bias.detach().clone()) if bias else None

    def forward(self, x):
        return conv1d_nlc(x, self.weight, self.bias, self.stride[0], self.padding[0])


def conv1d_nlc(x, weight, bias=None, stride=1, padding=0):
    """K6 1-D convolution of channels-last [N, L, Ci] input with an nn.Conv1d weight [Co, Ci, K]."""
    require_gpu()
    N, L, C = x.shape
    y = _Conv2dNHWCFn.apply(x.reshape(N, 1, L, C), weight, bias, (0, padding), (1, stride))
    return y.reshape(N, y.shape[2], weight.shape[0])


class _Conv1PoolFn(torch.autograd.Function):
    """conv1 + bias + MaxPool2d((1, pool)) of model_fbanks_cnn / model_spec_cnn (srk_conv1_pool_fwd /
    _wgrad): one input channel, the pooled NHWC output; the input (features) gets no gradient."""

    @staticmethod
    def forward(ctx, x, w, b, padding, pool, y16_only=False):
        x = x.contiguous()
        _check_cuda(x, w, b)
        N, H, W = x.shape
        Co, _, KH, KW = w.shape
        y = torch.empty((N, H, W // pool, Co), device=x.device)
        arg = torch.empty((N, H, W // pool, Co), device=x.device, dtype=torch.uint8)
        # training steps in a 16-bit mode: the kernel also writes y's 16-bit operand copy, which conv2's
        # fused conv + pool takes as ready (no second pass over the fp32 activation)
        y16 = None
        if _copy16_wanted(Co) and ctx.needs_input_grad[1]:   # (forward runs under no_grad: needs_input_grad tells)
            y16 = torch.empty(y.numel(), device=x.device, dtype=torch.int16)
        # y16_only: the caller's consumer reads only the copy (fbanks_cnn's fused conv2 + pool on 16-bit operands),
        # so the library may leave the fp32 y unwritten (it does only when it writes the copy)
        written = ctypes.c_int(3 if (y16_only and y16 is not None) else 0)
        call("srk_conv1_pool_fwd16", ptr(x), N, H, W, ptr(w.contiguous()), ptr(b), Co, KH, KW, padding[0], padding[1],
             pool, ptr(y), ptr(arg), ptr(y16) if y16 is not None else None, ctypes.byref(written), stream_ptr())
        if written.value:
            _copy16_put(y, y16)
        ctx.save_for_backward(x, arg)
        ctx.geom = (Co, KH, KW, padding, pool)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, arg = ctx.saved_tensors
        Co, KH, KW, padding, pool = ctx.geom
        N, H, W = x.shape
        dw = torch.empty((Co, 1, KH, KW), device=x.device)
        db = torch.empty((Co,), device=x.device)
        ws = torch.empty(int(_lib.lib().srk_conv1_pool_workspace_floats(Co, KH, KW)), device=x.device)
        call("srk_conv1_pool_wgrad", ptr(x), N, H, W, Co, KH, KW, padding[0], padding[1], pool, ptr(dy.contiguous()),
             ptr(arg), ptr(dw), ptr(db), ptr(ws), stream_ptr())
        return None, dw, db, None, None, None


def conv1_pool(x, conv, pool, next_conv_pool16=False):
    """Fused ``pool(conv(x))`` for a one-channel NHW input when the geometry is the one
    srk_conv1_pool supports (conv1 + maxpool1 of model_fbanks_cnn / model_spec_cnn) and ``x`` needs
    no gradient; otherwise the separate conv and pool kernels.  Returns NHWC.
    next_conv_pool16: the result goes straight into ``conv_pool`` (fbanks_cnn conv2): in a 16-bit training
    step with 16-bit conv forwards that reads only the 16-bit copy, so the fp32 activation is not stored."""
    geom = (tuple(conv.kernel_size), tuple(conv.padding), tuple(pool.kernel_size))
    if (conv.in_channels == 1 and conv.out_channels == 64 and tuple(conv.stride) == (1, 1) and conv.bias is not None
            and geom in (((7, 3), (3, 1), (1, 3)), ((3, 7), (1, 3), (1, 5))) and not x.requires_grad):
        require_gpu()
        y16_only = bool(next_conv_pool16 and _lib.fused_conv_pool() and not _lib.option("conv_fwd_fp32"))
        return _Conv1PoolFn.apply(x, conv.weight, conv.bias, conv.padding, pool.kernel_size[1], y16_only)
    return pool(conv(x.unsqueeze(-1)))


class _ConvPoolNHWCFn(torch.autograd.Function):
    """Conv2d (stride 1) + bias + MaxPool2d((1, 4)) with the pooling in the conv's epilogue
    (srk_conv2d_nhwc_fwd_pool / _bwd_pool): conv2 + maxpool2 of model_fbanks_cnn.py:74-75,91-92.
    Only the pooled activation and a uint8 argmax are kept; the backward routes the pooled gradient
    through the argmax inside the library."""

    @staticmethod
    def forward(ctx, x, w, b, padding, pool_w):
        x = x.contiguous()
        w = w.contiguous()
        _check_cuda(x, w, b)
        N, H, W, Ci = x.shape
        Co, _, KH, KW = w.shape
        ph, pw = padding
        Ho, Wo = H + 2 * ph - KH + 1, W + 2 * pw - KW + 1
        y = torch.empty((N, Ho, Wo // pool_w, Co), device=x.device)
        arg = torch.empty((N, Ho, Wo // pool_w, Co), device=x.device, dtype=torch.uint8)
        ws = torch.empty(int(_lib.lib().srk_conv2d_workspace_floats(Ci, Co, KH, KW)), device=x.device)
        x16, written = None, ctypes.c_int(0)
        if _lib.matmul_precision() != "fp32" and Ci % 8 == 0 and Co % 8 == 0:
            x16 = _copy16_get(x, pop=True)   # the producing srk_conv1_pool_fwd16's copy (written = 2: ready)
            if x16 is not None:
                written.value = 2
            elif ctx.needs_input_grad[1]:
                x16 = torch.empty(x.numel(), device=x.device, dtype=torch.int16)
        call("srk_conv2d_nhwc_fwd_pool", ptr(x), N, H, W, Ci, ptr(w), ptr(b) if b is not None else None, Co, KH, KW,
             ph, pw, pool_w, ptr(y), ptr(arg), ptr(ws), ptr(x16) if x16 is not None else None, ctypes.byref(written),
             stream_ptr())
        ctx.x16 = x16 if written.value else None
        ctx.prec = _lib.matmul_precision()
        ctx.save_for_backward(x, w, arg)
        ctx.geom = (padding, pool_w, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, arg = ctx.saved_tensors
        (ph, pw), pool_w, has_b = ctx.geom
        N, H, W, Ci = x.shape
        Co, _, KH, KW = w.shape
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w)
        db = torch.empty((Co,), device=x.device) if has_b else None
        ws = torch.empty(int(_lib.lib().srk_conv2d_workspace_floats(Ci, Co, KH, KW)), device=x.device)
        x16 = ctx.x16 if ctx.prec == _lib.matmul_precision() else None
        ctx.x16 = None
        call("srk_conv2d_nhwc_bwd_pool", ptr(x), N, H, W, Ci, ptr(w), Co, KH, KW, ph, pw, pool_w, ptr(dy), ptr(arg),
             ptr(dx) if dx is not None else None, ptr(dw), ptr(db) if db is not None else None, ptr(ws),
             ptr(x16) if x16 is not None else None, stream_ptr())
        return dx, dw, db, None, None


def conv_pool(x, conv, pool):
    """``pool(conv(x))`` for channels-last x: one fused launch (srk_conv2d_nhwc_fwd_pool) when the
    conv has stride 1 and the pool is (1, 4) with a window count that divides the output width
    (conv2 + maxpool2 of model_fbanks_cnn); otherwise the separate conv and pool kernels."""
    kh, kw = pool.kernel_size
    KH, KW = conv.kernel_size
    ph, pw = conv.padding
    Wo = x.shape[2] + 2 * pw - KW + 1
    if (tuple(conv.stride) == (1, 1) and (kh, kw) == (1, 4) and Wo % 4 == 0 and conv.out_channels % 4 == 0
            and _lib.fused_conv_pool()):
        require_gpu()
        return _ConvPoolNHWCFn.apply(x, conv.weight, conv.bias, conv.padding, 4)
    return pool(conv(x))


class _MaxPoolNHWCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kh, kw):
        x = x.contiguous()
        _check_cuda(x)
        N, H, W, C = x.shape
        y = torch.empty((N, H // kh, W // kw, C), device=x.device)
        call("srk_maxpool_nhwc_fwd", ptr(x), N, H, W, C, kh, kw, ptr(y), stream_ptr())
        ctx.save_for_backward(x)
        ctx.k = (kh, kw)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        kh, kw = ctx.k
        N, H, W, C = x.shape
        dx = torch.empty_like(x)
        call("srk_maxpool_nhwc_bwd", ptr(x), ptr(dy.contiguous()), N, H, W, C, kh, kw, ptr(dx), stream_ptr())
        return dx, None, None


class MaxPool2d(tnn.Module):
    """nn.MaxPool2d(kernel_size) (stride = kernel, floor mode) on channels-last input."""

    def __init__(self, kernel_size):
        super().__init__()
        self.kernel_size = _pair(kernel_size)

    def forward(self, x):
        return _MaxPoolNHWCFn.apply(x, self.kernel_size[0], self.kernel_size[1])


class MaxPool1d(tnn.Module):
    """nn.MaxPool1d(kernel_size) (stride = kernel) over the length axis of [N, L, C] input."""

    def __init__(self, kernel_size):
        super().__init__()
        self.kernel_size = kernel_size

    def forward(self, x):
        N, L, C = x.shape
        y = _MaxPoolNHWCFn.apply(x.reshape(N, L, 1, C), self.kernel_size, 1)
        return y.reshape(N, L // self.kernel_size, C)


_DROPOUT_STATE = {}   # device index -> int64[2] {base seed, call counter} read by srk_dropout_fwd_state
_MASK63 = (1 << 63) - 1
_DROPOUT_REPLAY = [0]


class dropout_replay_mode:
    """Within this block eager dropout calls draw their masks as a replayed HIP graph does: from the
    device state the last seeded call left, the kernel's counter advancing per call, without
    re-deriving the seed from torch's generator.  An eager step here is then the arithmetic of a
    graph replay, mask included (tests/test_graphs_gpu.py compares the two bit for bit)."""

    def __enter__(self):
        _DROPOUT_REPLAY[0] += 1
        return self

    def __exit__(self, *exc):
        _DROPOUT_REPLAY[0] -= 1
        return False


def _dropout_state(device):
    """The device-resident dropout seed of ``device``.  Outside a graph capture it is re-derived on
    every call from torch's CUDA generator of that device — (initial seed, Philox offset), the
    offset then advanced as torch's own dropout would — folded with the data-parallel rank, so
    ``torch.manual_seed`` governs the masks (as it does the reference's nn.Dropout on the GPU) and
    the CPU generator (DataLoader shuffles, the reference's numpy/random draws) is never touched.
    Inside a capture the state is left as the last eager call set it and the kernel's own counter
    advance gives every graph replay a fresh mask."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _DROPOUT_STATE.get(idx)
    if st is None:
        st = torch.zeros(2, dtype=torch.int64, device=device)
        _DROPOUT_STATE[idx] = st
    if not torch.cuda.is_current_stream_capturing() and not _DROPOUT_REPLAY[0]:
        gen = torch.cuda.default_generators[idx]
        seed, off = gen.initial_seed(), gen.get_offset()
        gen.set_offset(off + 4)
        rank = torch.distributed.get_rank() if torch.distributed.is_available() and torch.distributed.is_initialized() else 0
        base = ((seed * 0x9E3779B97F4A7C15) ^ (rank * 0xC2B2AE3D27D4EB4F) ^ (off << 17)) & _MASK63
        st[0].fill_(base)
        st[1].fill_(0)
    return st


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, state):
        x = x.contiguous()
        _check_cuda(x)
        y = torch.empty_like(x)
        keep = torch.empty(x.shape, device=x.device, dtype=torch.uint8)
        call("srk_dropout_fwd_state", ptr(x), x.numel(), float(p), ptr(state), ptr(y), ptr(keep), stream_ptr())
        ctx.save_for_backward(keep)
        ctx.scale = 1.0 / (1.0 - p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (keep,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        call("srk_dropout_apply", ptr(dy), ptr(keep), dy.numel(), float(ctx.scale), ptr(dx), stream_ptr())
        return dx, None, None


class _DropoutMaskFn(torch.autograd.Function):
    """y = x * keep / (1 - p) with a caller-supplied uint8 keep mask (srk_dropout_apply both ways)."""

    @staticmethod
    def forward(ctx, x, keep, scale):
        x = x.contiguous()
        _check_cuda(x)
        if keep.device != x.device or keep.dtype != torch.uint8 or keep.numel() != x.numel():
            raise _lib.SrkError("dropout keep mask must be a uint8 tensor of the input's size on its device")
        y = torch.empty_like(x)
        call("srk_dropout_apply", ptr(x), ptr(keep), x.numel(), float(scale), ptr(y), stream_ptr())
        ctx.save_for_backward(keep)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (keep,) = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        call("srk_dropout_apply", ptr(dy), ptr(keep), dy.numel(), float(ctx.scale), ptr(dx), stream_ptr())
        return dx, None, None


class Dropout(tnn.Module):
    """nn.Dropout(p=0.5): identity in eval mode; in training a Bernoulli(1-p) mask from a
    counter-based hash of a device-resident seed (``_dropout_state``: torch's CUDA generator state
    folded with the data-parallel rank, so ``torch.manual_seed`` governs the masks, ranks holding
    different clips draw independent masks, and a captured HIP graph draws a new mask per replay).

    ``set_mask(keep)`` supplies the keep mask (uint8, the input's shape) for the NEXT training
    forward instead of drawing one — how the parity tests replay a mask exported from the
    reference (tests/golden/fbanks_cnn_train_golden.npz)."""

    def __init__(self, p=0.5):
        super().__init__()
        self.p = p
        self._keep = None

    def set_mask(self, keep):
        self._keep = keep

    def forward(self, x):
        if not self.training or self.p == 0.0:
            return x
        if self._keep is not None:
            keep, self._keep = self._keep.to(device=x.device, dtype=torch.uint8).contiguous(), None
            if keep.shape != x.shape:
                raise ValueError("Dropout.set_mask: mask shape %s != input shape %s" % (tuple(keep.shape), tuple(x.shape)))
            return _DropoutMaskFn.apply(x, keep, 1.0 / (1.0 - self.p))
        return _DropoutFn.apply(x, self.p, _dropout_state(x.device))


# ----------------------------------------------------------------------------- batch norm
class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, running_mean, running_var, training, momentum, eps, relu):
        x = x.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        _check_cuda(x, gamma, beta, residual)
        y = torch.empty_like(x)
        mean = torch.empty(C, device=x.device)
        invstd = torch.empty(C, device=x.device)
        res = residual.contiguous() if residual is not None else None
        y16, written = None, ctypes.c_int(0)
        if training and any(ctx.needs_input_grad[:4]) and _copy16_wanted(C):   # the consuming conv's 16-bit copy of y
            y16 = torch.empty(y.numel(), device=x.device, dtype=torch.int16)
        # the ReLU pattern as bits for the backward (1/16 of y's bytes, read twice there)
        mask = None
        if relu and RELU_MASK and any(ctx.needs_input_grad[:4]):
            mask = torch.empty(M * C // 4, device=x.device, dtype=torch.uint8)
        call("srk_batchnorm_fwd16_mask", ptr(x), M, C, ptr(gamma), ptr(beta), float(eps), float(momentum),
             int(training), ptr(running_mean), ptr(running_var), ptr(res) if res is not None else None, int(relu),
             ptr(y), ptr(y16) if y16 is not None else None, ctypes.byref(written),
             ptr(mask) if mask is not None else None, ptr(mean), ptr(invstd), stream_ptr())
        if written.value:
            _copy16_put(y, y16)
        ctx.mask = mask
        ctx.save_for_backward(x, y, gamma, mean, invstd)
        ctx.params = (gamma, beta)
        ctx.flags = (int(training), int(relu), residual is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, mean, invstd = ctx.saved_tensors
        training, relu, has_res = ctx.flags
        C = x.shape[-1]
        M = x.numel() // C
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dres = torch.empty_like(x) if has_res and ctx.needs_input_grad[3] else None
        dgamma = torch.empty(C, device=x.device)
        dbeta = torch.empty(C, device=x.device)
        _copy16_drop(y)   # the forward's copy: its consumers' backward has run
        dx16, written = None, ctypes.c_int(0)
        if dx is not None and _copy16_wanted(C):   # dx is the producing conv's dY
            dx16 = torch.empty(dx.numel(), device=x.device, dtype=torch.int16)
        # dgamma / dbeta also ADDED to FlatParams-owned .grad buffers in the kernel that forms them
        gp, bp = ctx.params
        gg = _flat_grad(gp) if ctx.needs_input_grad[1] and INPLACE_GRADS else None
        gb = _flat_grad(bp) if ctx.needs_input_grad[2] and INPLACE_GRADS else None
        acc = gg is not None and gb is not None
        mask, ctx.mask = ctx.mask, None
        call("srk_batchnorm_bwd16_mask", ptr(x), ptr(y), ptr(mask) if mask is not None else None, ptr(dy), M, C,
             ptr(gamma), ptr(mean), ptr(invstd), training, relu, ptr(dx) if dx is not None else None,
             ptr(dx16) if dx16 is not None else None, ctypes.byref(written), ptr(dgamma), ptr(dbeta),
             ptr(dres) if dres is not None else None, ptr(gg) if acc else None, ptr(gb) if acc else None, stream_ptr())
        if written.value:
            _copy16_put(dx, dx16)
        if acc:
            red = _reducer_of(gp)
            if red is not None:
                red.mark_ready([gp, bp])
            return dx, None, None, dres, None, None, None, None, None, None
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None


class BatchNorm1d(tnn.Module):
    """nn.BatchNorm1d(C) parameters/buffers (weight, bias, running_mean, running_var,
    num_batches_tracked) on channels-last input [..., C]; optional fused residual add + ReLU."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1):
        super().__init__()
        self.num_features, self.eps, self.momentum = num_features, eps, momentum
        self.weight = tnn.Parameter(torch.ones(num_features))
        self.bias = tnn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def _normalize(self, x, gamma, beta, residual, running_mean, running_var, relu):
        """The K9 call on float4-aligned channels (SyncBatchNorm1d overrides it)."""
        return _BatchNormFn.apply(x, gamma, beta, residual, running_mean, running_var, self.training, self.momentum,
                                  self.eps, relu)

    def forward(self, x, residual=None, relu=False):
        require_gpu()
        if self.num_features % 4:
            return self.forward_padded(x, residual, relu)[..., :self.num_features]
        if self.training:
            self.num_batches_tracked.add_(1)
        return self._normalize(x, self.weight, self.bias, residual, self.running_mean, self.running_var, relu)

    def forward_padded(self, x, residual=None, relu=False):
        """K9 works on float4 channel groups: a channel count that is not a multiple of 4 (the
        resnet_bgru mode-1 head's 250 / 125) runs on zero-padded channels — their statistics are
        0 / 0, their outputs beta = 0 — and the result keeps the padding ([..., C rounded up to 4],
        pad channels 0; `forward` slices it off).  ``x`` may arrive padded already.  The running
        statistics are updated on padded copies and written back."""
        require_gpu()
        if self.training:
            self.num_batches_tracked.add_(1)
        C = self.num_features
        p = (-C) % 4
        if x.shape[-1] == C + p:
            xp = x
        else:
            assert x.shape[-1] == C, (x.shape, C)
            xp = tnn.functional.pad(x, (0, p))
        rp = tnn.functional.pad(residual, (0, C + p - residual.shape[-1])) if residual is not None else None
        g = torch.cat([self.weight, self.weight.new_ones(p)])
        b = torch.cat([self.bias, self.bias.new_zeros(p)])
        rm = torch.cat([self.running_mean, self.running_mean.new_zeros(p)])
        rv = torch.cat([self.running_var, self.running_var.new_ones(p)])
        y = self._normalize(xp, g, b, rp, rm, rv, relu)
        if self.training:
            with torch.no_grad():
                self.running_mean.copy_(rm[:C])
                self.running_var.copy_(rv[:C])
        return y


# ----------------------------------------------------------------------------- synchronized batch norm
class _SyncBatchNormFn(torch.autograd.Function):
    """Training-mode BatchNorm over the GLOBAL batch of all data-parallel ranks (torch.nn.SyncBatchNorm
    semantics): this rank's (count, mean, M2) per channel are all-gathered and combined in rank order
    on the device (identical statistics on every rank); the backward all-reduces (sum g, sum g * xhat)
    for dx, while dgamma / dbeta keep this rank's contribution (the data-parallel gradient all-reduce
    sums them, as for any parameter)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, residual, running_mean, running_var, momentum, eps, relu, group):
        import torch.distributed as dist
        x = x.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        _check_cuda(x, gamma, beta, residual)
        from . import parallel
        # under a HIP-graph capture the statistics exchange runs on the capture-only group, never on the
        # default group the eager warm-up steps used; the backward reuses the forward's choice
        group = parallel.group_for_now(group)
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        # all-gather as an all-reduce of rank-owned slots (x + 0 is exact; works on every backend)
        allst = torch.zeros((world, 3 * C), device=x.device)
        call("srk_batchnorm_stats", ptr(x), M, C, ptr(allst[rank]), stream_ptr())
        dist.all_reduce(allst, op=dist.ReduceOp.SUM, group=group)
        mean = torch.empty(C, device=x.device)
        invstd = torch.empty(C, device=x.device)
        total = torch.empty(1, device=x.device)
        call("srk_batchnorm_combine", ptr(allst), world, C, float(eps), float(momentum), ptr(running_mean),
             ptr(running_var), ptr(mean), ptr(invstd), ptr(total), stream_ptr())
        y = torch.empty_like(x)
        res = residual.contiguous() if residual is not None else None
        call("srk_batchnorm_apply", ptr(x), M, C, ptr(mean), ptr(invstd), ptr(gamma), ptr(beta),
             ptr(res) if res is not None else None, int(relu), ptr(y), stream_ptr())
        ctx.save_for_backward(x, y, gamma, mean, invstd, total)
        ctx.flags = (int(relu), residual is not None)
        ctx.group = group
        return y

    @staticmethod
    def backward(ctx, dy):
        import torch.distributed as dist
        x, y, gamma, mean, invstd, total = ctx.saved_tensors
        relu, has_res = ctx.flags
        C = x.shape[-1]
        M = x.numel() // C
        dy = dy.contiguous()
        sums = torch.empty(2 * C, device=x.device)
        call("srk_batchnorm_bwd_reduce", ptr(x), ptr(y), ptr(dy), M, C, ptr(mean), ptr(invstd), relu, ptr(sums),
             stream_ptr())
        dbeta, dgamma = sums[:C].clone(), sums[C:].clone()     # this rank's contributions
        dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=ctx.group)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dres = torch.empty_like(x) if has_res and ctx.needs_input_grad[3] else None
        if dx is not None or dres is not None:
            call("srk_batchnorm_bwd_dx", ptr(x), ptr(y), ptr(dy), M, C, ptr(total), ptr(gamma), ptr(mean), ptr(invstd),
                 ptr(sums), relu, ptr(dx) if dx is not None else None, ptr(dres) if dres is not None else None,
                 stream_ptr())
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None


class SyncBatchNorm1d(BatchNorm1d):
    """BatchNorm1d whose training statistics span every data-parallel rank (torch.nn.SyncBatchNorm).
    Same parameters / buffers / state_dict keys as BatchNorm1d; eval mode and a world of 1 take the
    plain BatchNorm1d path.  Build one with ``convert_sync_batchnorm(model)``."""

    # a 1-rank group normally takes the plain path; the GPU test of the captured exchange sets this
    collectives_at_world1 = False

    def __init__(self, num_features, eps=1e-5, momentum=0.1, process_group=None):
        super().__init__(num_features, eps, momentum)
        self.process_group = process_group

    def _normalize(self, x, gamma, beta, residual, running_mean, running_var, relu):
        # the padded path (channel counts not a multiple of 4: the resnet_bgru mode-1 head's 250 / 125)
        # comes through here too, so its statistics span the ranks as well
        import torch.distributed as dist
        if not (self.training and dist.is_available() and dist.is_initialized()
                and dist.get_world_size(self.process_group) > (0 if self.collectives_at_world1 else 1)):
            return super()._normalize(x, gamma, beta, residual, running_mean, running_var, relu)
        return _SyncBatchNormFn.apply(x, gamma, beta, residual, running_mean, running_var, self.momentum, self.eps,
                                      relu, self.process_group)


def convert_sync_batchnorm(module, process_group=None):
    """Replace every BatchNorm1d of ``module`` by a SyncBatchNorm1d sharing its parameters and
    buffers (torch.nn.SyncBatchNorm.convert_sync_batchnorm).  Call before FlatParams / the optimizer."""
    out = module
    if isinstance(module, BatchNorm1d) and not isinstance(module, SyncBatchNorm1d):
        out = SyncBatchNorm1d(module.num_features, module.eps, module.momentum, process_group)
        out.weight, out.bias = module.weight, module.bias
        out.running_mean, out.running_var = module.running_mean, module.running_var
        out.num_batches_tracked = module.num_batches_tracked
        out.train(module.training)
    for name, child in module.named_children():
        out.add_module(name, convert_sync_batchnorm(child, process_group))
    return out
