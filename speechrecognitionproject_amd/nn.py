"""Autograd modules over libsrk.so: the drop-in replacements for the torch.nn layers the
reference models use (nn.GRU, nn.Linear, nn.CrossEntropyLoss).  Parameter names and shapes are
torch's, so reference ``state_dict`` checkpoints load unchanged.

Every forward/backward runs a HIP kernel through the C ABI; there is no CPU or torch-kernel
fallback (the GPU and the library are required).
"""
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
class _GRULayerFn(torch.autograd.Function):
    """One bidirectional GRU layer (srk_gru_layer_fwd / srk_gru_layer_bwd)."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh):
        B, T, IN = x.shape
        H = w_hh.shape[-1]
        x = x.contiguous()
        _check_cuda(x, w_ih, w_hh, b_ih, b_hh)
        y = torch.empty((B, T, 2 * H), device=x.device, dtype=torch.float32)
        ws = torch.empty(int(_lib.lib().srk_gru_workspace_floats(B, T, IN, H, 0)), device=x.device)
        call("srk_gru_layer_fwd", ptr(x), B, T, IN, H, ptr(w_ih), ptr(w_hh), ptr(b_ih), ptr(b_hh), ptr(y), ptr(ws),
             stream_ptr())
        ctx.save_for_backward(x, w_ih, w_hh, y, ws)
        ctx.dims = (B, T, IN, H)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_ih, w_hh, y, ws = ctx.saved_tensors
        B, T, IN, H = ctx.dims
        dy = dy.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw_ih, dw_hh = torch.empty_like(w_ih), torch.empty_like(w_hh)
        db_ih = torch.empty((2, 3 * H), device=x.device)
        db_hh = torch.empty((2, 3 * H), device=x.device)
        ws2 = torch.empty(int(_lib.lib().srk_gru_workspace_floats(B, T, IN, H, 1)), device=x.device)
        call("srk_gru_layer_bwd", ptr(x), B, T, IN, H, ptr(w_ih), ptr(w_hh), ptr(y), ptr(ws), ptr(dy),
             ptr(dx) if dx is not None else None, ptr(dw_ih), ptr(dw_hh), ptr(db_ih), ptr(db_hh), ptr(ws2),
             stream_ptr())
        return dx, dw_ih, dw_hh, db_ih, db_hh


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

    def _stacked(self, name, layer):
        return torch.stack([getattr(self, "%s_l%d" % (name, layer)), getattr(self, "%s_l%d_reverse" % (name, layer))])

    def forward(self, x):
        require_gpu()
        h = x
        finals = []
        for layer in range(self.num_layers):
            h = _GRULayerFn.apply(h, self._stacked("weight_ih", layer), self._stacked("weight_hh", layer),
                                  self._stacked("bias_ih", layer), self._stacked("bias_hh", layer))
            H = self.hidden_size
            finals += [h[:, -1, :H], h[:, 0, H:]]
        return h, torch.stack(finals)


# ----------------------------------------------------------------------------- Linear
class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        # x may be a row-strided 2-D view (e.g. out[:, -1, :]); the GEMM takes its row stride
        if x.dim() != 2 or x.stride(1) != 1:
            x = x.contiguous()
        _check_cuda(x, w, b)
        w = w.contiguous()
        M, K = x.shape
        N = w.shape[0]
        y = torch.empty((M, N), device=x.device)
        call("srk_gemm_f32", 0, 1, M, N, K, 1.0, ptr(x), x.stride(0), ptr(w), K, 0.0, ptr(y), N,
             ptr(b) if b is not None else None, 1 if b is not None else 0, stream_ptr())
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
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
        if ctx.needs_input_grad[1]:
            dw = torch.empty((N, K), device=x.device)
            if want_db:   # dW = dy^T x with db = row sums of dy^T fused into the same kernel
                db = torch.empty((N,), device=x.device)
                call("srk_gemm_rowsum_f32", 1, 0, N, K, M, 1.0, ptr(dy), N, ptr(x), x.stride(0), 0.0, ptr(dw), K,
                     ptr(db), s)
            else:
                call("srk_gemm_f32", 1, 0, N, K, M, 1.0, ptr(dy), N, ptr(x), x.stride(0), 0.0, ptr(dw), K, None, 0, s)
        if want_db and db is None:
            db = torch.empty((N,), device=x.device)
            call("srk_colsum_f32", ptr(dy), M, N, N, ptr(db), 0.0, s)
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
