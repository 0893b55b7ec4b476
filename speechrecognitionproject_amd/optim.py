"""Flat parameter/gradient buffers and the fused Adam of training.py:74,91 (srk_adam_step).

``FlatParams`` re-homes every parameter of a module into ONE contiguous fp32 buffer (each
tensor 256-byte aligned) and points ``p.grad`` at views of ONE gradient buffer, so that
  * the optimizer step is a single kernel launch over the whole model, and
  * the data-parallel gradient exchange is a single all-reduce of one buffer (parallel.py).
"""
import torch

from ._lib import call, check_health
from .features import ptr, require_gpu, stream_ptr

_ALIGN = 64   # floats


class FlatParams:
    def __init__(self, params, device=None):
        require_gpu()
        # a parameter may name a partner to be laid out right behind it (``_srk_pair``: the
        # reverse-direction twin of a BiGRU weight), so the kernels see the stacked pair as ONE
        # [2, ...] tensor in place — no per-step torch.stack / unbind copies
        ps = [p for p in params if p.requires_grad]
        ids = {id(p) for p in ps}
        order, seen = [], set()
        for p in ps:
            if id(p) in seen:
                continue
            order.append(p)
            seen.add(id(p))
            q = getattr(p, "_srk_pair", None)
            if q is not None and id(q) in ids and id(q) not in seen:
                order.append(q)
                seen.add(id(q))
        self.params = order
        device = device or self.params[0].device
        offs, n = [], 0
        for p in self.params:
            offs.append(n)
            n += (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
        self.numel = n
        self.offsets = offs
        self.data = torch.zeros(n, device=device, dtype=torch.float32)
        self.grad = torch.zeros(n, device=device, dtype=torch.float32)
        with torch.no_grad():
            for p, o in zip(self.params, offs):
                k = p.numel()
                self.data[o:o + k].copy_(p.data.reshape(-1))
                p.data = self.data[o:o + k].view_as(p)
                p.grad = self.grad[o:o + k].view_as(p)
                p._srk_flat = self    # the layers may accumulate into this .grad in place (nn.py)
        self._slot = {id(p): o for p, o in zip(self.params, offs)}

    def owns_grad(self, p):
        """p.grad is (still) this buffer's view for p."""
        o = self._slot.get(id(p))
        g = p.grad
        return (o is not None and g is not None and g.is_contiguous()
                and g.data_ptr() == self.grad.data_ptr() + o * self.grad.element_size())

    def zero_grad(self):
        self.grad.zero_()
        # autograd may have replaced a view with a fresh tensor; re-attach the views
        for p, o in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + 1].data_ptr():
                p.grad = self.grad[o:o + p.numel()].view_as(p)


class LossScaler:
    """Loss scaling for fp16 training, torch.cuda.amp.GradScaler semantics with its state on the
    device (srk_grad_scaler_init / srk_adam_step_scaled), so a captured HIP graph replays it:

        loss = criterion(model(x), y)
        scaler.scale(loss).backward()         # loss x scale (the scale is read on the device)
        optimizer.step(scaler=scaler)         # non-finite gradients -> the step is skipped

    ``dynamic=False`` keeps ``init_scale`` fixed (bench.py's static 1024); a skipped step is still
    counted in ``overflows()``.  ``dynamic=True`` halves the scale on an overflow and doubles it
    after ``growth_interval`` clean steps (GradScaler's defaults, except the initial scale)."""

    def __init__(self, init_scale=1024.0, dynamic=True, growth_factor=2.0, backoff_factor=0.5,
                 growth_interval=2000, device=None):
        require_gpu()
        device = device or torch.device("cuda", torch.cuda.current_device())
        self.state = torch.zeros(8, dtype=torch.int32, device=device)
        self.dynamic = bool(dynamic)
        call("srk_grad_scaler_init", ptr(self.state), float(init_scale), float(growth_factor),
             float(backoff_factor), int(growth_interval) if dynamic else 0, stream_ptr())

    def scale(self, loss):
        return loss * self.state.view(torch.float32)[0]

    def get_scale(self):
        """The current scale (synchronizes)."""
        return float(self.state.view(torch.float32)[0].item())

    def overflows(self):
        """Steps skipped so far because a gradient was inf / NaN (synchronizes)."""
        return int(self.state[7].item())


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam semantics (betas=(0.9, 0.999), eps=1e-8, no weight decay), one fused
    HIP launch per step over a FlatParams buffer.  ``grad_scale`` (e.g. 1/world_size after a
    summed all-reduce) multiplies the gradient inside the kernel; ``step(scaler=LossScaler)``
    additionally unscales fp16 loss-scaled gradients and skips a step whose gradients overflowed.

    The step count lives on the device (``state_dev[0]``: a replayed HIP graph advances it without
    the host; a skipped step does not advance it); ``step_count`` reads it (synchronizes)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, flat=None):
        params = list(params)
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        self.flat = flat if flat is not None else FlatParams(params)
        self.exp_avg = torch.zeros_like(self.flat.data)
        self.exp_avg_sq = torch.zeros_like(self.flat.data)
        # {int64 step; float bc1, sqrt(bc2), lr, 0} on the device, so a captured HIP graph replays the
        # step count and follows lr changes (ExponentialLR) made between replays
        self.state_dev = torch.zeros(4, dtype=torch.int64, device=self.flat.data.device)
        self._lr_dev = None
        self.grad_scale = 1.0

    @property
    def step_count(self):
        return int(self.state_dev[0].item())

    def zero_grad(self, set_to_none=False):
        self.flat.zero_grad()

    @torch.no_grad()
    def sync_lr(self):
        """Write param_groups[0]["lr"] into the device state if it changed (a captured step reads lr
        there: call this after an lr scheduler step when replaying a graph)."""
        lr = self.param_groups[0]["lr"]
        if lr != self._lr_dev and not torch.cuda.is_current_stream_capturing():
            self.state_dev.view(torch.float32)[4].fill_(float(lr))
            self._lr_dev = lr

    @torch.no_grad()
    def step(self, closure=None, scaler=None):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        f = self.flat
        self.sync_lr()
        if scaler is not None:
            call("srk_adam_step_scaled", ptr(f.data), ptr(f.grad), ptr(self.exp_avg), ptr(self.exp_avg_sq), f.numel,
                 float(b1), float(b2), float(g["eps"]), ptr(self.state_dev), float(self.grad_scale),
                 ptr(scaler.state), stream_ptr())
        else:
            call("srk_adam_step_state", ptr(f.data), ptr(f.grad), ptr(self.exp_avg), ptr(self.exp_avg_sq), f.numel,
                 float(b1), float(b2), float(g["eps"]), ptr(self.state_dev), float(self.grad_scale), stream_ptr())
        # a persistent kernel that timed out produced invalid gradients: fail loudly (a host-pinned
        # word, no device sync; it sees every timeout of the work the GPU has reached so far)
        check_health(sync=False)
        return loss
