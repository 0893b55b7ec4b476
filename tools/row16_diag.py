"""Diagnostic: fbanks conv2 + pool, conv_row16 on / off — forward y and argmax, then the backward (same pooled
gradient) dx / dW / db, compared element-wise (where do they differ?)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speechrecognitionproject_amd import _lib  # noqa: E402
from speechrecognitionproject_amd._lib import call  # noqa: E402
from speechrecognitionproject_amd.features import ptr, stream_ptr  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 3
H, W, Ci, Co = 98, 40, 64, 128
g = torch.Generator().manual_seed(7)
x = torch.randn(N, H, W, Ci, generator=g).cuda()
w = (torch.randn(Co, Ci, 1, 7, generator=g) / 21.0).cuda()
b = torch.randn(Co, generator=g).cuda()
dyp = torch.randn(N, H, W // 4, Co, generator=g).cuda()
_lib.set_matmul_precision("bf16")
res = {}
for row in (1, 0):
    _lib.set_option("conv_row16", row)
    _lib.set_option("conv_row16_dgrad", row)
    y = torch.empty(N, H, W // 4, Co, device="cuda")
    arg = torch.empty(N, H, W // 4, Co, dtype=torch.uint8, device="cuda")
    ws = torch.empty(int(_lib.lib().srk_conv2d_workspace_floats(Ci, Co, 1, 7)), device="cuda")
    wr = ctypes.c_int(0)
    call("srk_conv2d_nhwc_fwd_pool", ptr(x), N, H, W, Ci, ptr(w), ptr(b), Co, 1, 7, 0, 3, 4, ptr(y), ptr(arg), ptr(ws),
         None, ctypes.byref(wr), stream_ptr())
    dx, dw, db = torch.empty_like(x), torch.empty_like(w), torch.empty(Co, device="cuda")
    call("srk_conv2d_nhwc_bwd_pool", ptr(x), N, H, W, Ci, ptr(w), Co, 1, 7, 0, 3, 4, ptr(dyp), ptr(arg), ptr(dx), ptr(dw),
         ptr(db), ptr(ws), None, stream_ptr())
    torch.cuda.synchronize()
    res[row] = (y, arg, dx, dw, db)
_lib.set_option("conv_row16", 1)
for name, a, c in zip(("y", "arg", "dx", "dw", "db"), res[1], res[0]):
    d = (a.double() - c.double()).abs()
    bad = (d > 0).nonzero()
    print(name, "equal" if torch.equal(a, c) else "DIFF max %.3g at %d elems, first %s" % (d.max().item(), len(bad),
                                                                                       bad[:3].tolist()))
a, c = res[1][2].reshape(-1, W, Ci), res[0][2].reshape(-1, W, Ci)
bad = ~torch.isclose(a, c, rtol=1e-3, atol=1e-3)
print("wrong fraction by pixel (w):", [round(v, 2) for v in bad.float().mean((0, 2)).tolist()])
print("wrong fraction by channel:", [round(v, 2) for v in bad.float().mean((0, 1)).tolist()][:64])
print("wrong fraction by image row (first 16):", [round(v, 2) for v in bad.float().mean((1, 2)).tolist()][:16])
# the plain (unpooled) conv backward with a dense random dY through the same conv_bwd hook
dyd = torch.randn(N, H, W, Co, generator=g).cuda()
res2 = {}
for row in (1, 0):
    _lib.set_option("conv_row16", row)
    _lib.set_option("conv_row16_dgrad", row)
    ws = torch.empty(int(_lib.lib().srk_conv2d_workspace_floats(Ci, Co, 1, 7)), device="cuda")
    dx, dw = torch.empty_like(x), torch.empty_like(w)
    call("srk_conv2d_nhwc_bwd", ptr(x), N, H, W, Ci, ptr(w), Co, 1, 7, 0, 3, 1, 1, ptr(dyd), ptr(dx), ptr(dw), None,
         ptr(ws), stream_ptr())
    torch.cuda.synchronize()
    res2[row] = (dx, dw)
_lib.set_option("conv_row16", 1)
for name, a, c in zip(("dense dx", "dense dw"), res2[1], res2[0]):
    d = (a.double() - c.double()).abs()
    print(name, "equal" if torch.equal(a, c) else "DIFF max %.3g at %d elems" % (d.max().item(), int((d > 0).sum())))
