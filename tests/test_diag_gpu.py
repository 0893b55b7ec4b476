"""Directed checks of the two patterns behind round 5's wrong row-staged data gradients (VERDICT r05 #8;
csrc/diag.hip holds the root-cause analysis).

* The epilogue's raw buffer stores of MFMA accumulators — the kernel's descriptor, voffset formula and
  drop value, at the full cfg3 size (6,272 tiles, offsets up to 513 MB): the product form stores every
  accumulator where it belongs.  The round-5 source form (`__builtin_bit_cast(unsigned, acc[j][r])`, a
  bit cast of a vector-component lvalue) compiles to stores of component 0 only (seen in the ISA on the
  host; tests/test_diag_isa.py checks the ISA on the CPU): on the device 15 of every 16 outputs are
  that value.
* ds_read_b64_tr_b16 B fragments of the 64-column TR image (the removed r16_off64 form) and of the
  128-column image the ring / row-staged kernels use equal the host model of the instruction:
  lane l receives M[kk + 8 (l >> 5) + e][r0 + (l & 31)], e = 0..7 — both images read right."""
import numpy as np
import pytest
import torch

from speechrecognitionproject_amd._lib import call
from speechrecognitionproject_amd.features import ptr, stream_ptr

pytestmark = pytest.mark.gpu


def _expected_acc_store(rows):
    tiles = rows // 8
    exp = np.full((tiles, 320, 64), -1.0, dtype=np.float32)
    p = np.arange(32)[:, None]
    c = np.arange(64)[None, :]
    exp[:, :32, :] = (1 + 64 * p + c)[None] + 2048.0 * np.arange(tiles)[:, None, None]
    return exp.reshape(rows, 40, 64)


@pytest.mark.parametrize("variant", [0, 1])
def test_acc_buffer_store_pattern(gpu, variant):
    rows = 512 * 98                       # cfg3's conv2 dX: 50,176 image rows x 40 px x 64 channels (513 MB)
    dx = torch.full((rows, 40, 64), -1.0, device="cuda")
    call("srk_diag_acc_store", ptr(dx), rows, variant, stream_ptr())
    torch.cuda.synchronize()
    got = dx.cpu().numpy()
    exp = _expected_acc_store(rows)
    if variant == 0:
        assert np.array_equal(got, exp)
    elif not np.array_equal(got, exp):   # a fixed compiler would store the right values: that passes too
        # the miscompiled form: register r of every lane stores component 0 (pixel 4 (l >> 5)); pixel
        # p = (r & 3) + 8 (r >> 2) + 4 (l >> 5) therefore receives the value of pixel 4 ((p >> 2) & 1)
        t = got.reshape(rows // 8, 320, 64)
        e = exp.reshape(rows // 8, 320, 64)
        src = 4 * ((np.arange(32) >> 2) & 1)
        assert np.array_equal(t[:, :32, :], e[:, src, :])
        assert np.array_equal(t[:, 32:, :], e[:, 32:, :])     # nothing else written


@pytest.mark.parametrize("cols", [64, 128])
def test_tr16_read_images(gpu, cols):
    rng = np.random.default_rng(cols)
    m = rng.integers(0, 65536, (32, cols)).astype(np.uint16)
    md = torch.from_numpy(m.view(np.int16)).cuda()
    nfrag = (cols // 32) * 2
    out = torch.zeros(nfrag * 64 * 4, dtype=torch.int32, device="cuda")
    call("srk_diag_tr16_read", ptr(md), cols, ptr(out), stream_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint16).reshape(nfrag, 64, 8)
    f = 0
    for r0 in range(0, cols, 32):
        for kk in (0, 16):
            lane = np.arange(64)
            exp = np.stack([m[kk + 8 * (lane >> 5) + e, r0 + (lane & 31)] for e in range(8)], axis=1)
            assert np.array_equal(got[f], exp), (cols, r0, kk)
            f += 1
