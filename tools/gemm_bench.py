"""GEMM micro-benchmark: the fp32 GEMM shapes of one model_mfcc_bgru train step (B = 256, T = 51,
H = 512 by default; --B 512 --T 49 for cfg5), timed with srk_prof events and checked against torch fp32 matmul on the same device.

    python tools/gemm_bench.py [--reps 10] [--precision fp32|bf16|fp16]
                                                 (env SRK_GEMM_REMAP=0 disables the XCD remap)
With --precision bf16 / fp16 the yardstick is torch.matmul on operands already converted to that
dtype (hipBLASLt reading 16-bit operands; ours reads the fp32 tensors and rounds on chip).
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speechrecognitionproject_amd import _lib  # noqa: E402

H = 512


def shapes(B, T):
    BT = B * T
    # name, ta, tb, M, N, K, lda, ldb  (A stored [M][K] or [K][M] when ta; B stored [K][N] or [N][K] when tb)
    return [
        ("gi_l1", 0, 1, BT, 6 * H, 1024, 1024, 1024),
        ("gi_l0", 0, 1, BT, 6 * H, 39, 39, 39),
        ("dx_l1", 0, 0, BT, 1024, 6 * H, 6 * H, 1024),
        ("dWih_l1", 1, 0, 6 * H, 1024, BT, 6 * H, 1024),
        ("dWih_l0", 1, 0, 6 * H, 39, BT, 6 * H, 39),
        ("dWhh", 1, 0, 3 * H, H, BT - 1, 3 * H, 2 * H),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16", "fp16"])
    ap.add_argument("--h16", action="store_true", help="operands pre-converted to 16 bit (srk_gemm_16)")
    ap.add_argument("--kernel16", type=int, default=0,
                    help="srk option gemm16_kernel: 0 by shape, 1 register-staged, 2 LDS-DMA ping-pong")
    ap.add_argument("--kernel32", type=int, default=0, help="srk option gemm32_kernel (the same for fp32)")
    ap.add_argument("--B", type=int, default=256, help="clips per step (cfg5: 512)")
    ap.add_argument("--T", type=int, default=51, help="frames per clip (cfg5: 49)")
    ap.add_argument("--only", default="", help="comma-separated shape names")
    a = ap.parse_args()
    _lib.set_matmul_precision(a.precision)
    _lib.call("srk_set_option", b"gemm16_kernel", a.kernel16)
    _lib.call("srk_set_option", b"gemm32_kernel", a.kernel32)
    pname = {"fp32": "gemm_f32", "bf16": "gemm_bf16", "fp16": "gemm_f16"}[a.precision]
    peak = 157.3 if a.precision == "fp32" else 2500.0
    tdt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[a.precision]
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    g = torch.Generator(device=dev).manual_seed(0)
    for name, ta, tb, M, N, K, lda, ldb in shapes(a.B, a.T):
        if a.only and name not in a.only.split(","):
            continue
        A = torch.randn((K if ta else M) * lda, device=dev, generator=g)
        Bm = torch.randn((N if tb else K) * ldb, device=dev, generator=g)
        C = torch.empty(M * N, device=dev)
        rs = torch.empty(M, device=dev)
        args = (ta, tb, M, N, K, 1.0, A.data_ptr(), lda, Bm.data_ptr(), ldb, 0.0, C.data_ptr(), N)
        fn = lambda: _lib.call("srk_gemm_rowsum_f32", *args, rs.data_ptr(), stream) if ta else \
            _lib.call("srk_gemm_f32", *args, None, 0, stream)
        if a.h16 and (M % 8 or N % 8 or K % 8):   # srk_gemm_16 needs 8-element multiples
            continue
        if a.h16:   # 16-bit operands in memory (leading dims rounded up to 8 elements)
            lda8, ldb8 = (lda + 7) // 8 * 8, (ldb + 7) // 8 * 8
            A16 = torch.zeros((K if ta else M), lda8, device=dev, dtype=tdt)
            A16[:, :lda] = A.view(-1, lda).to(tdt)
            B16 = torch.zeros((N if tb else K), ldb8, device=dev, dtype=tdt)
            B16[:, :ldb] = Bm.view(-1, ldb).to(tdt)
            Kp = K if (ta or K % 8 == 0) and (not tb or K % 8 == 0) else (K + 7) // 8 * 8
            args16 = (ta, tb, M, N, Kp, 1.0, A16.data_ptr(), lda8, B16.data_ptr(), ldb8, 0.0, C.data_ptr(), N)
            fn = lambda: _lib.call("srk_gemm_16", *args16, None, 0, stream)
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        _lib.prof_enable(True)
        for _ in range(a.reps):
            fn()
        c, ms, w = _lib.prof_read(pname)
        _lib.prof_enable(False)
        Am = (A.view(K, lda)[:, :M].t() if ta else A.view(M, lda)[:, :K])
        Bmm = (Bm.view(N, ldb)[:, :K].t() if tb else Bm.view(K, ldb)[:, :N])
        ref = Am.to(tdt).float() @ Bmm.to(tdt).float()
        err = float((C.view(M, N) - ref).abs().max() / ref.abs().max())
        tf = w / (ms * 1e-3) / 1e12
        # yardstick: torch.matmul (hipBLASLt / rocBLAS fp32) on the same operands
        Am, Bmm = Am.to(tdt), Bmm.to(tdt)
        out = torch.empty(ref.shape, device=dev, dtype=tdt)
        for _ in range(2):
            torch.matmul(Am, Bmm, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            torch.matmul(Am, Bmm, out=out)
        e1.record()
        torch.cuda.synchronize()
        t_us = e0.elapsed_time(e1) / a.reps * 1e3
        res[name] = {"us": round(ms / c * 1e3, 1), "TF": round(tf, 1), "frac": round(tf / peak, 3), "rel_err": err,
                     "torch_us": round(t_us, 1), "torch_TF": round(2.0 * M * N * K / (t_us * 1e-6) / 1e12, 1)}
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps({"remap": os.environ.get("SRK_GEMM_REMAP", "1"), "kernel16": a.kernel16, "kernel32": a.kernel32, "shapes": res}))


if __name__ == "__main__":
    main()
