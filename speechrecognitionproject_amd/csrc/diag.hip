// Directed diagnostics of two instruction patterns whose round-5 uses gave wrong results in
// conv_row16_dgrad_kernel (VERDICT r05 "next" #8; tests/test_diag_gpu.py runs each once).
//
// 1. The epilogue's raw buffer stores of MFMA accumulators, with the kernel's exact descriptor
//    (num_records 0x7ffffff0, word3 0x00020000), voffset formula (tile base + (p * 64 + lane) * 4, the
//    column block + 128 B) and out-of-range value (0x80000000 -> dropped).  Root cause found on the host
//    from the ISA (hipcc of ROCm 7.2, device -S): the round-5 source passed
//    `__builtin_bit_cast(unsigned, acc[i][j][r])` — a bit cast of an ext_vector COMPONENT lvalue — and clang
//    lowers it to a copy from the vector's address, i.e. component 0: every unrolled store of the r loop
//    stored the same register (`buffer_store_dword a16 ...` x 16), so 15 of 16 outputs were wrong.  The
//    buffer store itself, its descriptor and offsets are correct.  Fix: cast the component to a value first
//    (`__builtin_bit_cast(unsigned, (float)acc[i][j][r])` or `__float_as_uint`).  No such bit cast remains in
//    the product sources (grep: every other __builtin_bit_cast takes a whole vector or an array element).
//    variant 0 = the fixed form, variant 1 = the round-5 form (kept to show the bug on the device).
// 2. ds_read_b64_tr_b16 fragments of a 64-column TR image (the removed r16_off64 / r16_frag64 of the first
//    row-staged data gradient) and of the 128-column image the ring / row-staged kernels use (r16_off<false>):
//    the fragment lane l receives is M[kk + 8 (l >> 5) + e][r0 + (l & 31)], e = 0..7 (the 32x32x16 B operand).
#include "srk_internal.h"

namespace srk {
namespace {

typedef float f32x16d __attribute__((ext_vector_type(16)));
typedef unsigned u32x4d __attribute__((ext_vector_type(4)));
typedef unsigned u32x2d __attribute__((ext_vector_type(2)));
typedef short s16x4d __attribute__((ext_vector_type(4)));

// the row16 dgrad epilogue: tile g = 8 image rows x 40 pixels x 64 channels, its first 32 pixels in the 32x32
// accumulator layout of two column blocks j (register r of lane l: pixel p = (r & 3) + 8 (r >> 2) + 4 (l >> 5),
// channel 32 j + (l & 31)).  Known values from one MFMA with k = 2: A[p][0] = p, B[0][n] = 64, A[p][1] = 1,
// B[1][n] = 1 + 32 j + n + 2048 g, so C[p][32 j + n] = 1 + 64 p + 32 j + n + 2048 g (exact in fp32).
template <int VARIANT>
__global__ __launch_bounds__(64) void acc_store_kernel(float* dx, int rows_total) {
  const int lane = threadIdx.x, lh = lane >> 5, lc = lane & 31, g = blockIdx.x;
  f32x16d acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const float a = lh ? 1.f : (float)lc;                                            // A[m = l & 31][k = l >> 5]
    const float b = lh ? (float)(1 + 32 * j + lc + 2048 * g) : 64.f;                 // B[k = l >> 5][n = l & 31]
    acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
  }
  const auto rsX = __builtin_amdgcn_make_buffer_rsrc(dx, (short)0, 0x7ffffff0, 0x00020000);
  const int sbase = __builtin_amdgcn_readfirstlane(g * 8 * 40 * 64 * 4);
  const int nreal = (rows_total - g * 8) * 40;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int p = (r & 3) + 8 * (r >> 2) + 4 * lh;
    const int off = p < nreal ? sbase + (p * 64 + lc) * 4 : (int)0x80000000u;
    unsigned v0, v1;
    if (VARIANT == 0) {
      v0 = __builtin_bit_cast(unsigned, (float)acc[0][r]);
      v1 = __builtin_bit_cast(unsigned, (float)acc[1][r]);
    } else {
      v0 = __builtin_bit_cast(unsigned, acc[0][r]);   // the round-5 form: component lvalue
      v1 = __builtin_bit_cast(unsigned, acc[1][r]);
    }
    __builtin_amdgcn_raw_buffer_store_b32(v0, rsX, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(v1, rsX, p < nreal ? off + 128 : (int)0x80000000u, 0, 0);
  }
}

__device__ __forceinline__ int off64(int col, int k) {   // the removed r16_off64
  return k * 64 + ((((col >> 3) ^ (((k >> 1) & 1) << 2))) << 3) + (col & 7);
}
__device__ __forceinline__ int off128(int col, int k) {   // r16_off<false> (conv.hip)
  return k * 128 + ((((col >> 3) ^ ((k & 3) << 2))) << 3) + (col & 7);
}

// one wave: logical M [32 k][W cols] (16-bit) -> the swizzled TR image in LDS; every (r0, kk) fragment of
// the image -> out[frag][lane][4 dwords]
template <int W>
__global__ __launch_bounds__(64) void tr16_read_kernel(const unsigned short* M, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned short img[32 * W];
  const int lane = threadIdx.x;
  for (int i = lane; i < 32 * W; i += 64) {
    const int k = i / W, col = i % W;
    img[W == 64 ? off64(col, k) : off128(col, k)] = M[i];
  }
  __syncthreads();
  typedef __attribute__((address_space(3))) s16x4d lds_s16x4;
  int f = 0;
  for (int r0 = 0; r0 < W; r0 += 32)
    for (int kk = 0; kk < 32; kk += 16, ++f) {
      const int q = (lane >> 2) & 3, pp = lane & 3;
      const int k = kk + 8 * (lane >> 5) + q, col = r0 + 16 * ((lane >> 4) & 1) + 4 * pp;
      const int o0 = W == 64 ? off64(col, k) : off128(col, k), o1 = W == 64 ? off64(col, k + 4) : off128(col, k + 4);
      const s16x4d lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o0));
      const s16x4d hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o1));
      const u32x2d l2 = __builtin_bit_cast(u32x2d, lo), h2 = __builtin_bit_cast(u32x2d, hi);
      *reinterpret_cast<u32x4d*>(out + ((size_t)f * 64 + lane) * 4) = u32x4d{l2.x, l2.y, h2.x, h2.y};
    }
}

}  // namespace
}  // namespace srk

extern "C" {

int srk_diag_acc_store(float* dx, int64_t rows, int variant, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(dx && rows > 0 && rows % 8 == 0 && rows * 40 * 64 * 4 < 0x7ffffff0LL && rows / 8 * 2048 < (1 << 24) &&
                  (variant == 0 || variant == 1),
              SRK_ERR_INVALID, "diag_acc_store: rows a positive multiple of 8 (< 65536), variant 0 / 1");
  const dim3 grid((unsigned)(rows / 8));
  if (variant == 0) hipLaunchKernelGGL(srk::acc_store_kernel<0>, grid, dim3(64), 0, srk::as_stream(stream), dx, (int)rows);
  else hipLaunchKernelGGL(srk::acc_store_kernel<1>, grid, dim3(64), 0, srk::as_stream(stream), dx, (int)rows);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_diag_tr16_read(const uint16_t* m, int64_t cols, uint32_t* out, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(m && out && (cols == 64 || cols == 128), SRK_ERR_INVALID, "diag_tr16_read: cols 64 or 128");
  if (cols == 64)
    hipLaunchKernelGGL(srk::tr16_read_kernel<64>, dim3(1), dim3(64), 0, srk::as_stream(stream), m, out);
  else
    hipLaunchKernelGGL(srk::tr16_read_kernel<128>, dim3(1), dim3(64), 0, srk::as_stream(stream), m, out);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
