// fp32 GEMM on the gfx950 matrix cores: v_mfma_f32_16x16x4_f32 (exact fp32 fma chain, the same
// numerics class as the reference's fp32 cuDNN/CPU GEMMs; SURVEY.md Appendix A "logits 1e-4").
//
// Tile: BM x BN x BK per 256-thread workgroup (2 x 2 waves), each wave owns a (BM/2) x (BN/2)
// block of 16x16 MFMA tiles.  Operands are staged k-major in LDS ([k][m] and [k][n], rows padded
// by 16 floats so the two 32-lane halves of a ds_read_b32 hit disjoint banks), double-buffered
// with register prefetch of tile k+1 while tile k is multiplied.  Out-of-range rows/cols/k are
// zero-filled, so any M, N, K, leading dimension and transpose combination is valid.
#include "gemm.h"

namespace srk {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 load4(const float* __restrict__ p, int64_t ld, int64_t r, int64_t c0,
                                        int64_t R, int64_t C, bool vec) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (r < R) {
    const float* q = p + r * ld + c0;
    if (vec && c0 + 3 < C) {
      v = *reinterpret_cast<const float4*>(q);
    } else {
      if (c0 + 0 < C) v.x = q[0];
      if (c0 + 1 < C) v.y = q[1];
      if (c0 + 2 < C) v.z = q[2];
      if (c0 + 3 < C) v.w = q[3];
    }
  }
  return v;
}

template <bool TA, bool TB, int BM, int BN, int BK>
struct Tile {
  static constexpr int NT = 256;
  static constexpr int LA = BM + 16, LB = BN + 16;
  static constexpr int VA = BM * BK / 4 / NT;   // float4 vectors per thread
  static constexpr int VB = BN * BK / 4 / NT;
  static_assert(VA >= 1 && VB >= 1, "tile too small for 256 threads");
  static constexpr int TM = BM / 2 / 16, TN = BN / 2 / 16;
};

template <bool TA, bool TB, int BM, int BN, int BK>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmDesc d, int tiles_n, int vec_a, int vec_b) {
  using T = Tile<TA, TB, BM, BN, BK>;
  __shared__ float As[2][BK][T::LA];
  __shared__ float Bs[2][BK][T::LB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int64_t z = blockIdx.z;
  const float* __restrict__ A = d.A + z * d.sA;
  const float* __restrict__ B = d.B + z * d.sB;
  float* __restrict__ C = d.C + z * d.sC;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int wm0 = (wave >> 1) * (BM / 2), wn0 = (wave & 1) * (BN / 2);

  float4 ra[T::VA], rb[T::VB];
  auto load_tile = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < T::VA; ++i) {
      const int vi = tid + i * T::NT;
      if (!TA) {   // A [M][K]: vectors along k
        const int row = vi / (BK / 4), kq = (vi % (BK / 4)) * 4;
        ra[i] = load4(A, d.lda, m0 + row, k0 + kq, d.M, d.K, vec_a);
      } else {     // A stored [K][M]: vectors along m
        const int kr = vi / (BM / 4), mq = (vi % (BM / 4)) * 4;
        ra[i] = load4(A, d.lda, k0 + kr, m0 + mq, d.K, d.M, vec_a);
      }
    }
#pragma unroll
    for (int i = 0; i < T::VB; ++i) {
      const int vi = tid + i * T::NT;
      if (!TB) {   // B [K][N]: vectors along n
        const int kr = vi / (BN / 4), nq = (vi % (BN / 4)) * 4;
        rb[i] = load4(B, d.ldb, k0 + kr, n0 + nq, d.K, d.N, vec_b);
      } else {     // B stored [N][K]: vectors along k
        const int row = vi / (BK / 4), kq = (vi % (BK / 4)) * 4;
        rb[i] = load4(B, d.ldb, n0 + row, k0 + kq, d.N, d.K, vec_b);
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < T::VA; ++i) {
      const int vi = tid + i * T::NT;
      if (!TA) {
        const int row = vi / (BK / 4), kq = (vi % (BK / 4)) * 4;
        As[buf][kq + 0][row] = ra[i].x;
        As[buf][kq + 1][row] = ra[i].y;
        As[buf][kq + 2][row] = ra[i].z;
        As[buf][kq + 3][row] = ra[i].w;
      } else {
        const int kr = vi / (BM / 4), mq = (vi % (BM / 4)) * 4;
        *reinterpret_cast<float4*>(&As[buf][kr][mq]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < T::VB; ++i) {
      const int vi = tid + i * T::NT;
      if (!TB) {
        const int kr = vi / (BN / 4), nq = (vi % (BN / 4)) * 4;
        *reinterpret_cast<float4*>(&Bs[buf][kr][nq]) = rb[i];
      } else {
        const int row = vi / (BK / 4), kq = (vi % (BK / 4)) * 4;
        Bs[buf][kq + 0][row] = rb[i].x;
        Bs[buf][kq + 1][row] = rb[i].y;
        Bs[buf][kq + 2][row] = rb[i].z;
        Bs[buf][kq + 3][row] = rb[i].w;
      }
    }
  };

  f32x4 acc[T::TM][T::TN];
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t nk = (d.K + BK - 1) / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  const int lr = lane >> 4, lc = lane & 15;
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = (int)(kt & 1);
    if (kt + 1 < nk) load_tile((kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      float a[T::TM], b[T::TN];
#pragma unroll
      for (int i = 0; i < T::TM; ++i) a[i] = As[cur][kk + lr][wm0 + i * 16 + lc];
#pragma unroll
      for (int j = 0; j < T::TN; ++j) b[j] = Bs[cur][kk + lr][wn0 + j * 16 + lc];
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
#pragma unroll
        for (int j = 0; j < T::TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // epilogue: D[row][col], row = 4*(lane>>4) + r, col = lane & 15 within each 16x16 tile
#pragma unroll
  for (int i = 0; i < T::TM; ++i) {
#pragma unroll
    for (int j = 0; j < T::TN; ++j) {
      const int64_t col = n0 + wn0 + j * 16 + lc;
      if (col >= d.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm0 + i * 16 + lr * 4 + r;
        if (row >= d.M) continue;
        float v = d.alpha * acc[i][j][r];
        if (d.bias_mode == 1) v += d.bias[col];
        else if (d.bias_mode == 2) v += d.bias[row];
        float* c = C + row * d.ldc + col;
        if (d.beta != 0.f) v += d.beta * *c;
        *c = v;
      }
    }
  }
}

template <bool TA, bool TB, int BM, int BN, int BK>
int launch(const GemmDesc& d, hipStream_t s, bool vec_a, bool vec_b) {
  const int64_t tm = (d.M + BM - 1) / BM, tn = (d.N + BN - 1) / BN;
  SRK_REQUIRE(tm * tn <= INT32_MAX && d.batch <= 65535, SRK_ERR_INVALID, "gemm: grid too large");
  ProfScope prof("gemm_f32", s, 2.0 * (double)d.M * (double)d.N * (double)d.K * d.batch);
  hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, BM, BN, BK>), dim3((unsigned)(tm * tn), 1, (unsigned)d.batch),
                     dim3(256), 0, s, d, (int)tn, (int)vec_a, (int)vec_b);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

template <bool TA, bool TB>
int dispatch_tile(const GemmDesc& d, hipStream_t s, bool va, bool vb) {
  const int64_t big_tiles = ((d.M + 127) / 128) * ((d.N + 127) / 128) * d.batch;
  if (big_tiles >= 256) return launch<TA, TB, 128, 128, 16>(d, s, va, vb);
  return launch<TA, TB, 64, 64, 16>(d, s, va, vb);
}

// ------------------------------------------------------------------ column sums
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, int64_t M, int64_t N, int64_t ldx,
                                                     float* __restrict__ out, float beta) {
  __shared__ float part[4][64];
  const int c = threadIdx.x & 63, rp = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + c;
  float s = 0.f;
  if (col < N)
    for (int64_t m = rp; m < M; m += 4) s += X[m * ldx + col];
  part[rp][c] = s;
  __syncthreads();
  if (rp == 0 && col < N) {
    const float t = (part[0][c] + part[1][c]) + (part[2][c] + part[3][c]);
    out[col] = beta != 0.f ? beta * out[col] + t : t;
  }
}

}  // namespace

int gemm_f32(const GemmDesc& d, hipStream_t s) {
  SRK_REQUIRE(d.M >= 0 && d.N >= 0 && d.K >= 0 && d.batch >= 1, SRK_ERR_INVALID, "gemm: bad shape");
  if (d.M == 0 || d.N == 0) return SRK_OK;
  SRK_REQUIRE(d.C && (d.K == 0 || (d.A && d.B)), SRK_ERR_INVALID, "gemm: null operand");
  SRK_REQUIRE(d.bias_mode == 0 || d.bias, SRK_ERR_INVALID, "gemm: bias_mode without bias");
  const bool va = (d.lda % 4 == 0) && ((uintptr_t)d.A % 16 == 0) && (d.sA % 4 == 0);
  const bool vb = (d.ldb % 4 == 0) && ((uintptr_t)d.B % 16 == 0) && (d.sB % 4 == 0);
  if (!d.ta && !d.tb) return dispatch_tile<false, false>(d, s, va, vb);
  if (!d.ta && d.tb) return dispatch_tile<false, true>(d, s, va, vb);
  if (d.ta && !d.tb) return dispatch_tile<true, false>(d, s, va, vb);
  return dispatch_tile<true, true>(d, s, va, vb);
}

int colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, float beta, hipStream_t s) {
  if (N == 0) return SRK_OK;
  hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, s, X, M, N, ldx, out, beta);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

}  // namespace srk

extern "C" int srk_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                            int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc,
                            const float* bias, int bias_mode, void* stream) {
  SRK_API_BEGIN
  srk::GemmDesc d;
  d.M = M; d.N = N; d.K = K;
  d.A = A; d.lda = lda; d.ta = trans_a != 0;
  d.B = B; d.ldb = ldb; d.tb = trans_b != 0;
  d.C = C; d.ldc = ldc; d.alpha = alpha; d.beta = beta;
  d.bias = bias; d.bias_mode = bias_mode;
  SRK_REQUIRE(bias_mode >= 0 && bias_mode <= 2, SRK_ERR_INVALID, "gemm: bias_mode must be 0, 1 or 2");
  return srk::gemm_f32(d, srk::as_stream(stream));
  SRK_API_END
}

extern "C" int srk_colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, float beta, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(M >= 0 && N >= 0 && (N == 0 || (X && out)), SRK_ERR_INVALID, "colsum: bad args");
  return srk::colsum_f32(X, M, N, ldx, out, beta, srk::as_stream(stream));
  SRK_API_END
}
