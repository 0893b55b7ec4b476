// fp32 GEMM on the gfx950 matrix cores: v_mfma_f32_32x32x2_f32 (exact fp32 fma chain — the same
// numerics class as the reference's fp32 cuBLAS/CPU GEMMs; SURVEY.md Appendix A "logits 1e-4").
//
// Tile: BM x BN x BK per 256-thread workgroup (2 x 2 waves), each wave owns (BM/2) x (BN/2) as
// 32x32 MFMA tiles (64 FLOP/clk/SIMD, one f32 operand per lane per 2-deep k step).  Operands are
// staged k-major in LDS ([k][m], [k][n]) through registers, double-buffered: tile k+1 is fetched
// while tile k is multiplied.  Rows written by scalar transposing stores get a +1 float pad
// (conflict-free ds_write_b32), rows written by float4 stores stay unpadded.
//
// Tall-K shapes that would leave the chip under-filled (the weight-gradient GEMMs, K = B*T) are
// split over K: each split writes an fp32 partial slab, a second kernel sums the slabs in a fixed
// order (deterministic) and applies alpha / beta / bias.  Optionally the kernel also produces
// rowsum[m] = sum_k op(A)[m, k] from the A tiles it already stages (the bias gradient of a
// dW = dY^T X GEMM, fused: no separate pass over dY).
#include <mutex>

#include "gemm.h"

namespace srk {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// p[r][c0..c0+3] (contiguous along c), zero outside rows [0, r_end) and columns [0, c_end)
__device__ __forceinline__ float4 load4(const float* __restrict__ p, int64_t ld, int64_t r, int64_t r_end, int64_t c0,
                                        int64_t c_end, bool vec) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (r < r_end) {
    const float* q = p + r * ld + c0;
    if (vec && c0 + 3 < c_end) {
      v = *reinterpret_cast<const float4*>(q);
    } else {
      if (c0 + 0 < c_end) v.x = q[0];
      if (c0 + 1 < c_end) v.y = q[1];
      if (c0 + 2 < c_end) v.z = q[2];
      if (c0 + 3 < c_end) v.w = q[3];
    }
  }
  return v;
}

struct KernelArgs {
  GemmDesc d;
  int tiles_n;
  int vec_a, vec_b;
  int64_t kchunk;        // K range per split
  float* partial;        // [splits][M][N] when split
  float* rs_partial;     // [splits][M] when split and rowsum requested
};

template <bool TA, bool TB, int BM, int BN, int BK>
__global__ __launch_bounds__(256) void gemm_f32_kernel(KernelArgs ka) {
  constexpr int NT = 256;
  constexpr int LA = TA ? BM : BM + 1;   // float4 stores (TA) stay aligned; scalar stores get +1
  constexpr int LB = TB ? BN + 1 : BN;
  constexpr int VA = BM * BK / 4 / NT, VB = BN * BK / 4 / NT;
  constexpr int TM = BM / 64, TN = BN / 64;   // 32x32 tiles per wave per dim
  static_assert(VA >= 1 && VB >= 1 && TM >= 1 && TN >= 1, "bad tile");
  __shared__ float As[2][BK][LA];
  __shared__ float Bs[2][BK][LB];
  const GemmDesc& d = ka.d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tm = blockIdx.x / ka.tiles_n, tn = blockIdx.x % ka.tiles_n;
  const int split = blockIdx.y;
  const int64_t z = blockIdx.z;
  const float* __restrict__ A = d.A + z * d.sA;
  const float* __restrict__ B = d.B + z * d.sB;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kb = split * ka.kchunk;
  const int64_t ke = (kb + ka.kchunk < d.K) ? kb + ka.kchunk : d.K;
  const int wm0 = (wave >> 1) * (BM / 2), wn0 = (wave & 1) * (BN / 2);
  const bool do_rs = d.rowsum != nullptr && tn == 0;

  float4 ra[VA], rb[VB];
  auto load_tile = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < VA; ++i) {
      const int vi = tid + i * NT;
      if (!TA) {   // A [M][K]: vectors along k
        const int row = vi / (BK / 4), kq = (vi % (BK / 4)) * 4;
        ra[i] = load4(A, d.lda, m0 + row, d.M, k0 + kq, ke, ka.vec_a);
      } else {     // A stored [K][M]: vectors along m
        const int kr = vi / (BM / 4), mq = (vi % (BM / 4)) * 4;
        ra[i] = load4(A, d.lda, k0 + kr, ke, m0 + mq, d.M, ka.vec_a);
      }
    }
#pragma unroll
    for (int i = 0; i < VB; ++i) {
      const int vi = tid + i * NT;
      if (!TB) {   // B [K][N]: vectors along n
        const int kr = vi / (BN / 4), nq = (vi % (BN / 4)) * 4;
        rb[i] = load4(B, d.ldb, k0 + kr, ke, n0 + nq, d.N, ka.vec_b);
      } else {     // B stored [N][K]: vectors along k
        const int row = vi / (BK / 4), kq = (vi % (BK / 4)) * 4;
        rb[i] = load4(B, d.ldb, n0 + row, d.N, k0 + kq, ke, ka.vec_b);
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < VA; ++i) {
      const int vi = tid + i * NT;
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
    for (int i = 0; i < VB; ++i) {
      const int vi = tid + i * NT;
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

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // fused rowsum: thread owns row (tid % BM) and k phase (tid / BM)
  constexpr int RSP = NT / BM;
  float rs = 0.f;

  const int64_t nk = ke > kb ? (ke - kb + BK - 1) / BK : 0;
  const int lk = lane >> 5, lc = lane & 31;
  if (nk > 0) {
    load_tile(kb);
    store_tile(0);
  }
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = (int)(kt & 1);
    if (kt + 1 < nk) load_tile(kb + (kt + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[cur][kk + lk][wm0 + i * 32 + lc];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[cur][kk + lk][wn0 + j * 32 + lc];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (do_rs) {
#pragma unroll
      for (int k = tid / BM; k < BK; k += RSP) rs += As[cur][k][tid % BM];
    }
    asm volatile("" ::: "memory");      // keep the stage-k+1 LDS store (and its vmcnt wait)
      __builtin_amdgcn_sched_barrier(0);   // after this stage's MFMAs
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  const bool split_mode = ka.partial != nullptr;
  // epilogue.  32x32 accumulator: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t col = n0 + wn0 + j * 32 + lc;
      if (col >= d.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row >= d.M) continue;
        if (split_mode) {
          ka.partial[((int64_t)split * d.M + row) * d.N + col] = acc[i][j][r];
          continue;
        }
        float* C = d.C + z * d.sC;
        float v = d.alpha * acc[i][j][r];
        if (d.bias_mode == 1) v += d.bias[col];
        else if (d.bias_mode == 2) v += d.bias[row];
        float* c = C + row * d.ldc + col;
        if (d.beta != 0.f) v += d.beta * *c;
        *c = v;
      }
    }
  }
  if (do_rs) {
    float* red = &As[0][0][0];
    __syncthreads();
    red[tid] = rs;
    __syncthreads();
    if (tid < BM) {
      float t = 0.f;
#pragma unroll
      for (int p = 0; p < RSP; ++p) t += red[p * BM + tid];
      const int64_t row = m0 + tid;
      if (row < d.M) {
        if (split_mode) ka.rs_partial[(int64_t)split * d.M + row] = t;
        else d.rowsum[row] = d.rowsum_beta != 0.f ? d.rowsum_beta * d.rowsum[row] + t : t;
      }
    }
  }
}

// Sums the split-K slabs in split order and applies the GEMM epilogue.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmDesc d, const float* __restrict__ partial, int splits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.M * d.N) return;
  const int64_t row = i / d.N, col = i % d.N;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += partial[(int64_t)k * d.M * d.N + i];
  float v = d.alpha * s;
  if (d.bias_mode == 1) v += d.bias[col];
  else if (d.bias_mode == 2) v += d.bias[row];
  float* c = d.C + row * d.ldc + col;
  if (d.beta != 0.f) v += d.beta * *c;
  *c = v;
}

__global__ void rowsum_reduce_kernel(float* __restrict__ out, float beta, const float* __restrict__ rp, int64_t M,
                                     int splits) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float t = 0.f;
  for (int k = 0; k < splits; ++k) t += rp[(int64_t)k * M + m];
  out[m] = beta != 0.f ? beta * out[m] + t : t;
}

// ------------------------------------------------------------------ column sums (rows split)
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, int64_t M, int64_t N, int64_t ldx,
                                                     float* __restrict__ out, float beta, int64_t rows_per,
                                                     float* __restrict__ part_out) {
  __shared__ float part[4][64];
  const int c = threadIdx.x & 63, rp = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + c;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = r0 + rows_per < M ? r0 + rows_per : M;
  float s = 0.f;
  if (col < N)
    for (int64_t m = r0 + rp; m < r1; m += 4) s += X[m * ldx + col];
  part[rp][c] = s;
  __syncthreads();
  if (rp == 0 && col < N) {
    const float t = (part[0][c] + part[1][c]) + (part[2][c] + part[3][c]);
    if (part_out) part_out[(int64_t)blockIdx.y * N + col] = t;
    else out[col] = beta != 0.f ? beta * out[col] + t : t;
  }
}

// ------------------------------------------------------------------ scratch (split-K slabs)
struct Scratch {
  float* p = nullptr;
  size_t floats = 0;
};
Scratch g_scratch[64];
std::mutex g_scratch_mu;

int get_scratch(size_t floats, float** out) {
  int dev = 0;
  SRK_CHECK_HIP(hipGetDevice(&dev));
  SRK_REQUIRE(dev >= 0 && dev < 64, SRK_ERR_INVALID, "device out of range");
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  Scratch& s = g_scratch[dev];
  if (s.floats < floats) {   // grow-only: steady state never allocates
    if (s.p) {
      SRK_CHECK_HIP(hipDeviceSynchronize());
      SRK_CHECK_HIP(hipFree(s.p));
      s.p = nullptr;
    }
    const size_t want = floats + floats / 4;
    SRK_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&s.p), want * sizeof(float)));
    s.floats = want;
  }
  *out = s.p;
  return SRK_OK;
}

template <bool TA, bool TB, int BM, int BN, int BK>
int launch(const GemmDesc& d, hipStream_t s, bool vec_a, bool vec_b) {
  const int64_t tm = (d.M + BM - 1) / BM, tn = (d.N + BN - 1) / BN;
  SRK_REQUIRE(tm * tn <= INT32_MAX && d.batch <= 65535, SRK_ERR_INVALID, "gemm: grid too large");
  KernelArgs ka{};
  ka.d = d;
  ka.tiles_n = (int)tn;
  ka.vec_a = vec_a;
  ka.vec_b = vec_b;
  // split K when the output grid cannot fill the chip (256 CUs) and K is long
  int splits = 1;
  const int64_t tiles = tm * tn * d.batch;
  if (d.batch == 1 && tiles < 256 && d.K >= 16 * BK) {
    splits = (int)std::min<int64_t>((512 + tiles - 1) / tiles, d.K / (4 * BK));
    splits = std::max(1, std::min(splits, 16));
  }
  ka.kchunk = splits > 1 ? ((d.K + splits - 1) / splits + BK - 1) / BK * BK : std::max<int64_t>(d.K, 1);
  if (splits > 1) splits = (int)((d.K + ka.kchunk - 1) / ka.kchunk);
  if (splits > 1) {
    float* scratch = nullptr;
    const size_t need = (size_t)splits * d.M * d.N + (d.rowsum ? (size_t)splits * d.M : 0);
    if (int rc = get_scratch(need, &scratch)) return rc;
    ka.partial = scratch;
    ka.rs_partial = d.rowsum ? scratch + (size_t)splits * d.M * d.N : nullptr;
  }
  ProfScope prof("gemm_f32", s, 2.0 * (double)d.M * (double)d.N * (double)d.K * d.batch);
  hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, BM, BN, BK>), dim3((unsigned)(tm * tn), (unsigned)splits,
                     (unsigned)d.batch), dim3(256), 0, s, ka);
  SRK_CHECK_HIP(hipGetLastError());
  if (splits > 1) {
    const int64_t n = d.M * d.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, ka.partial,
                       splits);
    if (d.rowsum)
      hipLaunchKernelGGL(rowsum_reduce_kernel, dim3((unsigned)((d.M + 255) / 256)), dim3(256), 0, s, d.rowsum,
                         d.rowsum_beta, ka.rs_partial, d.M, splits);
    SRK_CHECK_HIP(hipGetLastError());
  }
  return SRK_OK;
}

template <bool TA, bool TB>
int dispatch_tile(const GemmDesc& d, hipStream_t s, bool va, bool vb) {
  const int64_t big_tiles = ((d.M + 127) / 128) * ((d.N + 127) / 128) * d.batch;
  if (big_tiles >= 64 || d.K >= 2048) return launch<TA, TB, 128, 128, 32>(d, s, va, vb);
  return launch<TA, TB, 64, 64, 32>(d, s, va, vb);
}

}  // namespace

int gemm_f32(const GemmDesc& d, hipStream_t s) {
  SRK_REQUIRE(d.M >= 0 && d.N >= 0 && d.K >= 0 && d.batch >= 1, SRK_ERR_INVALID, "gemm: bad shape");
  if (d.M == 0 || d.N == 0) return SRK_OK;
  SRK_REQUIRE(d.C && (d.K == 0 || (d.A && d.B)), SRK_ERR_INVALID, "gemm: null operand");
  SRK_REQUIRE(d.bias_mode == 0 || d.bias, SRK_ERR_INVALID, "gemm: bias_mode without bias");
  SRK_REQUIRE(!d.rowsum || d.batch == 1, SRK_ERR_INVALID, "gemm: rowsum needs batch == 1");
  const bool va = (d.lda % 4 == 0) && ((uintptr_t)d.A % 16 == 0) && (d.sA % 4 == 0);
  const bool vb = (d.ldb % 4 == 0) && ((uintptr_t)d.B % 16 == 0) && (d.sB % 4 == 0);
  if (!d.ta && !d.tb) return dispatch_tile<false, false>(d, s, va, vb);
  if (!d.ta && d.tb) return dispatch_tile<false, true>(d, s, va, vb);
  if (d.ta && !d.tb) return dispatch_tile<true, false>(d, s, va, vb);
  return dispatch_tile<true, true>(d, s, va, vb);
}

int colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, float beta, hipStream_t s) {
  if (N == 0) return SRK_OK;
  const int64_t cblocks = (N + 63) / 64;
  int64_t rsplit = 1;
  if (cblocks < 256 && M >= 2048) rsplit = std::min<int64_t>((512 + cblocks - 1) / cblocks, (M + 511) / 512);
  if (rsplit <= 1) {
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)cblocks, 1), dim3(256), 0, s, X, M, N, ldx, out, beta, M,
                       (float*)nullptr);
  } else {
    const int64_t rows_per = (M + rsplit - 1) / rsplit;
    float* part = nullptr;
    if (int rc = get_scratch((size_t)rsplit * N, &part)) return rc;
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)cblocks, (unsigned)rsplit), dim3(256), 0, s, X, M, N, ldx, out,
                       beta, rows_per, part);
    hipLaunchKernelGGL(rowsum_reduce_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, out, beta, part, N,
                       (int)rsplit);
  }
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

extern "C" int srk_gemm_rowsum_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha,
                                   const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                                   int64_t ldc, float* rowsum, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(rowsum, SRK_ERR_INVALID, "gemm_rowsum: null rowsum");
  srk::GemmDesc d;
  d.M = M; d.N = N; d.K = K;
  d.A = A; d.lda = lda; d.ta = trans_a != 0;
  d.B = B; d.ldb = ldb; d.tb = trans_b != 0;
  d.C = C; d.ldc = ldc; d.alpha = alpha; d.beta = beta;
  d.rowsum = rowsum;
  return srk::gemm_f32(d, srk::as_stream(stream));
  SRK_API_END
}

extern "C" int srk_colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, float beta, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(M >= 0 && N >= 0 && (N == 0 || (X && out)), SRK_ERR_INVALID, "colsum: bad args");
  return srk::colsum_f32(X, M, N, ldx, out, beta, srk::as_stream(stream));
  SRK_API_END
}
