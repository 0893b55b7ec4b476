// Internal GEMM interface (row-major):  C[M,N] = alpha * op(A) * op(B) + beta * C (+ bias)
//   op(A) = A [M,K] (lda)       or A^T with A stored [K,M] when ta
//   op(B) = B [K,N] (ldb)       or B^T with B stored [N,K] when tb
// bias_mode: 0 none, 1 bias[N] added to every row, 2 bias[M] added to every column.
// Batched over `batch` with element strides sA/sB/sC (0 = shared operand).
// Long-K shapes are split over K internally (deterministic slab reduction, grow-only scratch).
#pragma once
#include "srk_internal.h"

namespace srk {

struct GemmDesc {
  int64_t M = 0, N = 0, K = 0;
  const float* A = nullptr; int64_t lda = 0; bool ta = false;
  const float* B = nullptr; int64_t ldb = 0; bool tb = false;
  float* C = nullptr; int64_t ldc = 0;
  float alpha = 1.f, beta = 0.f;
  const float* bias = nullptr; int bias_mode = 0;
  int batch = 1; int64_t sA = 0, sB = 0, sC = 0;
  // optional fused row sums of op(A): rowsum[m] = rowsum_beta * rowsum[m] + sum_k op(A)[m, k]
  float* rowsum = nullptr; float rowsum_beta = 0.f;
  int64_t sRS = 0;   // batched launches: batch z's row sums at rowsum + z sRS
  // matrix-core operand precision (MatmulPrec); -1 = the process setting (srk_set_option)
  int prec = -1;
  // 16-bit operands already in memory (bf16 / fp16 per `prec`, same layouts and leading dimensions
  // in elements): when BOTH are set they replace A / B and no rounding happens on chip (half the
  // operand bytes).  No fused row sums on this path.
  const uint16_t* A16 = nullptr;
  const uint16_t* B16 = nullptr;
};

// Enqueue on `stream`; returns SRK_OK or an srk_status.
int gemm_f32(const GemmDesc& d, hipStream_t stream);

// Whether gemm_f32 accepts `d` with batch > 1 AND fused row sums (the fp32-operand ping-pong
// kernel only); callers fall back to one launch per batch entry otherwise.
bool gemm_f32_batched_rowsum_ok(const GemmDesc& d);

// Column sums: out[n] = beta*out[n] + sum_m X[m, n] (X row-major [M,N], ldx).
int colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, float beta, hipStream_t stream);

}  // namespace srk
