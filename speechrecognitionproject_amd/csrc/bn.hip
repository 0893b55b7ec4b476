// K9: BatchNorm1d (+ optional residual add + ReLU) on channels-last activations [M rows][C]
// (M = N * L), the normalisation layers of models/model_resnet_bgru.py:20-39,49-50 and its
// downsample branches (:67-70).
//
// Training mode uses the batch statistics (biased variance for the normalisation, unbiased for the
// running estimate, momentum 0.1 as nn.BatchNorm1d), computed in two deterministic passes
// (mean, then centred sum of squares) from per-row-chunk partial sums reduced in a fixed order.
// Eval mode normalises with the running statistics.
//   y = act( (x - mean) * invstd * gamma + beta  [+ residual] ),  act = ReLU or identity
// Backward (training statistics):
//   g = dy * act'(y);  dbeta = sum g;  dgamma = sum g * xhat
//   dx = gamma * invstd / M * (M g - dbeta - xhat * dgamma);  dresidual = g
#include <mutex>

#include "srk_internal.h"

namespace srk {
namespace {

constexpr int kChunkRows = 256;   // rows per partial-sum block

// partial[chunk][c] = sum over the chunk's rows of f(x[r][c]) with f = x (mode 0) or (x - mean)^2
// (mode 1) or dy*act' (mode 2: two outputs, g and g*xhat).
__global__ __launch_bounds__(256) void bn_partial_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                         const float* __restrict__ dy, int64_t M, int C,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd, int relu, int mode,
                                                         float* __restrict__ part0, float* __restrict__ part1) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rp = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.y * kChunkRows;
  const int64_t r1 = r0 + kChunkRows < M ? r0 + kChunkRows : M;
  __shared__ float s0[4][64], s1[4][64];
  float a0 = 0.f, a1 = 0.f;
  if (c < C) {
    const float mu = mode >= 1 ? mean[c] : 0.f;
    const float is = mode == 2 ? invstd[c] : 0.f;
    for (int64_t r = r0 + rp; r < r1; r += 4) {
      const float v = x[r * C + c];
      if (mode == 0) {
        a0 += v;
      } else if (mode == 1) {
        const float d = v - mu;
        a0 += d * d;
      } else {
        float g = dy[r * C + c];
        if (relu && y[r * C + c] <= 0.f) g = 0.f;
        a0 += g;
        a1 += g * (v - mu) * is;
      }
    }
  }
  s0[rp][threadIdx.x & 63] = a0;
  s1[rp][threadIdx.x & 63] = a1;
  __syncthreads();
  if (rp == 0 && c < C) {
    const int l = threadIdx.x & 63;
    part0[(int64_t)blockIdx.y * C + c] = (s0[0][l] + s0[1][l]) + (s0[2][l] + s0[3][l]);
    if (mode == 2) part1[(int64_t)blockIdx.y * C + c] = (s1[0][l] + s1[1][l]) + (s1[2][l] + s1[3][l]);
  }
}

// Sum the chunk partials in order; finalize per-channel statistics.
__global__ void bn_finalize_mean_kernel(const float* __restrict__ part, int chunks, int C, int64_t M,
                                        float* __restrict__ mean) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int k = 0; k < chunks; ++k) s += part[(int64_t)k * C + c];
  mean[c] = s / (float)M;
}

__global__ void bn_finalize_var_kernel(const float* __restrict__ part, int chunks, int C, int64_t M, float eps,
                                       float momentum, const float* __restrict__ mean, float* __restrict__ invstd,
                                       float* __restrict__ running_mean, float* __restrict__ running_var) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int k = 0; k < chunks; ++k) s += part[(int64_t)k * C + c];
  const float var = s / (float)M;
  invstd[c] = 1.0f / sqrtf(var + eps);
  if (running_mean) {
    const float unbiased = M > 1 ? s / (float)(M - 1) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean[c];
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
  }
}

__global__ void bn_apply_kernel(const float* __restrict__ x, int64_t M, int C, const float* __restrict__ mean,
                                const float* __restrict__ invstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const float* __restrict__ residual, int relu,
                                float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int c = (int)(i % C);
  float v = (x[i] - mean[c]) * invstd[c] * gamma[c] + beta[c];
  if (residual) v += residual[i];
  if (relu) v = v > 0.f ? v : 0.f;
  y[i] = v;
}

__global__ void bn_eval_stats_kernel(const float* __restrict__ rm, const float* __restrict__ rv, int C, float eps,
                                     float* __restrict__ mean, float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  invstd[c] = 1.0f / sqrtf(rv[c] + eps);
}

__global__ void bn_dgamma_kernel(const float* __restrict__ p0, const float* __restrict__ p1, int chunks, int C,
                                 float* __restrict__ dbeta, float* __restrict__ dgamma) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  for (int k = 0; k < chunks; ++k) {
    a += p0[(int64_t)k * C + c];
    b += p1[(int64_t)k * C + c];
  }
  dbeta[c] = a;
  dgamma[c] = b;
}

__global__ void bn_dx_kernel(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ dy,
                             int64_t M, int C, const float* __restrict__ mean, const float* __restrict__ invstd,
                             const float* __restrict__ gamma, const float* __restrict__ dbeta,
                             const float* __restrict__ dgamma, int relu, int train, float* __restrict__ dx,
                             float* __restrict__ dres) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * C) return;
  const int c = (int)(i % C);
  float g = dy[i];
  if (relu && y[i] <= 0.f) g = 0.f;
  if (dres) dres[i] = g;
  if (!dx) return;
  const float is = invstd[c];
  if (train) {
    const float xhat = (x[i] - mean[c]) * is;
    dx[i] = gamma[c] * is / (float)M * ((float)M * g - dbeta[c] - xhat * dgamma[c]);
  } else {
    dx[i] = gamma[c] * is * g;
  }
}

struct BnScratch {
  float* p = nullptr;
  size_t floats = 0;
};
BnScratch g_bs[64];
std::mutex g_bs_mu;

int bn_scratch(size_t floats, float** out) {
  int dev = 0;
  SRK_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_bs_mu);
  BnScratch& s = g_bs[dev & 63];
  if (s.floats < floats) {
    if (s.p) {
      SRK_CHECK_HIP(hipDeviceSynchronize());
      SRK_CHECK_HIP(hipFree(s.p));
    }
    s.floats = floats + floats / 4;
    SRK_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&s.p), s.floats * sizeof(float)));
  }
  *out = s.p;
  return SRK_OK;
}

}  // namespace
}  // namespace srk

extern "C" {

int srk_batchnorm_fwd(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta, float eps,
                      float momentum, int training, float* running_mean, float* running_var, const float* residual,
                      int relu, float* y, float* save_mean, float* save_invstd, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(M > 0 && C > 0 && C <= (1 << 24), SRK_ERR_INVALID, "batchnorm: bad shape");
  SRK_REQUIRE(x && gamma && beta && y && save_mean && save_invstd && running_mean && running_var, SRK_ERR_INVALID,
              "batchnorm: null pointer");
  hipStream_t s = srk::as_stream(stream);
  srk::ProfScope prof("batchnorm_fwd", s, (training ? 12.0 : 8.0) * (double)M * C);
  const unsigned cb = (unsigned)((C + 63) / 64);
  const int64_t chunks = (M + srk::kChunkRows - 1) / srk::kChunkRows;
  if (training) {
    float* part = nullptr;
    if (int rc = srk::bn_scratch((size_t)chunks * C, &part)) return rc;
    hipLaunchKernelGGL(srk::bn_partial_kernel, dim3(cb, (unsigned)chunks), dim3(256), 0, s, x, nullptr, nullptr, M,
                       (int)C, nullptr, nullptr, 0, 0, part, nullptr);
    hipLaunchKernelGGL(srk::bn_finalize_mean_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, part,
                       (int)chunks, (int)C, M, save_mean);
    hipLaunchKernelGGL(srk::bn_partial_kernel, dim3(cb, (unsigned)chunks), dim3(256), 0, s, x, nullptr, nullptr, M,
                       (int)C, save_mean, nullptr, 0, 1, part, nullptr);
    hipLaunchKernelGGL(srk::bn_finalize_var_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, part,
                       (int)chunks, (int)C, M, eps, momentum, save_mean, save_invstd, running_mean, running_var);
  } else {
    hipLaunchKernelGGL(srk::bn_eval_stats_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, running_mean,
                       running_var, (int)C, eps, save_mean, save_invstd);
  }
  hipLaunchKernelGGL(srk::bn_apply_kernel, dim3((unsigned)((M * C + 255) / 256)), dim3(256), 0, s, x, M, (int)C,
                     save_mean, save_invstd, gamma, beta, residual, relu, y);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_batchnorm_bwd(const float* x, const float* y, const float* dy, int64_t M, int64_t C, const float* gamma,
                      const float* save_mean, const float* save_invstd, int training, int relu, float* dx,
                      float* dgamma, float* dbeta, float* dresidual, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(M > 0 && C > 0, SRK_ERR_INVALID, "batchnorm_bwd: bad shape");
  SRK_REQUIRE(x && y && dy && gamma && save_mean && save_invstd && dgamma && dbeta, SRK_ERR_INVALID,
              "batchnorm_bwd: null pointer");
  hipStream_t s = srk::as_stream(stream);
  srk::ProfScope prof("batchnorm_bwd", s, 16.0 * (double)M * C);
  const unsigned cb = (unsigned)((C + 63) / 64);
  const int64_t chunks = (M + srk::kChunkRows - 1) / srk::kChunkRows;
  float* part = nullptr;
  if (int rc = srk::bn_scratch((size_t)2 * chunks * C, &part)) return rc;
  hipLaunchKernelGGL(srk::bn_partial_kernel, dim3(cb, (unsigned)chunks), dim3(256), 0, s, x, y, dy, M, (int)C,
                     save_mean, save_invstd, relu, 2, part, part + chunks * C);
  hipLaunchKernelGGL(srk::bn_dgamma_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, part,
                     part + chunks * C, (int)chunks, (int)C, dbeta, dgamma);
  hipLaunchKernelGGL(srk::bn_dx_kernel, dim3((unsigned)((M * C + 255) / 256)), dim3(256), 0, s, x, y, dy, M, (int)C,
                     save_mean, save_invstd, gamma, dbeta, dgamma, relu, training, dx, dresidual);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
