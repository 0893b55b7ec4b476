// K7/K8: the small training-step kernels around the acoustic models.
//  * cross-entropy (mean over the batch) forward + backward  — nn.CrossEntropyLoss, training.py:73,87
//  * Adam (beta1, beta2, eps; no weight decay, no amsgrad)     — torch.optim.Adam, training.py:74,91
//    over one flat fp32 parameter buffer (one launch for the whole model)
//  * inverted dropout with an explicit mask                     — nn.Dropout(), model_fbanks_cnn.py:79,98
#include <cfloat>
#include <cmath>

#include "srk_internal.h"

namespace srk {
namespace {

// One wave per row; C <= 64 * 4.  loss_rows[b] = logsumexp(x_b) - x_b[label_b];
// dx = (softmax(x_b) - onehot(label_b)) * scale.
__global__ __launch_bounds__(256) void ce_rows_kernel(const float* __restrict__ x, const int64_t* __restrict__ labels,
                                                      int B, int C, float scale, float* __restrict__ loss_rows,
                                                      float* __restrict__ dx, int* __restrict__ bad) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  const float* row = x + (size_t)b * C;
  const int64_t lab = labels[b];
  if (lab < 0 || lab >= C) {   // out-of-range label: the loss becomes NaN (loud), flag set
    if (lane == 0) {
      atomicExch(bad, 1);
      loss_rows[b] = NAN;
    }
    return;
  }
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, row[c]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += expf(row[c] - m);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float lse = m + logf(s);
  if (lane == 0) loss_rows[b] = lse - row[lab];
  if (dx)
    for (int c = lane; c < C; c += 64) dx[(size_t)b * C + c] = (expf(row[c] - lse) - (c == lab ? 1.f : 0.f)) * scale;
}

// Deterministic mean of the per-row losses (one workgroup).
__global__ __launch_bounds__(256) void mean_kernel(const float* __restrict__ v, int n, float* __restrict__ out) {
  __shared__ float part[256];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = part[0] / (float)n;
}

// torch.optim.Adam single-tensor update, in torch's operation order:
//   m = b1*m + (1-b1)*g ; v = b2*v + (1-b2)*g*g
//   denom = sqrt(v) / sqrt(1 - b2^t) + eps ; p -= (lr / (1 - b1^t)) * m / denom
// grad_scale multiplies g first (1/world for a summed all-reduce, or 1).
__device__ __forceinline__ void adam_body(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                          float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                                          float bc1, float bc2_sqrt, float grad_scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      float4 gv = *reinterpret_cast<const float4*>(g + i);
      float4 mv = *reinterpret_cast<float4*>(m + i);
      float4 vv = *reinterpret_cast<float4*>(v + i);
      float4 pv = *reinterpret_cast<float4*>(p + i);
      float* gp = &gv.x; float* mp = &mv.x; float* vp = &vv.x; float* pp = &pv.x;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gg = gp[k] * grad_scale;
        mp[k] = mp[k] * b1 + (1.f - b1) * gg;
        vp[k] = vp[k] * b2 + (1.f - b2) * gg * gg;
        const float denom = sqrtf(vp[k]) / bc2_sqrt + eps;
        pp[k] = pp[k] - (lr / bc1) * (mp[k] / denom);
      }
      *reinterpret_cast<float4*>(m + i) = mv;
      *reinterpret_cast<float4*>(v + i) = vv;
      *reinterpret_cast<float4*>(p + i) = pv;
    } else {
      for (int64_t k = i; k < n; ++k) {
        const float gg = g[k] * grad_scale;
        m[k] = m[k] * b1 + (1.f - b1) * gg;
        v[k] = v[k] * b2 + (1.f - b2) * gg * gg;
        const float denom = sqrtf(v[k]) / bc2_sqrt + eps;
        p[k] = p[k] - (lr / bc1) * (m[k] / denom);
      }
    }
  }
}

__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                            float bc1, float bc2_sqrt, float grad_scale) {
  adam_body(p, g, m, v, n, lr, b1, b2, eps, bc1, bc2_sqrt, grad_scale);
}

// Counter-based Bernoulli mask (splitmix64 of seed ^ index): keep with probability 1 - p.
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);   // 24 random bits -> [0, 1)
}

__global__ void dropout_fwd_kernel(const float* __restrict__ x, int64_t n, float p, float scale, uint64_t seed,
                                   float* __restrict__ y, uint8_t* __restrict__ keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool k = uniform01(seed, (uint64_t)i) >= p;
  keep[i] = k;
  y[i] = k ? x[i] * scale : 0.f;
}

// Loss-scaler state (include/srk.h srk_grad_scaler_init): 8 words on the device.
struct ScalerState {
  float scale, inv_scale, growth, backoff;
  int found_inf, good_steps, interval, overflows;
};

__global__ void scaler_init_kernel(ScalerState* __restrict__ s, float scale, float growth, float backoff,
                                   int interval) {
  s->scale = scale;
  s->inv_scale = 1.0f / scale;
  s->growth = growth;
  s->backoff = backoff;
  s->found_inf = 0;
  s->good_steps = 0;
  s->interval = interval;
  s->overflows = 0;
}

// found_inf |= any non-finite gradient element (16-B loads; one atomic per wave that saw one).
__global__ __launch_bounds__(256) void finite_check_kernel(const float* __restrict__ g, int64_t n,
                                                           ScalerState* __restrict__ s) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  bool bad = false;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 3 < n) {
      const float4 v = *reinterpret_cast<const float4*>(g + i);
      // |x| <= FLT_MAX is false exactly for +-inf and NaN
      bad |= !(fabsf(v.x) <= FLT_MAX) || !(fabsf(v.y) <= FLT_MAX) || !(fabsf(v.z) <= FLT_MAX) ||
             !(fabsf(v.w) <= FLT_MAX);
    } else {
      for (int64_t k = i; k < n; ++k) bad |= !(fabsf(g[k]) <= FLT_MAX);
    }
  }
  if (__ballot(bad) != 0 && (threadIdx.x & 63) == 0) atomicOr(&s->found_inf, 1);
}

// After the (possibly skipped) update: count / back off on an overflow, grow the scale after
// `interval` clean steps (interval 0 = static scale), clear the flag for the next step.
__global__ void scaler_update_kernel(ScalerState* __restrict__ s) {
  if (s->found_inf) {
    s->overflows += 1;
    s->good_steps = 0;
    if (s->interval > 0) {
      s->scale *= s->backoff;
      s->inv_scale = 1.0f / s->scale;
    }
  } else if (s->interval > 0 && ++s->good_steps >= s->interval) {
    s->scale *= s->growth;
    s->inv_scale = 1.0f / s->scale;
    s->good_steps = 0;
  }
  s->found_inf = 0;
}

// Device-resident optimizer step (graph-replayable): one lane advances the step count and stores the
// bias corrections the host path would compute (double precision, rounded to float) beside it.  A
// step the loss scaler skips (non-finite gradients) does not count, as with torch's GradScaler.
__global__ void adam_prep_kernel(int64_t* __restrict__ state, float beta1, float beta2,
                                 const ScalerState* __restrict__ sc) {
  if (sc && sc->found_inf) return;
  const int64_t step = state[0] + 1;
  state[0] = step;
  float* bc = reinterpret_cast<float*>(state + 1);
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  bc[0] = (float)bc1;
  bc[1] = (float)sqrt(bc2);
}

__global__ __launch_bounds__(256) void adam_state_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                         float b1, float b2, float eps,
                                                         const int64_t* __restrict__ state, float grad_scale,
                                                         const ScalerState* __restrict__ sc) {
  if (sc) {
    if (sc->found_inf) return;     // skipped step: parameters and moments stay as they are
    grad_scale *= sc->inv_scale;
  }
  const float* f = reinterpret_cast<const float*>(state + 1);   // bc1, sqrt(bc2), lr
  adam_body(p, g, m, v, n, f[2], b1, b2, eps, f[0], f[1], grad_scale);
}

// Dropout whose seed lives on the device ([base, counter]): the mask of call k hashes base + k, and
// the counter advances behind the mask kernel — so a captured graph draws a fresh mask per replay.
__global__ void dropout_state_kernel(const float* __restrict__ x, int64_t n, float p, float scale,
                                     const uint64_t* __restrict__ state, float* __restrict__ y,
                                     uint8_t* __restrict__ keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t seed = state[0] + 0xD1B54A32D192ED03ull * state[1];
  const bool k = uniform01(seed, (uint64_t)i) >= p;
  keep[i] = k;
  y[i] = k ? x[i] * scale : 0.f;
}

__global__ void counter_inc_kernel(uint64_t* __restrict__ c) { c[0] += 1; }

__global__ void dropout_kernel(const float* __restrict__ x, const uint8_t* __restrict__ keep, int64_t n, float scale,
                               float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = keep[i] ? x[i] * scale : 0.f;
}

}  // namespace
}  // namespace srk

extern "C" {

int srk_cross_entropy(const float* logits, const int64_t* labels, int64_t B, int64_t C, float* loss,
                      float* dlogits, float* ws, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(B > 0 && C > 0 && C <= 4096, SRK_ERR_INVALID, "cross_entropy: bad shape");
  SRK_REQUIRE(logits && labels && loss && ws, SRK_ERR_INVALID, "cross_entropy: null pointer");
  hipStream_t s = srk::as_stream(stream);
  // ws: B floats of per-row loss, then one int error flag
  int* bad = reinterpret_cast<int*>(ws + B);
  SRK_CHECK_HIP(hipMemsetAsync(bad, 0, sizeof(int), s));
  hipLaunchKernelGGL(srk::ce_rows_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, logits, labels, (int)B,
                     (int)C, 1.0f / (float)B, ws, dlogits, bad);
  hipLaunchKernelGGL(srk::mean_kernel, dim3(1), dim3(256), 0, s, ws, (int)B, loss);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float lr,
                  float beta1, float beta2, float eps, int64_t step, float grad_scale, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n >= 0 && step >= 1, SRK_ERR_INVALID, "adam: bad n/step");
  if (n == 0) return SRK_OK;
  SRK_REQUIRE(param && grad && exp_avg && exp_avg_sq, SRK_ERR_INVALID, "adam: null pointer");
  SRK_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
              SRK_ERR_INVALID, "adam: buffers must be 16-byte aligned");
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  const int nt = 256;
  const int64_t blocks = std::min<int64_t>((n + nt * 4 - 1) / (nt * 4), 256 * 8);
  srk::ProfScope prof("adam", srk::as_stream(stream), 28.0 * (double)n);   // p,g,m,v read + p,m,v written
  hipLaunchKernelGGL(srk::adam_kernel, dim3((unsigned)blocks), dim3(nt), 0, srk::as_stream(stream), param, grad,
                     exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, (float)bc1, (float)std::sqrt(bc2), grad_scale);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_adam_step_state(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float beta1,
                        float beta2, float eps, int64_t* state, float grad_scale, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n >= 0 && state, SRK_ERR_INVALID, "adam_state: bad n / null state");
  if (n == 0) return SRK_OK;
  SRK_REQUIRE(param && grad && exp_avg && exp_avg_sq, SRK_ERR_INVALID, "adam_state: null pointer");
  SRK_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0 &&
              (uintptr_t)state % 8 == 0, SRK_ERR_INVALID, "adam_state: buffers must be 16-byte aligned");
  hipStream_t s = srk::as_stream(stream);
  hipLaunchKernelGGL(srk::adam_prep_kernel, dim3(1), dim3(1), 0, s, state, beta1, beta2,
                     (const srk::ScalerState*)nullptr);
  const int nt = 256;
  const int64_t blocks = std::min<int64_t>((n + nt * 4 - 1) / (nt * 4), 256 * 8);
  srk::ProfScope prof("adam", s, 28.0 * (double)n);   // p,g,m,v read + p,m,v written
  hipLaunchKernelGGL(srk::adam_state_kernel, dim3((unsigned)blocks), dim3(nt), 0, s, param, grad, exp_avg, exp_avg_sq,
                     n, beta1, beta2, eps, state, grad_scale, (const srk::ScalerState*)nullptr);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_grad_scaler_init(int32_t* scaler, float init_scale, float growth_factor, float backoff_factor,
                         int growth_interval, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(scaler && (uintptr_t)scaler % 4 == 0, SRK_ERR_INVALID, "grad_scaler_init: null / misaligned state");
  SRK_REQUIRE(init_scale > 0.f && std::isfinite(init_scale) && growth_factor >= 1.f && backoff_factor > 0.f &&
                  backoff_factor <= 1.f && growth_interval >= 0,
              SRK_ERR_INVALID, "grad_scaler_init: bad scale / growth / backoff / interval");
  hipLaunchKernelGGL(srk::scaler_init_kernel, dim3(1), dim3(1), 0, srk::as_stream(stream),
                     reinterpret_cast<srk::ScalerState*>(scaler), init_scale, growth_factor, backoff_factor,
                     growth_interval);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_adam_step_scaled(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, float beta1,
                         float beta2, float eps, int64_t* state, float grad_scale, int32_t* scaler, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n >= 0 && state && scaler, SRK_ERR_INVALID, "adam_scaled: bad n / null state");
  SRK_REQUIRE(n == 0 || (param && grad && exp_avg && exp_avg_sq), SRK_ERR_INVALID, "adam_scaled: null pointer");
  SRK_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0 &&
                  (uintptr_t)state % 8 == 0 && (uintptr_t)scaler % 4 == 0,
              SRK_ERR_INVALID, "adam_scaled: buffers must be 16-byte aligned");
  hipStream_t s = srk::as_stream(stream);
  auto* sc = reinterpret_cast<srk::ScalerState*>(scaler);
  const int nt = 256;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((n + nt * 4 - 1) / (nt * 4), 256 * 8));
  if (n > 0) {
    srk::ProfScope prof("grad_check", s, 4.0 * (double)n);
    hipLaunchKernelGGL(srk::finite_check_kernel, dim3((unsigned)blocks), dim3(nt), 0, s, grad, n, sc);
  }
  hipLaunchKernelGGL(srk::adam_prep_kernel, dim3(1), dim3(1), 0, s, state, beta1, beta2, (const srk::ScalerState*)sc);
  if (n > 0) {
    srk::ProfScope prof("adam", s, 28.0 * (double)n);
    hipLaunchKernelGGL(srk::adam_state_kernel, dim3((unsigned)blocks), dim3(nt), 0, s, param, grad, exp_avg,
                       exp_avg_sq, n, beta1, beta2, eps, state, grad_scale, (const srk::ScalerState*)sc);
  }
  hipLaunchKernelGGL(srk::scaler_update_kernel, dim3(1), dim3(1), 0, s, sc);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_dropout_fwd_state(const float* x, int64_t n, float p, uint64_t* state, float* y, uint8_t* keep,
                          void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n >= 0 && p >= 0.f && p < 1.f && state && (n == 0 || (x && y && keep)), SRK_ERR_INVALID,
              "dropout_fwd_state: bad args");
  if (n == 0) return SRK_OK;
  hipStream_t s = srk::as_stream(stream);
  hipLaunchKernelGGL(srk::dropout_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n, p,
                     1.0f / (1.0f - p), state, y, keep);
  hipLaunchKernelGGL(srk::counter_inc_kernel, dim3(1), dim3(1), 0, s, state + 1);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_dropout_fwd(const float* x, int64_t n, float p, uint64_t seed, float* y, uint8_t* keep, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n >= 0 && p >= 0.f && p < 1.f && (n == 0 || (x && y && keep)), SRK_ERR_INVALID, "dropout_fwd: bad args");
  if (n == 0) return SRK_OK;
  hipLaunchKernelGGL(srk::dropout_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, srk::as_stream(stream), x,
                     n, p, 1.0f / (1.0f - p), seed, y, keep);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_dropout_apply(const float* x, const uint8_t* keep, int64_t n, float scale, float* y, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n >= 0 && (n == 0 || (x && keep && y)), SRK_ERR_INVALID, "dropout: bad args");
  if (n == 0) return SRK_OK;
  hipLaunchKernelGGL(srk::dropout_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, srk::as_stream(stream), x,
                     keep, n, scale, y);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
