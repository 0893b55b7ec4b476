// K10 batched training-mode augmentation (dataset.py:103-118 with the helpers :148-223):
// speed tuning (cv2 INTER_LINEAR resample + random pad / centre cut), time shift, uniform noise,
// SNR noise and silence synthesis, one op per clip, for a whole batch in one launch.
//
// One workgroup per clip.  The clip's int16 PCM (32 KB) is staged in LDS so the resampler's
// gathers never touch HBM twice; every output sample is produced by exactly one thread as
// 8-sample groups (2 x 16-B float4 stores).  Memory-bound by construction: 32 KB read (+ 32 KB of
// noise for the noise ops) and 64 KB written per clip.
//
// Arithmetic follows the numpy/OpenCV reference bit for bit (oracle/augment.py): float64 with
// contraction off, truncation toward zero on the int16 casts, and for the resampler OpenCV's
// fp32 coordinate / coefficient path.  The one reduction (SNR powers) is a fixed-order fp64 tree.
#include "srk_internal.h"

namespace srk {
namespace {

constexpr int kLen = 16000;
constexpr int kThreads = 256;

__device__ __forceinline__ float i16f(double v) { return (float)(int16_t)(int)v; }

// oracle/augment.py aug_fill: splitmix64 of (seed, clip, position) -> [-32, 32)
__device__ __forceinline__ float aug_fill(uint64_t seed, int64_t clip, int i) {
  uint64_t x = seed + (uint64_t)clip * 0x9E3779B97F4A7C15ull + (uint64_t)(i + 1) * 0xD1B54A32D192ED03ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (float)((int)(x >> 58) - 32);
}

// cv2.resize(x, (1, n_out), INTER_LINEAR) sample dy of a float64 column (resizeGeneric_ with
// VResizeLinear<double, double, float>): fp32 fy / coefficients, rows clamped, weight not clamped.
__device__ __forceinline__ double resample(const int16_t* s, double scale, int dy) {
#pragma clang fp contract(off)
  float fy = (float)(((double)dy + 0.5) * scale - 0.5);
  const int sy = (int)floorf(fy);
  fy -= (float)sy;
  const float b0 = 1.f - fy, b1 = fy;
  const int r0 = min(max(sy, 0), kLen - 1), r1 = min(max(sy + 1, 0), kLen - 1);
  const double t0 = (double)s[r0] * (double)b0;
  const double t1 = (double)s[r1] * (double)b1;
  return t0 + t1;
}

__device__ double block_sum(double v, double* red) {
  // fixed order: wave-level xor tree, then the 4 wave sums in wave order
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(kThreads) void augment_kernel(const int16_t* __restrict__ pcm,
                                                           const int16_t* __restrict__ bank, int64_t bank_len,
                                                           const int32_t* __restrict__ op,
                                                           const int64_t* __restrict__ iparam,
                                                           const int64_t* __restrict__ noise_pos,
                                                           const double* __restrict__ dparam, uint64_t seed,
                                                           float* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ int16_t s[kLen];
  __shared__ double red[4];
  const int64_t clip = blockIdx.x;
  const int o = op[clip];
  const int64_t ip = iparam[clip];
  const double dp = dparam[clip];
  int64_t pos = noise_pos[clip];
  const bool has_noise = pos >= 0 && pos <= bank_len - kLen;   // the host validates; never read out of range
  if (!has_noise) pos = 0;
  const int16_t* nz = bank + pos;
  const int16_t* src = pcm + clip * kLen;
  // stage the clip: 16-B loads (pcm rows are 32000 B, 16-B aligned by the API contract)
  for (int i = threadIdx.x; i < kLen / 8; i += kThreads)
    reinterpret_cast<int4*>(s)[i] = reinterpret_cast<const int4*>(src)[i];
  double factor = 0.0;
  if (o == 4) {   // add_noise_snr: powers of the sample and the noise window (dataset.py:176-178)
    double ps = 0.0, pn = 0.0;
    for (int i = threadIdx.x; i < kLen; i += kThreads) {
      const double a = (double)src[i] / 32768.0, b = has_noise ? (double)nz[i] / 32768.0 : 0.0;
      ps += a * a;
      pn += b * b;
    }
    const double sp = block_sum(ps, red) / (double)kLen;
    const double np_ = block_sum(pn, red) / (double)kLen;
    factor = sqrt((sp / np_) / dp);
  }
  __syncthreads();
  float* dst = out + clip * kLen;
  // speed tuning geometry (dataset.py:212-223)
  const int n_out = (int)ip;
  const double scale = 1.0 / ((double)n_out / (double)kLen);
  const int left = n_out < kLen ? (kLen - n_out) / 2 : 0;
  const int cut = n_out >= kLen ? (n_out - kLen) / 2 : 0;
  for (int g = threadIdx.x; g < kLen / 8; g += kThreads) {
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = g * 8 + j;
      float v;
      if (o == 1) {                       // speed_tuning
        if (n_out < kLen) {
          const int k = i - left;
          v = (k >= 0 && k < n_out) ? i16f(resample(s, scale, k)) : aug_fill(seed, clip, i);
        } else {
          v = i16f(resample(s, scale, i + cut));
        }
      } else if (o == 2) {                // time_stretching (:195-204)
        const int k = i + (int)ip;
        v = (k >= 0 && k < kLen) ? (float)s[k] : aug_fill(seed, clip, i);
      } else if (o == 3) {                // add_noise_uniform (:183-193)
        v = i16f((double)s[i] + dp * (double)(has_noise ? nz[i] : 0));
      } else if (o == 4) {                // add_noise_snr (:179-181)
        v = i16f((double)s[i] + factor * (double)(has_noise ? nz[i] : 0));
      } else if (o == 5) {                // generate_silence_sample (:150-160)
        v = has_noise ? (float)((double)nz[i] * dp) : 0.f;
      } else {
        v = (float)s[i];
      }
      r[j] = v;
    }
    float4* q = reinterpret_cast<float4*>(dst + g * 8);
    q[0] = make_float4(r[0], r[1], r[2], r[3]);
    q[1] = make_float4(r[4], r[5], r[6], r[7]);
  }
}

}  // namespace
}  // namespace srk

extern "C" int srk_augment(const int16_t* pcm, int64_t n_clips, const int16_t* bank, int64_t bank_len,
                           const int32_t* op, const int64_t* iparam, const int64_t* noise_pos, const double* dparam,
                           uint64_t seed, float* out, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n_clips >= 0 && n_clips < ((int64_t)1 << 31), SRK_ERR_INVALID, "srk_augment: bad n_clips");
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(pcm && op && iparam && noise_pos && dparam && out, SRK_ERR_INVALID, "srk_augment: null pointer");
  SRK_REQUIRE(bank_len == 0 || bank, SRK_ERR_INVALID, "srk_augment: null bank");
  SRK_REQUIRE((uintptr_t)pcm % 16 == 0 && (uintptr_t)out % 16 == 0, SRK_ERR_INVALID,
              "srk_augment: pcm/out must be 16-byte aligned");
  hipStream_t s = srk::as_stream(stream);
  srk::ProfScope prof("augment", s, 96000.0 * (double)n_clips);   // 32000 in + 64000 out per clip
  hipLaunchKernelGGL(srk::augment_kernel, dim3((unsigned)n_clips), dim3(srk::kThreads), 0, s, pcm, bank, bank_len, op,
                     iparam, noise_pos, dparam, seed, out);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}
