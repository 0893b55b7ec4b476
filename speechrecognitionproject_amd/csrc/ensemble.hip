// K11 softmax ensemble of the evaluation callers (predictions.py:56-69, models/model_analyst.py:
// 22-53, analyst_training.py:94-101): per clip, the softmax of each of K models' logits, then
//   * the concatenation [p_1 | ... | p_K] that feeds the stacking "analyst" network, and/or
//   * the mean (p_1 + ... + p_K) / K (summed left to right, as the reference's (o1 + o2) / 2) and
//     its first arg-max (torch.max's tie rule) — the submission label.
// The reference runs this per clip (batch_size = 1) on the host side of the model outputs; here it
// is one launch per batch, one thread per clip (K * C <= 8 * 64 values: tiny, latency-bound).
#include "srk_internal.h"

namespace srk {
namespace {

constexpr int kMaxC = 64;
constexpr int kMaxK = 8;

__global__ void ensemble_kernel(const float* __restrict__ logits, int K, int64_t B, int C, float* __restrict__ cat,
                                float* __restrict__ mean, int64_t* __restrict__ pred) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float acc[kMaxC];
  for (int c = 0; c < C; ++c) acc[c] = 0.f;
  for (int k = 0; k < K; ++k) {
    const float* x = logits + ((int64_t)k * B + b) * C;
    float m = x[0];
    for (int c = 1; c < C; ++c) m = fmaxf(m, x[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += expf(x[c] - m);
    for (int c = 0; c < C; ++c) {
      const float p = expf(x[c] - m) / s;
      if (cat) cat[(b * K + k) * C + c] = p;
      acc[c] += p;
    }
  }
  if (!mean && !pred) return;
  int best = 0;
  float bv = 0.f;
  for (int c = 0; c < C; ++c) {
    const float v = acc[c] / (float)K;
    if (mean) mean[b * C + c] = v;
    if (c == 0 || v > bv) { bv = v; best = c; }
  }
  if (pred) pred[b] = best;
}

}  // namespace
}  // namespace srk

extern "C" int srk_softmax_ensemble(const float* logits, int64_t K, int64_t B, int64_t C, float* probs_cat,
                                    float* mean, int64_t* pred, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(K >= 1 && K <= srk::kMaxK && C >= 1 && C <= srk::kMaxC && B >= 0, SRK_ERR_INVALID,
              "srk_softmax_ensemble: need 1 <= K <= 8 models, 1 <= C <= 64 classes");
  if (B == 0) return SRK_OK;
  SRK_REQUIRE(logits && (probs_cat || mean || pred), SRK_ERR_INVALID, "srk_softmax_ensemble: null pointer");
  hipStream_t s = srk::as_stream(stream);
  hipLaunchKernelGGL(srk::ensemble_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, logits, (int)K, B,
                     (int)C, probs_cat, mean, pred);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}
