// K6: 2-D convolution (stride 1, zero padding) as implicit GEMM on the fp32 matrix cores, plus
// window max-pooling — the layers of models/model_fbanks_cnn.py:72-78,89-96 (and the 1-D
// convolutions of model_resnet_bgru.py, which are the KH = 1 case with a stride).
//
// Activations are channels-last (NHWC) inside the model: the GEMM k index (kh, kw, ci) then walks
// contiguous channels, the output tile [pixels x Co] is stored as-is, and the model boundary needs
// no transpose (the fbank input has C = 1; the last conv output is pooled to [B, C]).
//   forward  : Y[p, co]       = sum_(kh,kw,ci) X[n, ho*s+kh-ph, wo*s+kw-pw, ci] Wt[(kh,kw,ci), co]
//   data grad: dX[q, ci]      = sum_(kh,kw,co) dY[n, (h+ph-kh)/s, (w+pw-kw)/s, co] Wd[(kh,kw,co), ci]
//   wgrad    : dWt[(kh,kw,ci), co] = sum_p X[n, ho*s+kh-ph, wo*s+kw-pw, ci] dY[p, co]   (K = N*Ho*Wo)
// The gathers are done by the operand loaders (no im2col buffer).  Weights are re-laid out once
// per call from the torch layout [Co][Ci][KH][KW] (a 1.4 MB copy for the whole fbanks_cnn model).
#include <mutex>

#include "gemm.h"

namespace srk {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

enum { kFwd = 0, kDgrad = 1, kWgrad = 2 };

struct ConvArgs {
  int N, H, W, Ci, Ho, Wo, Co, KH, KW, ph, pw, sh, sw;
  const float* x;      // [N][H][W][Ci]
  const float* dy;     // [N][Ho][Wo][Co]
  const float* wmat;   // fwd: Wt [KH*KW*Ci][Co]; dgrad: Wd [KH*KW*Co][Ci]
  float* out;          // fwd: Y [N*Ho*Wo][Co]; dgrad: dX [N*H*W][Ci]; wgrad: dWt [KH*KW*Ci][Co]
  const float* bias;   // fwd only, [Co]
  int64_t M, Nn, K;    // GEMM dims
  int tiles_n;
  int64_t kchunk;
  float* partial;      // split-K slabs (wgrad)
};

// ---- operand element gathers (return 0 outside the image / problem)
__device__ __forceinline__ float gather_fwd_a(const ConvArgs& c, int64_t m, int64_t k) {
  if (m >= c.M || k >= c.K) return 0.f;
  const int ci = (int)(k % c.Ci);
  const int64_t t = k / c.Ci;
  const int kw = (int)(t % c.KW), kh = (int)(t / c.KW);
  const int wo = (int)(m % c.Wo);
  const int64_t u = m / c.Wo;
  const int ho = (int)(u % c.Ho), n = (int)(u / c.Ho);
  const int hi = ho * c.sh + kh - c.ph, wi = wo * c.sw + kw - c.pw;
  if (hi < 0 || hi >= c.H || wi < 0 || wi >= c.W) return 0.f;
  return c.x[(((int64_t)n * c.H + hi) * c.W + wi) * c.Ci + ci];
}

__device__ __forceinline__ float gather_dgrad_a(const ConvArgs& c, int64_t m, int64_t k) {
  if (m >= c.M || k >= c.K) return 0.f;
  const int co = (int)(k % c.Co);
  const int64_t t = k / c.Co;
  const int kw = (int)(t % c.KW), kh = (int)(t / c.KW);
  const int w = (int)(m % c.W);
  const int64_t u = m / c.W;
  const int h = (int)(u % c.H), n = (int)(u / c.H);
  const int ht = h + c.ph - kh, wt = w + c.pw - kw;
  if (ht < 0 || wt < 0 || ht % c.sh || wt % c.sw) return 0.f;
  const int ho = ht / c.sh, wo = wt / c.sw;
  if (ho >= c.Ho || wo >= c.Wo) return 0.f;
  return c.dy[(((int64_t)n * c.Ho + ho) * c.Wo + wo) * c.Co + co];
}

// wgrad: op(A)[m = (kh,kw,ci)][k = pixel] = X gathered at that pixel's receptive field
__device__ __forceinline__ float gather_wgrad_a(const ConvArgs& c, int64_t m, int64_t k) {
  if (m >= c.M || k >= c.K) return 0.f;
  const int ci = (int)(m % c.Ci);
  const int64_t t = m / c.Ci;
  const int kw = (int)(t % c.KW), kh = (int)(t / c.KW);
  const int wo = (int)(k % c.Wo);
  const int64_t u = k / c.Wo;
  const int ho = (int)(u % c.Ho), n = (int)(u / c.Ho);
  const int hi = ho * c.sh + kh - c.ph, wi = wo * c.sw + kw - c.pw;
  if (hi < 0 || hi >= c.H || wi < 0 || wi >= c.W) return 0.f;
  return c.x[(((int64_t)n * c.H + hi) * c.W + wi) * c.Ci + ci];
}

template <int MODE>
__device__ __forceinline__ v4f load_a4(const ConvArgs& c, int64_t m, int64_t k, bool along_k) {
  // four consecutive elements along k (fwd/dgrad) or along m (wgrad) of op(A)
  v4f v;
  if (MODE == kFwd) {
    if (c.Ci % 4 == 0 && m < c.M && k + 3 < c.K) {   // one contiguous channel run
      const int ci = (int)(k % c.Ci);
      const int64_t t = k / c.Ci;
      const int kw = (int)(t % c.KW), kh = (int)(t / c.KW);
      const int wo = (int)(m % c.Wo);
      const int64_t u = m / c.Wo;
      const int ho = (int)(u % c.Ho), n = (int)(u / c.Ho);
      const int hi = ho * c.sh + kh - c.ph, wi = wo * c.sw + kw - c.pw;
      if (hi < 0 || hi >= c.H || wi < 0 || wi >= c.W) return v4f{0.f, 0.f, 0.f, 0.f};
      return *reinterpret_cast<const v4f*>(c.x + (((int64_t)n * c.H + hi) * c.W + wi) * c.Ci + ci);
    }
    for (int i = 0; i < 4; ++i) v[i] = gather_fwd_a(c, m, k + i);
  } else if (MODE == kDgrad) {
    if (c.Co % 4 == 0 && m < c.M && k + 3 < c.K) {
      const int co = (int)(k % c.Co);
      const int64_t t = k / c.Co;
      const int kw = (int)(t % c.KW), kh = (int)(t / c.KW);
      const int w = (int)(m % c.W);
      const int64_t u = m / c.W;
      const int h = (int)(u % c.H), n = (int)(u / c.H);
      const int ht = h + c.ph - kh, wt = w + c.pw - kw;
      if (ht < 0 || wt < 0 || ht % c.sh || wt % c.sw) return v4f{0.f, 0.f, 0.f, 0.f};
      const int ho = ht / c.sh, wo = wt / c.sw;
      if (ho >= c.Ho || wo >= c.Wo) return v4f{0.f, 0.f, 0.f, 0.f};
      return *reinterpret_cast<const v4f*>(c.dy + (((int64_t)n * c.Ho + ho) * c.Wo + wo) * c.Co + co);
    }
    for (int i = 0; i < 4; ++i) v[i] = gather_dgrad_a(c, m, k + i);
  } else {   // wgrad, vectors along m (channel run of one pixel)
    if (c.Ci % 4 == 0 && k < c.K && m + 3 < c.M) {
      const int ci = (int)(m % c.Ci);
      const int64_t t = m / c.Ci;
      const int kw = (int)(t % c.KW), kh = (int)(t / c.KW);
      const int wo = (int)(k % c.Wo);
      const int64_t u = k / c.Wo;
      const int ho = (int)(u % c.Ho), n = (int)(u / c.Ho);
      const int hi = ho * c.sh + kh - c.ph, wi = wo * c.sw + kw - c.pw;
      if (hi < 0 || hi >= c.H || wi < 0 || wi >= c.W) return v4f{0.f, 0.f, 0.f, 0.f};
      return *reinterpret_cast<const v4f*>(c.x + (((int64_t)n * c.H + hi) * c.W + wi) * c.Ci + ci);
    }
    for (int i = 0; i < 4; ++i) v[i] = gather_wgrad_a(c, m + i, k);
  }
  (void)along_k;
  return v;
}

// B operand: a plain row-major [K][Nn] matrix (fwd: Wt, dgrad: Wd, wgrad: dY as [pixels][Co]).
__device__ __forceinline__ v4f load_b4(const float* B, int64_t ldb, int64_t k, int64_t n0, int64_t K, int64_t N,
                                       bool vec) {
  v4f v = {0.f, 0.f, 0.f, 0.f};
  if (k >= K) return v;
  const float* q = B + k * ldb + n0;
  if (vec && n0 + 3 < N) return *reinterpret_cast<const v4f*>(q);
  for (int i = 0; i < 4; ++i)
    if (n0 + i < N) v[i] = q[i];
  return v;
}

template <int MODE, int BM, int BN, int BK>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs c) {
  constexpr int NT = 256;
  constexpr bool A_ALONG_M = (MODE == kWgrad);
  constexpr int LA = A_ALONG_M ? BM : BM + 1;
  constexpr int LB = BN;
  constexpr int VA = BM * BK / 4 / NT, VB = BN * BK / 4 / NT;
  constexpr int TM = BM / 64, TN = BN / 64;
  __shared__ float As[2][BK][LA];
  __shared__ float Bs[2][BK][LB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tm = blockIdx.x / c.tiles_n, tn = blockIdx.x % c.tiles_n;
  const int split = blockIdx.y;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kb = split * c.kchunk;
  const int64_t ke = (kb + c.kchunk < c.K) ? kb + c.kchunk : c.K;
  const int wm0 = (wave >> 1) * (BM / 2), wn0 = (wave & 1) * (BN / 2);
  const float* Bmat = MODE == kWgrad ? c.dy : c.wmat;
  const bool vec_b = (c.Nn % 4 == 0);
  ConvArgs cc = c;
  cc.K = ke;   // gathers zero-fill past this split's k range

  v4f ra[VA], rb[VB];
  auto load_tile = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < VA; ++i) {
      const int vi = tid + i * NT;
      if (!A_ALONG_M) {
        const int row = vi / (BK / 4), kq = (vi % (BK / 4)) * 4;
        ra[i] = load_a4<MODE>(cc, m0 + row, k0 + kq, true);
      } else {
        const int kr = vi / (BM / 4), mq = (vi % (BM / 4)) * 4;
        ra[i] = load_a4<MODE>(cc, m0 + mq, k0 + kr, false);
      }
    }
#pragma unroll
    for (int i = 0; i < VB; ++i) {
      const int vi = tid + i * NT;
      const int kr = vi / (BN / 4), nq = (vi % (BN / 4)) * 4;
      rb[i] = load_b4(Bmat, c.Nn, k0 + kr, n0 + nq, ke, c.Nn, vec_b);
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < VA; ++i) {
      const int vi = tid + i * NT;
      if (!A_ALONG_M) {
        const int row = vi / (BK / 4), kq = (vi % (BK / 4)) * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) As[buf][kq + q][row] = ra[i][q];
      } else {
        const int kr = vi / (BM / 4), mq = (vi % (BM / 4)) * 4;
        *reinterpret_cast<v4f*>(&As[buf][kr][mq]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < VB; ++i) {
      const int vi = tid + i * NT;
      const int kr = vi / (BN / 4), nq = (vi % (BN / 4)) * 4;
      *reinterpret_cast<v4f*>(&Bs[buf][kr][nq]) = rb[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

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
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t col = n0 + wn0 + j * 32 + lc;
      if (col >= c.Nn) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row >= c.M) continue;
        float v = acc[i][j][r];
        if (c.partial) {
          c.partial[((int64_t)split * c.M + row) * c.Nn + col] = v;
        } else {
          if (MODE == kFwd && c.bias) v += c.bias[col];
          c.out[row * c.Nn + col] = v;
        }
      }
    }
  }
}

__global__ void splitk_sum_kernel(const float* __restrict__ partial, int splits, int64_t n, int64_t ncol,
                                  const float* __restrict__ bias, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int k = 0; k < splits; ++k) s += partial[(int64_t)k * n + i];
  out[i] = bias ? s + bias[i % ncol] : s;
}

// [Co][Ci][KH][KW] -> fwd Wt [(kh,kw,ci)][co]  or  dgrad Wd [(kh,kw,co)][ci]
__global__ void weight_layout_kernel(const float* __restrict__ w, int Co, int Ci, int KH, int KW, int to_dgrad,
                                     float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)Co * Ci * KH * KW;
  if (i >= n) return;
  const int kw = (int)(i % KW);
  int64_t t = i / KW;
  const int kh = (int)(t % KH);
  t /= KH;
  const int ci = (int)(t % Ci), co = (int)(t / Ci);
  if (!to_dgrad) out[(((int64_t)kh * KW + kw) * Ci + ci) * Co + co] = w[i];
  else out[(((int64_t)kh * KW + kw) * Co + co) * Ci + ci] = w[i];
}

// dWt [(kh,kw,ci)][co] -> [Co][Ci][KH][KW]
__global__ void weight_grad_layout_kernel(const float* __restrict__ dwt, int Co, int Ci, int KH, int KW,
                                          float* __restrict__ dw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)Co * Ci * KH * KW;
  if (i >= n) return;
  const int kw = (int)(i % KW);
  int64_t t = i / KW;
  const int kh = (int)(t % KH);
  t /= KH;
  const int ci = (int)(t % Ci), co = (int)(t / Ci);
  dw[i] = dwt[(((int64_t)kh * KW + kw) * Ci + ci) * Co + co];
}

// ------------------------------------------------------------------ max pooling (NHWC)
// window = stride = (kh, kw), floor mode (nn.MaxPool2d((1,3)), MaxPool1d(98) as (98,1)).
// Backward routes each output gradient to the FIRST maximum of its window (PyTorch's rule).
__global__ void maxpool_fwd_kernel(const float* __restrict__ x, int N, int H, int W, int C, int kh, int kw,
                                   float* __restrict__ y) {
  const int Ho = H / kh, Wo = W / kw;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n_out = (int64_t)N * Ho * Wo * C;
  if (i >= n_out) return;
  const int c = (int)(i % C);
  int64_t t = i / C;
  const int wo = (int)(t % Wo);
  t /= Wo;
  const int ho = (int)(t % Ho), n = (int)(t / Ho);
  float m = -INFINITY;
  for (int a = 0; a < kh; ++a)
    for (int b = 0; b < kw; ++b) {
      const float v = x[(((int64_t)n * H + ho * kh + a) * W + wo * kw + b) * C + c];
      if (v > m || v != v) m = v;
    }
  y[i] = m;
}

__global__ void maxpool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, int N, int H, int W,
                                   int C, int kh, int kw, float* __restrict__ dx) {
  const int Ho = H / kh, Wo = W / kw;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n_out = (int64_t)N * Ho * Wo * C;
  if (i >= n_out) return;
  const int c = (int)(i % C);
  int64_t t = i / C;
  const int wo = (int)(t % Wo);
  t /= Wo;
  const int ho = (int)(t % Ho), n = (int)(t / Ho);
  float m = -INFINITY;
  int64_t arg = -1;
  for (int a = 0; a < kh; ++a)
    for (int b = 0; b < kw; ++b) {
      const int64_t idx = (((int64_t)n * H + ho * kh + a) * W + wo * kw + b) * C + c;
      const float v = x[idx];
      if (arg < 0 || v > m || (v != v && m == m)) { m = v; arg = idx; }
      dx[idx] = 0.f;
    }
  dx[arg] = dy[i];
}

__global__ void zero_kernel(float* __restrict__ p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

struct ConvScratch {
  float* p = nullptr;
  size_t floats = 0;
};
ConvScratch g_cs[64];
std::mutex g_cs_mu;

int conv_scratch(size_t floats, float** out) {
  int dev = 0;
  SRK_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_cs_mu);
  ConvScratch& s = g_cs[dev & 63];
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

template <int MODE>
int run_conv_gemm(ConvArgs c, hipStream_t s, const char* name) {
  constexpr int BK = 32;
  const bool big = ((c.M + 127) / 128) * ((c.Nn + 127) / 128) >= 128;
  const int BM = big ? 128 : 64, BN = big ? 128 : 64;
  const int64_t tm = (c.M + BM - 1) / BM, tn = (c.Nn + BN - 1) / BN;
  c.tiles_n = (int)tn;
  int splits = 1;
  if (tm * tn < 256 && c.K >= 16 * BK) {
    splits = (int)std::min<int64_t>((1024 + tm * tn - 1) / (tm * tn), c.K / (8 * BK));
    splits = std::max(1, std::min(splits, 256));
  }
  c.kchunk = splits > 1 ? ((c.K + splits - 1) / splits + BK - 1) / BK * BK : std::max<int64_t>(c.K, 1);
  if (splits > 1) splits = (int)((c.K + c.kchunk - 1) / c.kchunk);
  c.partial = nullptr;
  float* final_out = c.out;
  if (splits > 1) {
    if (int rc = conv_scratch((size_t)splits * c.M * c.Nn, &c.partial)) return rc;
  }
  ProfScope prof(name, s, 2.0 * (double)c.M * (double)c.Nn * (double)c.K);
  const dim3 grid((unsigned)(tm * tn), (unsigned)splits);
  if (big) hipLaunchKernelGGL((conv_gemm_kernel<MODE, 128, 128, BK>), grid, dim3(256), 0, s, c);
  else hipLaunchKernelGGL((conv_gemm_kernel<MODE, 64, 64, BK>), grid, dim3(256), 0, s, c);
  SRK_CHECK_HIP(hipGetLastError());
  if (splits > 1) {
    const int64_t n = c.M * c.Nn;
    hipLaunchKernelGGL(splitk_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c.partial, splits, n,
                       c.Nn, MODE == kFwd ? c.bias : nullptr, final_out);
    SRK_CHECK_HIP(hipGetLastError());
  }
  return SRK_OK;
}

int check(int64_t N, int64_t H, int64_t W, int64_t Ci, int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw,
          int64_t sh, int64_t sw, int64_t* Ho, int64_t* Wo) {
  SRK_REQUIRE(N > 0 && H > 0 && W > 0 && Ci > 0 && Co > 0 && KH > 0 && KW > 0 && ph >= 0 && pw >= 0 && sh > 0 && sw > 0,
              SRK_ERR_INVALID, "conv: bad dims");
  *Ho = (H + 2 * ph - KH) / sh + 1;
  *Wo = (W + 2 * pw - KW) / sw + 1;
  SRK_REQUIRE(*Ho > 0 && *Wo > 0, SRK_ERR_INVALID, "conv: empty output");
  SRK_REQUIRE(N * H * W * Ci < ((int64_t)1 << 40) && N * (*Ho) * (*Wo) * Co < ((int64_t)1 << 40), SRK_ERR_INVALID,
              "conv: too large");
  return SRK_OK;
}

}  // namespace
}  // namespace srk

extern "C" {

int64_t srk_conv2d_workspace_floats(int64_t Ci, int64_t Co, int64_t KH, int64_t KW) { return Ci * Co * KH * KW; }

int srk_conv2d_nhwc_fwd(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                        const float* bias, int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh,
                        int64_t sw, float* y, float* ws, void* stream) {
  SRK_API_BEGIN
  int64_t Ho, Wo;
  if (int rc = srk::check(N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw, &Ho, &Wo)) return rc;
  SRK_REQUIRE(x && w && y && ws, SRK_ERR_INVALID, "conv fwd: null pointer");
  hipStream_t s = srk::as_stream(stream);
  const int64_t nw = Co * Ci * KH * KW;
  hipLaunchKernelGGL(srk::weight_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, w, (int)Co,
                     (int)Ci, (int)KH, (int)KW, 0, ws);
  srk::ConvArgs c{};
  c.N = (int)N; c.H = (int)H; c.W = (int)W; c.Ci = (int)Ci; c.Ho = (int)Ho; c.Wo = (int)Wo; c.Co = (int)Co;
  c.KH = (int)KH; c.KW = (int)KW; c.ph = (int)ph; c.pw = (int)pw; c.sh = (int)sh; c.sw = (int)sw;
  c.x = x; c.wmat = ws; c.out = y; c.bias = bias;
  c.M = N * Ho * Wo; c.Nn = Co; c.K = KH * KW * Ci;
  return srk::run_conv_gemm<srk::kFwd>(c, s, "conv_fwd");
  SRK_API_END
}

int srk_conv2d_nhwc_bwd(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w, int64_t Co,
                        int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw, const float* dy,
                        float* dx, float* dw, float* db, float* ws, void* stream) {
  SRK_API_BEGIN
  int64_t Ho, Wo;
  if (int rc = srk::check(N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw, &Ho, &Wo)) return rc;
  SRK_REQUIRE(x && w && dy && dw && ws, SRK_ERR_INVALID, "conv bwd: null pointer");
  hipStream_t s = srk::as_stream(stream);
  const int64_t nw = Co * Ci * KH * KW;
  srk::ConvArgs c{};
  c.N = (int)N; c.H = (int)H; c.W = (int)W; c.Ci = (int)Ci; c.Ho = (int)Ho; c.Wo = (int)Wo; c.Co = (int)Co;
  c.KH = (int)KH; c.KW = (int)KW; c.ph = (int)ph; c.pw = (int)pw; c.sh = (int)sh; c.sw = (int)sw;
  c.x = x; c.dy = dy;
  int rc;
  if (dx) {
    hipLaunchKernelGGL(srk::weight_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, w, (int)Co,
                       (int)Ci, (int)KH, (int)KW, 1, ws);
    srk::ConvArgs d = c;
    d.wmat = ws; d.out = dx;
    d.M = N * H * W; d.Nn = Ci; d.K = KH * KW * Co;
    if ((rc = srk::run_conv_gemm<srk::kDgrad>(d, s, "conv_dgrad"))) return rc;
  }
  {
    srk::ConvArgs g = c;
    g.out = ws;   // dWt [(kh,kw,ci)][co], then re-laid out into dw
    g.M = KH * KW * Ci; g.Nn = Co; g.K = N * Ho * Wo;
    if ((rc = srk::run_conv_gemm<srk::kWgrad>(g, s, "conv_wgrad"))) return rc;
    hipLaunchKernelGGL(srk::weight_grad_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, ws,
                       (int)Co, (int)Ci, (int)KH, (int)KW, dw);
  }
  if (db && (rc = srk::colsum_f32(dy, N * Ho * Wo, Co, Co, db, 0.f, s))) return rc;
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_maxpool_nhwc_fwd(const float* x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t kh, int64_t kw,
                         float* y, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(x && y && N > 0 && C > 0 && kh > 0 && kw > 0 && H >= kh && W >= kw, SRK_ERR_INVALID, "maxpool: bad args");
  const int64_t n = N * (H / kh) * (W / kw) * C;
  srk::ProfScope prof("maxpool_fwd", srk::as_stream(stream), 4.0 * (N * H * W * C + n));
  hipLaunchKernelGGL(srk::maxpool_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, srk::as_stream(stream), x,
                     (int)N, (int)H, (int)W, (int)C, (int)kh, (int)kw, y);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_maxpool_nhwc_bwd(const float* x, const float* dy, int64_t N, int64_t H, int64_t W, int64_t C, int64_t kh,
                         int64_t kw, float* dx, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(x && dy && dx && N > 0 && C > 0 && kh > 0 && kw > 0 && H >= kh && W >= kw, SRK_ERR_INVALID,
              "maxpool bwd: bad args");
  hipStream_t s = srk::as_stream(stream);
  const int64_t Ho = H / kh, Wo = W / kw;
  const int64_t n = N * Ho * Wo * C;
  if (Ho * kh != H || Wo * kw != W) {   // rows/cols dropped by floor mode get zero gradient
    const int64_t all = N * H * W * C;
    hipLaunchKernelGGL(srk::zero_kernel, dim3((unsigned)((all + 255) / 256)), dim3(256), 0, s, dx, all);
  }
  srk::ProfScope prof("maxpool_bwd", s, 4.0 * (2 * N * H * W * C + n));
  hipLaunchKernelGGL(srk::maxpool_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, dy, (int)N, (int)H,
                     (int)W, (int)C, (int)kh, (int)kw, dx);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
