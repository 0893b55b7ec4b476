// K6 fused first layer of the one-channel image CNNs:
//   model_fbanks_cnn (models/model_fbanks_cnn.py:72-73,89-90): Conv2d(1, 64, (7, 3), padding=(3, 1))
//     + bias, then MaxPool2d((1, 3)) over the [N, 98, 120] fbank image;
//   model_spec_cnn (models/model_spec_cnn.py:24-25,44-45): Conv2d(1, 64, (3, 7), padding=(1, 3))
//     + bias, then MaxPool2d((1, 5)) over the [N, 49, 321] spectrogram,
// as ONE pass over the image instead of an implicit GEMM that writes the pre-pool activation
// (1.5 GB for fbanks_cnn at B = 512) and a pooling kernel that reads it back.
//
// Forward  : each output pixel's 21-tap dot product on the VALU (a single input channel gives a
//            K = 21 GEMM that the matrix cores cannot use well), max over the pool window in
//            registers; writes the pooled activation [N][H][W/3][64] and the window argmax (uint8,
//            PyTorch's first-maximum rule, NaN wins) that the backward needs.
// Backward : the pooled gradient routes to exactly one pixel per (window, channel) (the argmax),
//            so dW[co][kh][kw] = sum_q dP[q][co] * x[pixel*(q, co) + tap] and db[co] = sum_q dP[q][co]
//            are accumulated straight from dP — the dense 1.5 GB unpooled gradient is never formed.
//            Per-block partial sums are reduced in a fixed order (deterministic).
// The input needs no gradient (it is the feature tensor, computed under no_grad).
#include "srk_internal.h"

namespace srk {
namespace {

typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int kCo = 64;              // output channels (model_fbanks_cnn.py:72)
constexpr int kC4 = kCo / 4;         // threads per pixel group (4 channels each)
constexpr int kPG = 256 / kC4;       // pixel groups per block
#ifndef SRK_C1_ROWS   // (experiment builds: -DSRK_C1_ROWS=n)
#define SRK_C1_ROWS 8
#endif
constexpr int kRows = SRK_C1_ROWS;   // image rows per block (forward): 2 -> 8 = 340 -> 276 us at cfg3 (r05r), the
                                     // per-block weight loads and the halo amortised over 4x the outputs
constexpr int kRowsW = 8;            // image rows per grid-stride step of the weight gradient: the
                                     // (KH - 1)-row halo and the two barriers amortised over 4x the rows
#ifndef SRK_C1W_PF   // weight gradient: next slab's patch prefetched into registers (1: 295 -> 274 us, r05t) or per slab (0)
#define SRK_C1W_PF 1
#endif
constexpr int kWgradBlocks = 1024;   // persistent blocks of the backward (partials: 5.8 MB)

struct C1Args {
  int N, H, W, ph, pw;
  const float* x;      // [N][H][W]
  const float* w;      // [64][1][KH][KW] (torch layout)
  const float* bias;   // [64]
  float* y;            // fwd: pooled [N][H][W/PW][64]
  uint8_t* arg;        // [N][H][W/PW][64] window argmax
  const float* dy;     // bwd: pooled gradient [N][H][W/PW][64]
  float* partial;      // bwd: [blocks][64 * (KH*KW + 1)]
  unsigned short* y16; // fwd (16-bit matmul modes, optional): the pooled activation's 16-bit operand copy
};

typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2c __attribute__((ext_vector_type(2)));

__device__ __forceinline__ bool takes(float v, float m, bool first) { return first || v > m || (v != v && m == m); }

// x rows [h0 - ph, h0 + kRows - 1 + KH - 1 - ph], cols [-pw, W - 1 + KW - 1 - pw] -> LDS, zero padded
template <int KH, int KW, int ROWS = kRows>
__device__ __forceinline__ void load_patch(const C1Args& a, int n, int h0, float* patch, int pitch) {
  constexpr int PR = ROWS + KH - 1;
  const int PC = a.W + KW - 1;
  for (int i = threadIdx.x; i < PR * PC; i += 256) {
    const int r = i / PC, cidx = i % PC;
    const int h = h0 - a.ph + r, w = cidx - a.pw;
    patch[r * pitch + cidx] = (h >= 0 && h < a.H && w >= 0 && w < a.W) ? a.x[((size_t)n * a.H + h) * a.W + w] : 0.f;
  }
}

// LP: 0 fp32 output only; 1 / 2 also the bf16 / fp16 copy of it (RNE, the conversion srk's to16 makes), which
// conv2's 16-bit implicit GEMMs read instead of converting the 514 MB fp32 activation again
template <int KH, int KW, int PW, int LP>
__global__ __launch_bounds__(256) void conv1_pool_fwd_kernel(C1Args a) {
  constexpr int T = KH * KW;
  extern __shared__ float patch[];
  const int pitch = a.W + KW - 1 + 1;
  const int c4 = threadIdx.x % kC4, pg = threadIdx.x / kC4;
  const int hp = (a.H + kRows - 1) / kRows;
  const int n = blockIdx.x / hp, h0 = (blockIdx.x % hp) * kRows;
  load_patch<KH, KW>(a, n, h0, patch, pitch);
  v4f wr[T];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[t][e] = a.w[(c4 * 4 + e) * T + t];
  v4f bv;
#pragma unroll
  for (int e = 0; e < 4; ++e) bv[e] = a.bias[c4 * 4 + e];
  __syncthreads();
  const int Wq = a.W / PW;
  const int rows = min(kRows, a.H - h0);
  for (int wi = pg; wi < rows * Wq; wi += kPG) {
    const int r = wi / Wq, wq = wi % Wq;
    v4f best = {0.f, 0.f, 0.f, 0.f};
    unsigned idx = 0;
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int col = wq * PW + p;
      v4f acc = bv;
#pragma unroll
      for (int kh = 0; kh < KH; ++kh)
#pragma unroll
        for (int kw = 0; kw < KW; ++kw) {
          const float xv = patch[(r + kh) * pitch + col + kw];
          acc += xv * wr[kh * KW + kw];
        }
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (takes(acc[e], best[e], p == 0)) {
          best[e] = acc[e];
          idx = (idx & ~(0xFFu << (8 * e))) | ((unsigned)p << (8 * e));
        }
    }
    const size_t o = (((size_t)n * a.H + h0 + r) * Wq + wq) * kCo + c4 * 4;
    if (a.y) *reinterpret_cast<v4f*>(a.y + o) = best;   // null: only the 16-bit copy is consumed
    *reinterpret_cast<unsigned*>(a.arg + o) = idx;
    if (LP == 1) *reinterpret_cast<u32x2c*>(a.y16 + o) = __builtin_bit_cast(u32x2c, __builtin_convertvector(best, bf4));
    if (LP == 2) *reinterpret_cast<u32x2c*>(a.y16 + o) = __builtin_bit_cast(u32x2c, __builtin_convertvector(best, h4));
  }
}

// Measured and dropped in round 5 (git history keeps it): the same forward on the fp32 matrix cores
// (bitwise this kernel, but its per-element stores from the accumulator layout cost 406-423 vs 330 us).

template <int KH, int KW, int PW>
__global__ __launch_bounds__(256) void conv1_pool_wgrad_kernel(C1Args a) {
  constexpr int T = KH * KW;
  extern __shared__ float smem[];
  float* patch = smem;
  const int pitch = a.W + KW - 1 + 1;
  const int c4 = threadIdx.x % kC4, pg = threadIdx.x / kC4;
  const int hp = (a.H + kRowsW - 1) / kRowsW;
  const int Wq = a.W / PW;
  v4f acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = v4f{0.f, 0.f, 0.f, 0.f};
  v4f dbacc = {0.f, 0.f, 0.f, 0.f};
  // the next slab's input patch is fetched into registers under this slab's taps (8 per thread: up to 2,048
  // patch values; larger patches take the synchronous load)
  constexpr int PR = kRowsW + KH - 1;
  const int PC = a.W + KW - 1;
  const bool pf = SRK_C1W_PF && PR * PC <= 256 * 8;
  float pr[8];
  auto fetch_patch = [&](int b) {
    const int n = b / hp, h0 = (b % hp) * kRowsW;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = threadIdx.x + j * 256;
      const int r = i / PC, cidx = i % PC;
      const int h = h0 - a.ph + r, w = cidx - a.pw;
      pr[j] = (i < PR * PC && h >= 0 && h < a.H && w >= 0 && w < a.W) ? a.x[((size_t)n * a.H + h) * a.W + w] : 0.f;
    }
  };
  if (pf && (int)blockIdx.x < a.N * hp) fetch_patch(blockIdx.x);
  for (int blk = blockIdx.x; blk < a.N * hp; blk += gridDim.x) {
    const int n = blk / hp, h0 = (blk % hp) * kRowsW;
    __syncthreads();   // previous patch fully consumed
    if (pf) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = threadIdx.x + j * 256;
        if (i < PR * PC) patch[(i / PC) * pitch + i % PC] = pr[j];
      }
    } else {
      load_patch<KH, KW, kRowsW>(a, n, h0, patch, pitch);
    }
    __syncthreads();
    if (pf && blk + (int)gridDim.x < a.N * hp) fetch_patch(blk + gridDim.x);
    const int rows = min(kRowsW, a.H - h0);
    // the dY quads and argmax words of the next two pixels are in flight while this one's taps run (the loop
    // was bound by their load latency at 2 waves per SIMD, not by its LDS reads or FMAs: 336 -> 297 us with one)
    const int npx = rows * Wq;
    auto at = [&](int wi) { return (((size_t)n * a.H + h0 + wi / Wq) * Wq + wi % Wq) * kCo + c4 * 4; };
    v4f gn = {0.f, 0.f, 0.f, 0.f}, gm = gn;   // pixels wi + kPG, wi + 2 kPG
    unsigned in = 0u, im = 0u;
    if (pg < npx) {
      gn = *reinterpret_cast<const v4f*>(a.dy + at(pg));
      in = *reinterpret_cast<const unsigned*>(a.arg + at(pg));
    }
    if (pg + kPG < npx) {
      gm = *reinterpret_cast<const v4f*>(a.dy + at(pg + kPG));
      im = *reinterpret_cast<const unsigned*>(a.arg + at(pg + kPG));
    }
    for (int wi = pg; wi < npx; wi += kPG) {
      const int r = wi / Wq, wq = wi % Wq;
      const v4f g = gn;
      const unsigned idx = in;
      gn = gm;
      in = im;
      if (wi + 2 * kPG < npx) {
        gm = *reinterpret_cast<const v4f*>(a.dy + at(wi + 2 * kPG));
        im = *reinterpret_cast<const unsigned*>(a.arg + at(wi + 2 * kPG));
      }
      dbacc += g;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int col = wq * PW + (int)((idx >> (8 * e)) & 0xFFu);
        const float* pp = patch + r * pitch + col;
#pragma unroll
        for (int kh = 0; kh < KH; ++kh)
#pragma unroll
          for (int kw = 0; kw < KW; ++kw) acc[kh * KW + kw][e] = fmaf(g[e], pp[kh * pitch + kw], acc[kh * KW + kw][e]);
      }
    }
  }
  // Reduce the kPG pixel groups of each channel quad (fixed order): the 4 groups of a wave with
  // xor-shuffles (lanes c4, c4+16, c4+32, c4+48), then the 4 waves through LDS.  One partial row
  // [64 x (T + 1)] per block.
  constexpr int S = (T + 1) * 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t <= T; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = t < T ? acc[t][e] : dbacc[e];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (t < T) acc[t][e] = v; else dbacc[e] = v;
    }
  __syncthreads();   // patch reads done
  float* red = smem;   // [4 waves][kC4][T + 1][4]
  if (lane < kC4) {
#pragma unroll
    for (int t = 0; t < T; ++t) *reinterpret_cast<v4f*>(red + ((wave * kC4 + c4) * (T + 1) + t) * 4) = acc[t];
    *reinterpret_cast<v4f*>(red + ((wave * kC4 + c4) * (T + 1) + T) * 4) = dbacc;
  }
  __syncthreads();
  float* out = a.partial + (size_t)blockIdx.x * kCo * (T + 1);
  for (int i = threadIdx.x; i < kC4 * S; i += 256) {   // i = (c4, t, e)
    const float s = (red[i] + red[kC4 * S + i]) + (red[2 * kC4 * S + i] + red[3 * kC4 * S + i]);
    const int cq = i / S, rem = i % S, t = rem / 4, e = rem % 4;
    out[(cq * 4 + e) * (T + 1) + t] = s;   // [co][t], t == T -> bias
  }
}

// dw[co][t] = sum over blocks; db[co] likewise.  A workgroup owns 64 outputs (lane = output); its 16
// waves each sum a contiguous run of blocks (8 loads in flight per lane), then the 16 wave sums are
// added in wave order through LDS — a fixed order (deterministic), and 16 x shorter chains than one
// thread walking all blocks (which left the reduction load-latency-bound: ~300 us for 1,024 blocks).
constexpr int kRedWaves = 16;
__global__ __launch_bounds__(64 * kRedWaves) void conv1_pool_reduce_kernel(const float* __restrict__ partial,
                                                                           int blocks, int T, float* __restrict__ dw,
                                                                           float* __restrict__ db) {
  __shared__ float red[kRedWaves][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per = kCo * (T + 1);
  const int i = blockIdx.x * 64 + lane;
  const int run = (blocks + kRedWaves - 1) / kRedWaves;
  const int b0 = wave * run, b1 = min(blocks, b0 + run);
  float s = 0.f;
  if (i < per) {
    int b = b0;
    for (; b + 8 <= b1; b += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = partial[(size_t)(b + u) * per + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < b1; ++b) s += partial[(size_t)b * per + i];
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && i < per) {
    float t = red[0][lane];
#pragma unroll
    for (int w = 1; w < kRedWaves; ++w) t += red[w][lane];
    const int co = i / (T + 1), tap = i % (T + 1);
    if (tap < T) dw[co * T + tap] = t;
    else if (db) db[co] = t;
  }
}

int check_c1(int64_t N, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t pool) {
  const bool fb = KH == 7 && KW == 3 && ph == 3 && pw == 1 && pool == 3;
  const bool sc = KH == 3 && KW == 7 && ph == 1 && pw == 3 && pool == 5;
  SRK_REQUIRE(Co == kCo && (fb || sc), SRK_ERR_INVALID,
              "conv1_pool: only the fbanks_cnn (7x3, pad (3,1), pool (1,3)) and spec_cnn (3x7, pad (1,3), pool (1,5)) "
              "conv1 geometries with Co 64 are fused");
  SRK_REQUIRE(N > 0 && H > 0 && W >= pool && N * H * W < ((int64_t)1 << 31), SRK_ERR_INVALID, "conv1_pool: bad dims");
  return SRK_OK;
}

}  // namespace
}  // namespace srk

extern "C" {

int64_t srk_conv1_pool_workspace_floats(int64_t Co, int64_t KH, int64_t KW) {
  return (int64_t)srk::kWgradBlocks * Co * (KH * KW + 1);
}

int srk_conv1_pool_fwd(const float* x, int64_t N, int64_t H, int64_t W, const float* w, const float* bias, int64_t Co,
                       int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t pool, float* y, uint8_t* argmax,
                       void* stream) {
  return srk_conv1_pool_fwd16(x, N, H, W, w, bias, Co, KH, KW, ph, pw, pool, y, argmax, nullptr, nullptr, stream);
}

int srk_conv1_pool_fwd16(const float* x, int64_t N, int64_t H, int64_t W, const float* w, const float* bias,
                         int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t pool, float* y,
                         uint8_t* argmax, void* y16, int* y16_written, void* stream) {
  SRK_API_BEGIN
  // *y16_written == 3 on entry: the caller consumes only the 16-bit copy (fbanks_cnn's fused conv2 + pool in a
  // 16-bit training step), so the fp32 pooled activation is not stored — 5 instead of 7 B per output of the
  // 0.92 GB this launch writes at cfg3; ignored unless the copy is written
  const bool only16 = y16_written && *y16_written == 3;
  if (y16_written) *y16_written = 0;
  if (int rc = srk::check_c1(N, H, W, Co, KH, KW, ph, pw, pool)) return rc;
  SRK_REQUIRE(x && w && bias && y && argmax, SRK_ERR_INVALID, "conv1_pool_fwd: null pointer");
  SRK_REQUIRE((uintptr_t)y % 16 == 0 && (uintptr_t)argmax % 4 == 0 && (uintptr_t)y16 % 8 == 0, SRK_ERR_INVALID,
              "conv1_pool_fwd: misaligned output");
  const int prec = srk::matmul_prec();
  const int lp = y16 && prec != srk::kPrecF32 ? (prec == srk::kPrecBF16 ? 1 : 2) : 0;
  srk::C1Args a{};
  a.N = (int)N; a.H = (int)H; a.W = (int)W; a.ph = (int)ph; a.pw = (int)pw;
  a.x = x; a.w = w; a.bias = bias; a.y = y; a.arg = argmax;
  a.y16 = static_cast<unsigned short*>(y16);
  const bool skip_y = only16 && lp;
  if (skip_y) a.y = nullptr;
  hipStream_t s = srk::as_stream(stream);
  const int hp = (int)((H + srk::kRows - 1) / srk::kRows);
  const size_t lds = (size_t)(srk::kRows + KH - 1) * (W + KW) * 4;
  // algorithmic: the input image once + pooled output + argmax (+ the 16-bit copy)
  srk::ProfScope prof("conv1_pool_fwd", s,
                      4.0 * N * H * W + ((lp ? 7.0 : 5.0) - (skip_y ? 4.0 : 0.0)) * N * H * (W / pool) * Co);
  prof.detail("conv1_pool_fwd_valu<%lldx%lld,pool%lld>", (long long)KH, (long long)KW, (long long)pool);
  const dim3 g((unsigned)(N * hp));
#define SRK_C1F(KH_, KW_, PW_)                                                                                  \
  if (lp == 1) hipLaunchKernelGGL((srk::conv1_pool_fwd_kernel<KH_, KW_, PW_, 1>), g, dim3(256), lds, s, a); \
  else if (lp == 2) hipLaunchKernelGGL((srk::conv1_pool_fwd_kernel<KH_, KW_, PW_, 2>), g, dim3(256), lds, s, a);  \
  else hipLaunchKernelGGL((srk::conv1_pool_fwd_kernel<KH_, KW_, PW_, 0>), g, dim3(256), lds, s, a);
  if (KH == 7) {
    SRK_C1F(7, 3, 3)
  } else {
    SRK_C1F(3, 7, 5)
  }
#undef SRK_C1F
  SRK_CHECK_HIP(hipGetLastError());
  if (lp && y16_written) *y16_written = 1;
  return SRK_OK;
  SRK_API_END
}

int srk_conv1_pool_wgrad(const float* x, int64_t N, int64_t H, int64_t W, int64_t Co, int64_t KH, int64_t KW,
                         int64_t ph, int64_t pw, int64_t pool, const float* dy, const uint8_t* argmax, float* dw,
                         float* db, float* ws, void* stream) {
  SRK_API_BEGIN
  if (int rc = srk::check_c1(N, H, W, Co, KH, KW, ph, pw, pool)) return rc;
  SRK_REQUIRE(x && dy && argmax && dw && ws, SRK_ERR_INVALID, "conv1_pool_wgrad: null pointer");
  srk::C1Args a{};
  a.N = (int)N; a.H = (int)H; a.W = (int)W; a.ph = (int)ph; a.pw = (int)pw;
  a.x = x; a.dy = dy; a.arg = const_cast<uint8_t*>(argmax); a.partial = ws;
  hipStream_t s = srk::as_stream(stream);
  const int T = (int)(KH * KW);
  const int hp = (int)((H + srk::kRowsW - 1) / srk::kRowsW);
  const int blocks = (int)std::min<int64_t>(srk::kWgradBlocks, N * hp);
  const size_t patch = (size_t)(srk::kRowsW + KH - 1) * (W + KW) * 4;
  const size_t red = (size_t)4 * srk::kC4 * (T + 1) * 4 * 4;
  srk::ProfScope prof("conv1_pool_wgrad", s, 4.0 * N * H * W + 5.0 * N * H * (W / pool) * Co);
  if (KH == 7)
    hipLaunchKernelGGL((srk::conv1_pool_wgrad_kernel<7, 3, 3>), dim3((unsigned)blocks), dim3(256), std::max(patch, red),
                       s, a);
  else
    hipLaunchKernelGGL((srk::conv1_pool_wgrad_kernel<3, 7, 5>), dim3((unsigned)blocks), dim3(256), std::max(patch, red),
                       s, a);
  const int per = (int)(Co * (T + 1));
  hipLaunchKernelGGL(srk::conv1_pool_reduce_kernel, dim3((unsigned)((per + 63) / 64)), dim3(64 * srk::kRedWaves), 0, s,
                     ws, blocks, T, dw, db);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
