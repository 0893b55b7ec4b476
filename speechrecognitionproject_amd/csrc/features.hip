// K1 MFCC, K2 log-mel fbank, K3 log spectrogram, K4 noise-mix — gfx950 HIP kernels.
//
// STFT design: a wave computes several frames at once entirely in registers —
// the N-point real FFT is an N/2-point complex FFT of z[n] = x[2n] + i x[2n+1] factored 16 x M2:
// pass A (lane per (frame, j)) runs an M2-point DFT over its samples in registers and applies the
// twiddles W^(j k1); one LDS transpose (row pitch 17 complex: conflict-free); pass B (lane per
// (frame, k1)) runs a 16-point DFT.  The real spectrum is untangled from Z[k] and Z[N/2 - k], then
// the feature-specific reduction (sparse mel pairs, log, DCT ...) runs on the wave's own LDS
// slice — no workgroup barrier inside the frame loop for fbank / spectrogram (waves take
// (clip, frame-chunk) items independently).  Lane-constant operands (window samples, pass-A
// twiddles, untangle twiddles, mel weights) live in registers for the whole kernel.
// The DC and Nyquist bins come from fp64 sums of the windowed samples (pre-emphasis makes the DC
// bin a cancellation: an fp32 FFT costs up to 0.17 dB in fbank column 1 — SURVEY.md App. A).
#include <algorithm>

#include "fft_regs.h"

namespace srk {
namespace {

using namespace fftr;

constexpr int kPcmLen = 16000;

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Hardware log2 (v_log_f32, ~1 ulp on normal inputs; every caller feeds values >= 1e-10) scaled to
// log10 / ln: the features are compared in dB / log units where this is far inside the tolerances.
__device__ __forceinline__ float fast_log10(float x) { return __builtin_amdgcn_logf(x) * 0.30102999566398120f; }
__device__ __forceinline__ float fast_ln(float x) { return __builtin_amdgcn_logf(x) * 0.69314718055994531f; }

// sum over the 16 lanes of a frame group (lanes 16f .. 16f+15)
__device__ __forceinline__ double group16_sum(double v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------------- K2 fbank
// models/model_fbanks_cnn.py:15-66.  N = 512 (400-sample frames, Hamming, zero-padded), hop 160,
// 98 frames; 256-point complex FFT = 16 (j) x 16 (i), n = j + 16 i, k = k1 + 16 k2.
// A wave = 4 frames (lanes 16 f + j in pass A, 16 f + k1 in pass B): 25 chunks per clip.
constexpr float kFbEpsDb = -313.07119549076395f;   // 20*log10(np.finfo(float).eps), :61-62
constexpr int kFbChunks = 25;
constexpr int kFbPairs = 60, kFbPairTaps = 12;     // filters (l, 119 - l); max pair width 11

struct FbankTables {
  const double* hamming400;
  const float2* tw256;      // W256^t
  const float2* post512;    // W512^k, k = 0..256
  const int4* pair_meta;    // [60] {lo_a, cnt_a, lo_b, cnt_b}
  const float* pair_w;      // [60][12] weights of filter a then filter b, zero padded
};

// 4 waves per SIMD (<= 128 VGPRs): the window and the pass-A twiddles are read from LDS tables
// staged once per workgroup; only the small lane constants stay in registers.
__global__ __launch_bounds__(256, 4) void fbank_kernel(const float* __restrict__ pcm, float* __restrict__ out,
                                                       int64_t n_clips, FbankTables t) {
  __shared__ v2f sbuf[4][4 * 272];   // per wave: 4 frames x (16 x 17) transpose, reused for spectra / power
  __shared__ double s_win[400];
  __shared__ v2f s_tw[16 * 16];      // W256^(j k1) at [k1][j]
  __shared__ v2f s_post[257];        // W512^k
  __shared__ float s_pw[kFbPairs * kFbPairTaps];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int f = lane >> 4, j = lane & 15;
  for (int i = threadIdx.x; i < 400; i += 256) s_win[i] = t.hamming400[i];
  for (int i = threadIdx.x; i < 257; i += 256) s_post[i] = v2f{t.post512[i].x, t.post512[i].y};
  for (int i = threadIdx.x; i < kFbPairs * kFbPairTaps; i += 256) s_pw[i] = t.pair_w[i];
  {
    const int k1 = threadIdx.x >> 4, jj = threadIdx.x & 15;
    const float2 w = t.tw256[(jj * k1) & 255];
    s_tw[threadIdx.x] = v2f{w.x, w.y};
  }
  __syncthreads();
  v2f* tb = sbuf[wave];
  float* pb = reinterpret_cast<float*>(tb);   // power [4][260] after the untangle
  const int pl = lane < kFbPairs ? lane : 0;
  const int4 meta = t.pair_meta[pl];
  const float* pw = s_pw + pl * kFbPairTaps;

  const int64_t items = n_clips * kFbChunks;
  for (int64_t it = (int64_t)blockIdx.x * 4 + wave; it < items; it += (int64_t)gridDim.x * 4) {
    const int64_t clip = it / kFbChunks;
    const int c = (int)(it % kFbChunks);
    const int gf = 4 * c + f;                     // this lane's frame (pass A)
    const bool live = gf < 98;
    const float* __restrict__ x = pcm + clip * kPcmLen + 160 * (live ? gf : 0);
    // pre-emphasis (fp32, numpy's two roundings) x Hamming (fp64, :33-41), DC / Nyquist sums in fp64
    v2f a[16];
    double dc = 0.0, ny = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      a[i] = v2f{0.f, 0.f};
      const int n = j + 16 * i;
      if (i < 13 && n < 200 && live) {
#pragma clang fp contract(off)
        const v2f xv = *reinterpret_cast<const v2f*>(x + 2 * n);
        const bool first = (gf == 0 && n == 0);
        const float xm = first ? 0.f : x[2 * n - 1];
        const float e0 = first ? xv.x : xv.x - 0.97f * xm;
        const float e1 = xv.y - 0.97f * xv.x;
        const double d0 = (double)e0 * s_win[2 * n], d1 = (double)e1 * s_win[2 * n + 1];
        a[i] = v2f{(float)d0, (float)d1};
        dc += d0 + d1;
        ny += d0 - d1;
      }
    }
    dc = group16_sum(dc);
    ny = group16_sum(ny);
    // pass A: 16-point DFT over i, twiddle W256^(j k1), transpose
    dft16v(a);
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) tb[f * 272 + k1 * 17 + j] = k1 ? cm2(a[k1], s_tw[k1 * 16 + j]) : a[0];
    wave_lds_fence();
    // pass B: lane = (f, k1): 16-point DFT over j -> Z[k1 + 16 k2]
    v2f b[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) b[jj] = tb[f * 272 + j * 17 + jj];
    dft16v(b);
    wave_lds_fence();
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) tb[f * 272 + j + 16 * k2] = b[k2];
    wave_lds_fence();
    // untangle -> |X[k]|^2 (k = 0..256) of the 4 frames, held in registers, then written over tb
    float p[4][5];
#pragma unroll
    for (int ff = 0; ff < 4; ++ff) {
      const double dcf = __shfl(dc, 16 * ff, 64), nyf = __shfl(ny, 16 * ff, 64);
#pragma unroll
      for (int m = 0; m < 5; ++m) {
        const int k = lane + 64 * m;
        const v2f A = tb[ff * 272 + (k & 255)];
        const v2f Bz = tb[ff * 272 + ((256 - k) & 255)];
        const v2f Bc = v2f{Bz.x, -Bz.y};
        const v2f e = 0.5f * (A + Bc), o = mi2(0.5f * (A - Bc));
        const v2f X = e + cm2(s_post[min(k, 256)], o);
        float v = X.x * X.x + X.y * X.y;
        if (k == 0) v = (float)(dcf * dcf);
        if (k == 256) v = (float)(nyf * nyf);
        p[ff][m] = v;
      }
    }
    wave_lds_fence();
#pragma unroll
    for (int ff = 0; ff < 4; ++ff)
#pragma unroll
      for (int m = 0; m < 5; ++m)
        if (lane + 64 * m <= 256) pb[ff * 260 + lane + 64 * m] = p[ff][m];
    wave_lds_fence();
    // mel pairs (filter l and 119 - l), |X|^2 / 512 (:44, an exact power of two), eps floor, 20 log10
    if (lane < kFbPairs) {
      float* o = out + (clip * 98 + 4 * c) * 120;
#pragma unroll
      for (int ff = 0; ff < 4; ++ff) {
        if (4 * c + ff >= 98) break;
        const float* pp = pb + ff * 260;
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int q = 0; q < kFbPairTaps; ++q) {
          const bool in_a = q < meta.y;
          const int k = in_a ? meta.x + q : meta.z + (q - meta.y);
          const float v = pw[q] * pp[min(k, 256)];
          sa += in_a ? v : 0.f;
          sb += in_a ? 0.f : v;
        }
        sa *= (1.0f / 512.0f);
        sb *= (1.0f / 512.0f);
        o[ff * 120 + lane] = sa == 0.f ? kFbEpsDb : 20.0f * fast_log10(sa);
        o[ff * 120 + 119 - lane] = sb == 0.f ? kFbEpsDb : 20.0f * fast_log10(sb);
      }
    }
    wave_lds_fence();
  }
}

// ------------------------------------------------------------------------- K3 spectrogram
// models/model_spec_bgru.py:11-17: scipy.signal.spectrogram(fs=16000, nperseg=640, noverlap=320)
// = 49 frames of 640 samples (no padding), periodic Tukey(0.25), PSD density scaling, one-sided
// (interior bins doubled), then log(S + 1e-10).  320-point complex FFT = 16 (j) x 20 (i); a wave
// = 3 frames (17 chunks per clip, the last one holds frame 48 only).
constexpr int kSpChunks = 17;

struct SpecTables {
  const double* tukey640;
  const float2* tw320;
  const float2* post640;
  float scale;              // 1 / (fs * sum(w^2))
};

__global__ __launch_bounds__(256, 4) void spec_kernel(const float* __restrict__ pcm, float* __restrict__ out,
                                                      int64_t n_clips, int transposed, SpecTables t) {
  __shared__ v2f sbuf[4][3 * 340];
  __shared__ double s_win[640];
  __shared__ v2f s_tw[20 * 16];      // W320^(j k1) at [k1][j]
  __shared__ v2f s_post[321];        // W640^k
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fa = lane >> 4, j = lane & 15;       // pass A: frame, j
  const int fb = lane / 20, k1b = lane % 20;     // pass B: frame, k1
  for (int i = threadIdx.x; i < 640; i += 256) s_win[i] = t.tukey640[i];
  for (int i = threadIdx.x; i < 321; i += 256) s_post[i] = v2f{t.post640[i].x, t.post640[i].y};
  for (int i = threadIdx.x; i < 320; i += 256) {
    const float2 w = t.tw320[((i & 15) * (i >> 4)) % 320];
    s_tw[i] = v2f{w.x, w.y};
  }
  __syncthreads();
  v2f* tb = sbuf[wave];
  const int64_t items = n_clips * kSpChunks;
  for (int64_t it = (int64_t)blockIdx.x * 4 + wave; it < items; it += (int64_t)gridDim.x * 4) {
    const int64_t clip = it / kSpChunks;
    const int c = (int)(it % kSpChunks);
    const int gf = 3 * c + fa;
    const bool live = fa < 3 && gf < 49;
    const float* __restrict__ x = pcm + clip * kPcmLen + 320 * (live ? gf : 0);
    v2f a[20];
    double dc = 0.0, ny = 0.0;
#pragma unroll
    for (int i = 0; i < 20; ++i) {
      const v2f xv = *reinterpret_cast<const v2f*>(x + 2 * (j + 16 * i));
      const int n = j + 16 * i;
      const double d0 = live ? (double)xv.x * s_win[2 * n] : 0.0, d1 = live ? (double)xv.y * s_win[2 * n + 1] : 0.0;
      a[i] = v2f{(float)d0, (float)d1};
      dc += d0 + d1;
      ny += d0 - d1;
    }
    dc = group16_sum(dc);
    ny = group16_sum(ny);
    dft20v(a);
    if (fa < 3) {
#pragma unroll
      for (int k1 = 0; k1 < 20; ++k1) tb[fa * 340 + k1 * 17 + j] = k1 ? cm2(a[k1], s_tw[k1 * 16 + j]) : a[0];
    }
    wave_lds_fence();
    v2f b[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) b[jj] = fb < 3 ? tb[fb * 340 + k1b * 17 + jj] : v2f{0.f, 0.f};
    dft16v(b);
    wave_lds_fence();
    if (fb < 3) {
#pragma unroll
      for (int k2 = 0; k2 < 16; ++k2) tb[fb * 320 + k1b + 20 * k2] = b[k2];
    }
    wave_lds_fence();
#pragma unroll
    for (int ff = 0; ff < 3; ++ff) {
      const int f = 3 * c + ff;
      if (f >= 49) break;
      const double dcf = __shfl(dc, 16 * ff, 64), nyf = __shfl(ny, 16 * ff, 64);
      float* o = out + clip * 49 * 321;
#pragma unroll
      for (int m = 0; m < 6; ++m) {
        const int k = lane + 64 * m;
        if (k > 320) continue;
        const v2f A = tb[ff * 320 + (k == 320 ? 0 : k)];
        const v2f Bz = tb[ff * 320 + (k == 0 ? 0 : 320 - k)];
        const v2f Bc = v2f{Bz.x, -Bz.y};
        const v2f e = 0.5f * (A + Bc), oo = mi2(0.5f * (A - Bc));
        const v2f X = e + cm2(s_post[k], oo);
        float v = X.x * X.x + X.y * X.y;
        if (k == 0) v = (float)(dcf * dcf);
        if (k == 320) v = (float)(nyf * nyf);
        v *= t.scale;
        if (k > 0 && k < 320) v *= 2.0f;           // one-sided, DC / Nyquist not doubled
        v = fast_ln(__fadd_rn(v, 1e-10f));         // model_spec_bgru.py:14
        if (transposed) o[f * 321 + k] = v; else o[k * 49 + f] = v;
      }
    }
    wave_lds_fence();
  }
}

// ------------------------------------------------------------------------- K1 MFCC (v2)
// Workgroup = 4 waves, persistent over clips (grid-stride), 2 workgroups per CU: the pass-A
// twiddles and the Hann window are staged in LDS once per workgroup; the 16-tap mel windows
// (filters lane and lane+64, [q][128] so a wave's loads coalesce), the untangle twiddles and the
// DCT rows are read through L1.  Per clip the waves split the 17 chunks of 3 frames; the
// per-clip top_db max is combined across the waves through LDS.
constexpr int kMfWaves = 4;   // 2 workgroups (8 waves) per CU: LDS = 80,096 B each

__device__ __forceinline__ void mfcc_load_chunk(const float* __restrict__ x, int c, int lane, v2f (&raw)[20]) {
  const int fa = lane >> 4, j = lane & 15;
  const int gf = 3 * c + (fa < 3 ? fa : 0);
  if (c > 0 && c < 16) {   // wave-uniform: frames 3..47 never touch the reflected padding
#pragma unroll
    for (int i = 0; i < 20; ++i) raw[i] = *reinterpret_cast<const v2f*>(x + 320 * gf + 2 * (j + 16 * i) - 320);
  } else {
#pragma unroll
    for (int i = 0; i < 20; ++i) {
      int s0 = 320 * gf + 2 * (j + 16 * i) - 320, s1 = s0 + 1;
      s0 = s0 < 0 ? -s0 : (s0 > kPcmLen - 1 ? 2 * (kPcmLen - 1) - s0 : s0);
      s1 = s1 < 0 ? -s1 : (s1 > kPcmLen - 1 ? 2 * (kPcmLen - 1) - s1 : s1);
      raw[i] = v2f{x[s0], x[s1]};
    }
  }
}

// 2 workgroups per CU need <= 256 VGPRs (no AGPR spill-over): waves_per_eu(2) and no prefetch
// of the next chunk (measured: prefetch + 1 wave/SIMD 7.2 ms, prefetch + spills 4.95 ms, no
// prefetch 4.65 ms per 65,536 clips).
__global__ __launch_bounds__(64 * kMfWaves) __attribute__((amdgpu_waves_per_eu(2, 2))) void mfcc2_kernel(const float* __restrict__ pcm, float* __restrict__ out,
                                                              int layout, int64_t n_clips, DeviceTables t) {
  __shared__ v2f tbuf[kMfWaves][3 * 340];
  __shared__ float pbuf[kMfWaves][3 * 321];
  __shared__ __attribute__((aligned(16))) float db[51 * 132];   // row pitch 132: conflict-free b128 reads
  __shared__ v2f s_tw[20 * 16];   // W320^(j k1) at [k1][j]
  __shared__ float s_hann[640];
  __shared__ float red[kMfWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 320; i += 64 * kMfWaves)
    s_tw[i] = *reinterpret_cast<const v2f*>(t.tw320 + ((i >> 4) * (i & 15)));   // [k1][j]
  for (int i = threadIdx.x; i < 640; i += 64 * kMfWaves) s_hann[i] = t.hann640f[i];
  __syncthreads();
  // mel windows / DCT / untangle twiddles stay in global memory (L1/L2-resident, coalesced)
  const int lo0 = t.mel16_lo[lane], lo1 = t.mel16_lo[lane + 64];
  const float* w0 = t.mel16_wt + lane;        // [q][128] layout: w0[q * 128]
  const float* w1 = t.mel16_wt + lane + 64;
  const v2f* __restrict__ s_post = reinterpret_cast<const v2f*>(t.post640);
  const int fa = lane >> 4, j = lane & 15;
  v2f* tb = tbuf[wave];
  float* pb = pbuf[wave];

  for (int64_t clip = blockIdx.x; clip < n_clips; clip += gridDim.x) {
    const float* __restrict__ x = pcm + clip * kPcmLen;
    float vmax = -INFINITY;
    for (int c = wave; c < 17; c += kMfWaves) {
      v2f raw[20];
      mfcc_load_chunk(x, c, lane, raw);
      const int f0 = 3 * c;
      v2f a[20];
#pragma unroll
      for (int i = 0; i < 20; ++i) {
        const v2f w = *reinterpret_cast<const v2f*>(s_hann + 2 * (j + 16 * i));
        a[i] = raw[i] * w;
      }
      // pass A: 20-point DFTs + twiddle, transpose through LDS
      dft20v(a);
      if (fa < 3) {
#pragma unroll
        for (int k1 = 0; k1 < 20; ++k1) tb[fa * 340 + k1 * 17 + j] = k1 ? cm2(a[k1], s_tw[k1 * 16 + j]) : a[0];
      }
      wave_lds_fence();
      // pass B: 16-point DFTs -> natural-order spectra (overwrite the transpose slice)
      const int fb = lane / 20, k1 = lane % 20;
      v2f b[16];
      if (fb < 3) {
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) b[jj] = tb[fb * 340 + k1 * 17 + jj];
      }
      dft16v(b);
      wave_lds_fence();
      if (fb < 3) {
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) tb[fb * 320 + k1 + 20 * k2] = b[k2];
      }
      wave_lds_fence();
      // untangle the packed real FFT -> |X[k]|^2, k = 0..320
#pragma unroll
      for (int f = 0; f < 3; ++f) {
#pragma unroll
        for (int m = 0; m < 6; ++m) {
          const int k = lane + 64 * m;
          if (k <= 320) {
            const v2f A = tb[f * 320 + (k == 320 ? 0 : k)];
            const v2f Bz = tb[f * 320 + (k == 0 ? 0 : 320 - k)];
            const v2f Bc = v2f{Bz.x, -Bz.y};
            const v2f e = 0.5f * (A + Bc), o = mi2(0.5f * (A - Bc));
            const v2f X = e + cm2(s_post[k], o);
            pb[f * 321 + k] = X.x * X.x + X.y * X.y;
          }
        }
      }
      wave_lds_fence();
      // Slaney mel (two 16-tap filters per lane) -> power_to_db(ref=1, amin=1e-10)
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        const float* p = pb + f * 321;
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          s0 = fmaf(w0[q * 128], p[lo0 + q], s0);
          s1 = fmaf(w1[q * 128], p[lo1 + q], s1);
        }
        const float v0 = s0 > 1e-10f ? 10.0f * fast_log10(s0) : -100.0f;
        const float v1 = s1 > 1e-10f ? 10.0f * fast_log10(s1) : -100.0f;
        db[(f0 + f) * 132 + lane] = v0;
        db[(f0 + f) * 132 + lane + 64] = v1;
        vmax = fmaxf(vmax, fmaxf(v0, v1));
      }
      wave_lds_fence();
    }
    vmax = wave_max(vmax);
    if (lane == 0) red[wave] = vmax;
    __syncthreads();
    float mx = red[0];
#pragma unroll
    for (int w = 1; w < kMfWaves; ++w) mx = fmaxf(mx, red[w]);
    const float floor_db = mx - 80.0f;
    float* C = reinterpret_cast<float*>(&tbuf[0][0]);   // 13 x 51 coefficients
    float* D = C + 13 * 51;                             // deltas
    for (int it = threadIdx.x; it < 13 * 51; it += 64 * kMfWaves) {
      const int cc = it / 51, f = it % 51;
      const float* d = db + f * 132;
      const float* w = t.dct + cc * 128;
      v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
      for (int k = 0; k < 128; k += 4) {
        const v4f dv = *reinterpret_cast<const v4f*>(d + k);
        const v4f wv = *reinterpret_cast<const v4f*>(w + k);
        acc.x = fmaf(wv.x, fmaxf(dv.x, floor_db), acc.x);
        acc.y = fmaf(wv.y, fmaxf(dv.y, floor_db), acc.y);
        acc.z = fmaf(wv.z, fmaxf(dv.z, floor_db), acc.z);
        acc.w = fmaf(wv.w, fmaxf(dv.w, floor_db), acc.w);
      }
      C[it] = (acc.x + acc.y) + (acc.z + acc.w);
    }
    __syncthreads();
    auto grad = [](const float* r, int f) {
      return f == 0 ? r[1] - r[0] : (f == 50 ? r[50] - r[49] : (r[f + 1] - r[f - 1]) * 0.5f);
    };
    for (int it = threadIdx.x; it < 13 * 51; it += 64 * kMfWaves) D[it] = grad(C + (it / 51) * 51, it % 51);
    __syncthreads();
    float* o = out + clip * 39 * 51;
    for (int it = threadIdx.x; it < 39 * 51; it += 64 * kMfWaves) {
      const int row = it / 51, f = it % 51;
      float v;
      if (row < 13) v = C[row * 51 + f];
      else if (row < 26) v = D[(row - 13) * 51 + f];
      else v = grad(D + (row - 26) * 51, f);
      if (layout == 0) o[row * 51 + f] = v; else o[f * 39 + row] = v;
    }
    __syncthreads();   // tbuf / db are reused by the next clip
  }
}

// ------------------------------------------------------------------------- K4 noise mix
// numpy: sample + (gain * noise) in float64 (two roundings, never fused), then np.int16()
// truncates toward zero.
__device__ __forceinline__ float mix_one(short s, double g, short n) {
#pragma clang fp contract(off)
  const double v = (double)s + g * (double)n;
  return (float)(int16_t)(int)v;
}

__global__ void noise_mix_kernel(const int16_t* __restrict__ pcm, const int16_t* __restrict__ bank,
                                 int64_t bank_len, const int64_t* __restrict__ file_idx,
                                 const int64_t* __restrict__ offs, const double* __restrict__ gains,
                                 int64_t n_clips, float* __restrict__ out) {
  // 8 samples per thread: 16-B int16 loads of pcm, 16-B + 16-B fp32 stores.
  const int64_t i8 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total8 = n_clips * (kPcmLen / 8);
  if (i8 >= total8) return;
  const int64_t clip = i8 / (kPcmLen / 8);
  const int s0 = (int)(i8 % (kPcmLen / 8)) * 8;
  const int16_t* nz = bank + file_idx[clip] * bank_len + offs[clip] + s0;
  const double g = gains[clip];
  const short4 a = *reinterpret_cast<const short4*>(pcm + clip * kPcmLen + s0);
  const short4 b = *reinterpret_cast<const short4*>(pcm + clip * kPcmLen + s0 + 4);
  const short sv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = mix_one(sv[j], g, nz[j]);
  float4* o = reinterpret_cast<float4*>(out + clip * kPcmLen + s0);
  o[0] = make_float4(r[0], r[1], r[2], r[3]);
  o[1] = make_float4(r[4], r[5], r[6], r[7]);
}

}  // namespace
}  // namespace srk

using srk::DeviceTables;

extern "C" {

int srk_fbank_fwd(const float* pcm, int64_t n_clips, float* out, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n_clips >= 0 && n_clips <= INT32_MAX, SRK_ERR_INVALID, "srk_fbank_fwd: bad n_clips %lld", (long long)n_clips);
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(pcm && out, SRK_ERR_INVALID, "srk_fbank_fwd: null pointer");
  SRK_REQUIRE((uintptr_t)pcm % 8 == 0, SRK_ERR_INVALID, "srk_fbank_fwd: pcm must be 8-byte aligned");
  const DeviceTables* t = nullptr;
  if (int rc = srk::get_tables(&t)) return rc;
  srk::FbankTables ft{t->hamming400, t->tw256, t->post512, t->fbp_meta, t->fbp_w};
  const int64_t items = n_clips * srk::kFbChunks;
  const int64_t blocks = std::min<int64_t>((items + 3) / 4, 2048);   // waves take (clip, 4-frame chunk) items
  srk::ProfScope prof("fbank", srk::as_stream(stream), 111040.0 * (double)n_clips);   // 64000 in + 47040 out B/clip
  hipLaunchKernelGGL(srk::fbank_kernel, dim3((unsigned)blocks), dim3(256), 0, srk::as_stream(stream), pcm, out, n_clips,
                     ft);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_spec_fwd(const float* pcm, int64_t n_clips, float* out, int transposed, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n_clips >= 0 && n_clips <= INT32_MAX, SRK_ERR_INVALID, "srk_spec_fwd: bad n_clips");
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(pcm && out, SRK_ERR_INVALID, "srk_spec_fwd: null pointer");
  SRK_REQUIRE((uintptr_t)pcm % 8 == 0, SRK_ERR_INVALID, "srk_spec_fwd: pcm must be 8-byte aligned");
  const DeviceTables* t = nullptr;
  if (int rc = srk::get_tables(&t)) return rc;
  srk::SpecTables st{t->tukey640, t->tw320, t->post640, (float)t->spec_scale};
  const int64_t items = n_clips * srk::kSpChunks;
  const int64_t blocks = std::min<int64_t>((items + 3) / 4, 2048);
  srk::ProfScope prof("spec", srk::as_stream(stream), 126916.0 * (double)n_clips);    // 64000 + 62916 B/clip
  hipLaunchKernelGGL(srk::spec_kernel, dim3((unsigned)blocks), dim3(256), 0, srk::as_stream(stream), pcm, out, n_clips,
                     transposed ? 1 : 0, st);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_mfcc_fwd(const float* pcm, int64_t n_clips, float* out, int layout, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n_clips >= 0 && n_clips <= INT32_MAX, SRK_ERR_INVALID, "srk_mfcc_fwd: bad n_clips");
  SRK_REQUIRE(layout == 0 || layout == 1, SRK_ERR_INVALID, "srk_mfcc_fwd: layout must be 0 or 1");
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(pcm && out, SRK_ERR_INVALID, "srk_mfcc_fwd: null pointer");
  const DeviceTables* t = nullptr;
  if (int rc = srk::get_tables(&t)) return rc;
  srk::ProfScope prof("mfcc", srk::as_stream(stream), 71956.0 * (double)n_clips);     // 64000 + 7956 B/clip
  const int64_t grid = std::min<int64_t>(n_clips, 256 * 4);   // persistent over clips
  hipLaunchKernelGGL(srk::mfcc2_kernel, dim3((unsigned)grid), dim3(64 * srk::kMfWaves), 0,
                     srk::as_stream(stream), pcm, out, layout, n_clips, *t);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_noise_mix(const int16_t* pcm, const int16_t* bank, int64_t n_files, int64_t bank_len,
                  const int64_t* file_idx, const int64_t* offset, const double* gain, int64_t n_clips,
                  float* out, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n_clips >= 0, SRK_ERR_INVALID, "srk_noise_mix: bad n_clips");
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(pcm && bank && file_idx && offset && gain && out, SRK_ERR_INVALID, "srk_noise_mix: null pointer");
  SRK_REQUIRE(n_files > 0 && bank_len >= 16000, SRK_ERR_INVALID, "srk_noise_mix: bank must hold >= 1 file of >= 16000 samples");
  SRK_REQUIRE(((uintptr_t)pcm % 16) == 0 && ((uintptr_t)out % 16) == 0, SRK_ERR_INVALID,
              "srk_noise_mix: pcm/out must be 16-byte aligned");
  const int64_t total8 = n_clips * (16000 / 8);
  const int nt = 256;
  const int64_t blocks = (total8 + nt - 1) / nt;
  srk::ProfScope prof("noise_mix", srk::as_stream(stream), 128000.0 * (double)n_clips); // 32000+32000+64000 B/clip
  hipLaunchKernelGGL(srk::noise_mix_kernel, dim3((unsigned)blocks), dim3(nt), 0, srk::as_stream(stream), pcm, bank,
                     bank_len, file_idx, offset, gain, n_clips, out);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
