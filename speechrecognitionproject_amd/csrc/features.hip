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

__device__ __forceinline__ float bperm(int src_byte, float v) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src_byte, __float_as_int(v)));
}

// PCM sample loads: float32 (what Dataset yields) or int16 (what the WAV holds — half the upload;
// the reference's float32 samples are int16-valued, dataset.py:117, so the widened values are equal)
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const int16_t* p) { return (float)*p; }
__device__ __forceinline__ v2f ld2(const float* p) { return *reinterpret_cast<const v2f*>(p); }
__device__ __forceinline__ v2f ld2(const int16_t* p) {
  const short2 v = *reinterpret_cast<const short2*>(p);
  return v2f{(float)v.x, (float)v.y};
}

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
template <typename T>
__global__ __launch_bounds__(256, 4) void fbank_kernel(const T* __restrict__ pcm, float* __restrict__ out,
                                                       int64_t n_clips, FbankTables t) {
  __shared__ v2f sbuf[4][4 * 272];   // per wave: 4 frames x (16 x 17) transpose, reused for spectra / power
  __shared__ __attribute__((aligned(16))) double s_win[400];
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
  float* pb = reinterpret_cast<float*>(tb);   // power [4][272] after the untangle (pitch = 16 mod 32:
                                              // two frames' 16-lane stores fill the 32 banks)
  const int pl = lane < kFbPairs ? lane : 0;
  const int4 meta = t.pair_meta[pl];
  const float* pw = s_pw + pl * kFbPairTaps;

  const int64_t items = n_clips * kFbChunks;
  for (int64_t it = (int64_t)blockIdx.x * 4 + wave; it < items; it += (int64_t)gridDim.x * 4) {
    const int64_t clip = it / kFbChunks;
    const int c = (int)(it % kFbChunks);
    const int gf = 4 * c + f;                     // this lane's frame (pass A)
    const bool live = gf < 98;
    const T* __restrict__ x = pcm + clip * kPcmLen + 160 * (live ? gf : 0);
    // pre-emphasis (fp32, numpy's two roundings) x Hamming (fp64, :33-41), DC / Nyquist sums in fp64
    // every lane loads (dead lanes read in-clip samples) and the products are masked after: with the
    // loads under the condition the compiler serialises their waits
    v2f xv[13];
    float xm[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) {
      const int n = j + 16 * i;
      xv[i] = ld2(x + 2 * n);
      xm[i] = ld1(x + ((n == 0 && !(live && gf > 0)) ? 0 : 2 * n - 1));   // x[-1] only inside the clip
    }
    v2f a[16];
    double dc = 0.0, ny = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      a[i] = v2f{0.f, 0.f};
      const int n = j + 16 * i;
      if (i < 13) {
#pragma clang fp contract(off)
        const bool first = (gf == 0 && n == 0);
        const float e0 = first ? xv[i].x : xv[i].x - 0.97f * xm[i];
        const float e1 = xv[i].y - 0.97f * xv[i].x;
        const double2 w = *reinterpret_cast<const double2*>(s_win + 2 * (n < 200 ? n : 199));
        double d0 = (double)e0 * w.x, d1 = (double)e1 * w.y;
        const bool valid = live && n < 200;
        d0 = valid ? d0 : 0.0;
        d1 = valid ? d1 : 0.0;
        a[i] = v2f{(float)d0, (float)d1};
        dc += d0 + d1;
        ny += d0 - d1;
      }
    }
    dc = group16_sum(dc);
    ny = group16_sum(ny);
    // pass A: 16-point DFT over i, twiddle W256^(j k1), transpose
    dft16v(a);
    tb[f * 272 + j] = a[0];
#pragma unroll
    for (int g = 1; g < 16; g += 5) {   // twiddles read 5 at a time ahead of their stores (3 LDS round trips)
      v2f tw[5];
#pragma unroll
      for (int u = 0; u < 5; ++u) tw[u] = s_tw[(g + u) * 16 + j];
#pragma unroll
      for (int u = 0; u < 5; ++u) tb[f * 272 + (g + u) * 17 + j] = pcmul(a[g + u], tw[u]);
    }
    wave_lds_fence();
    // pass B: lane = (f, k1): 16-point DFT over j -> Z[k1 + 16 k2]
    v2f b[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) b[jj] = tb[f * 272 + j * 17 + jj];
    dft16v(b);
    wave_lds_fence();
    // untangle (as K1): with A = Z[k], B = Z[256 - k], W = W512^k, S = (A.x + B.x, A.y - B.y),
    // U = (A.y + B.y, B.x - A.x): 2 X[k] = S + W U and 2 X[256 - k] = (S - W U)*.  Lane (f, k1) pairs
    // its k2 < 8 with lane (f, 16 - k1) at 15 - k2 (ds_bpermute); k1 = 0 and 8 pair inside the lane,
    // k1 = 0 also takes the self-paired bin 128 and writes the fp64 DC / Nyquist powers for k = 0 / 256.
    {
      const int pbyte = 4 * (16 * f + ((16 - j) & 15));
      float Bx[8], By[8];
      v2f wpost[8];
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) wpost[k2] = s_post[j + 16 * k2];
      const v2f w128 = s_post[128];
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) {
        Bx[k2] = bperm(pbyte, b[15 - k2].x);
        By[k2] = bperm(pbyte, b[15 - k2].y);
      }
      __builtin_amdgcn_sched_barrier(0);
      float* pf = pb + f * 272;
      auto two_bins = [&](v2f A, v2f B, v2f w, int k) {
        const v2f p = 0.25f * untangle_pk(A, B, w);
        pf[256 - k] = p.y;   // first: bin 128 pairs with itself
        pf[k] = p.x;
      };
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) {
        const float bx = j == 0 ? b[(16 - k2) & 15].x : Bx[k2];
        const float by = j == 0 ? b[(16 - k2) & 15].y : By[k2];
        two_bins(b[k2], v2f{bx, by}, wpost[k2], j + 16 * k2);
      }
      if (j == 0) {
        two_bins(b[8], b[8], w128, 128);
        pf[0] = (float)(dc * dc);     // DC / Nyquist from the fp64 sums (the pre-emphasised DC bin
        pf[256] = (float)(ny * ny);   // cancels in fp32)
      }
    }
    wave_lds_fence();
    // mel pairs (filter l and 119 - l), |X|^2 / 512 (:44, an exact power of two), eps floor, 20 log10
    if (lane < kFbPairs) {
      float* o = out + (clip * 98 + 4 * c) * 120;
      // the pair's tap weights, read once per item, split into the two filters (zero elsewhere): a
      // tap is then one LDS read and two multiply-adds, no per-tap selects
      float wa[kFbPairTaps], wb[kFbPairTaps];
#pragma unroll
      for (int q = 0; q < kFbPairTaps; ++q) {
        const float w = pw[q];
        wa[q] = q < meta.y ? w : 0.f;
        wb[q] = q < meta.y ? 0.f : w;
      }
      const int ka = meta.x, kb = meta.z - meta.y;   // tap q reads bin (q < cnt_a ? ka : kb) + q
#pragma unroll
      for (int ff = 0; ff < 4; ++ff) {
        if (4 * c + ff >= 98) break;
        const float* pp = pb + ff * 272;
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int q = 0; q < kFbPairTaps; ++q) {
          const float v = pp[min((q < meta.y ? ka : kb) + q, 256)];
          sa += wa[q] * v;
          sb += wb[q] * v;
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

// ------------------------------------------------------------------------- K4 noise mix (shared)
// numpy: sample + (gain * noise) in float64 (two roundings, never fused), then np.int16()
// truncates toward zero.
__device__ __forceinline__ float mix_one(short s, double g, short n) {
#pragma clang fp contract(off)
  const double v = (double)s + g * (double)n;
  return (float)(int16_t)(int)v;
}

// K4 fused into K3's sample loads (srk_spec_noise_fwd, model_spec_bgru + dataset.py:183-193): the kernel
// reads the int16 clip and its noise window and mixes each sample as it loads it, so the mixed fp32 PCM
// never goes through HBM (128,000 B/clip for the separate K4 + 64,000 re-read by K3 -> 64,000 in).
struct NoiseArgs {
  const int16_t* bank;       // [n_files][bank_len]
  int64_t n_files, bank_len;
  const int64_t* file_idx;   // [n_clips]
  const int64_t* offs;       // [n_clips]
  const double* gains;       // [n_clips]
};

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

template <typename T, bool MIX = false>
__global__ __launch_bounds__(256, 4) void spec_kernel(const T* __restrict__ pcm, float* __restrict__ out,
                                                      int64_t n_clips, int transposed, SpecTables t,
                                                      NoiseArgs nm = NoiseArgs{}) {
  __shared__ v2f sbuf[4][3 * 340];
  __shared__ __attribute__((aligned(16))) double s_win[640];
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
    const T* __restrict__ x = pcm + clip * kPcmLen + 320 * (live ? gf : 0);
    // every lane loads (a dead lane's x is frame 0 of the clip) and the products are masked after:
    // with the loads under the `live` condition the compiler serialises 40 load / LDS waits
    v2f xv[20];
    if constexpr (MIX) {
      // the clip's noise window (file, offset clamped into the bank as in noise_mix_kernel) mixed in at load
      const int64_t fi = min(max(nm.file_idx[clip], (int64_t)0), nm.n_files - 1);
      const int64_t off = min(max(nm.offs[clip], (int64_t)0), nm.bank_len - kPcmLen);
      const double g = nm.gains[clip];
      const int64_t base = fi * nm.bank_len + off;
      const int16_t* __restrict__ nz = nm.bank + base + 320 * (live ? gf : 0);
      if ((base & 1) == 0) {   // wave-uniform: sample pairs of the noise window are 4-B aligned
#pragma unroll
        for (int i = 0; i < 20; ++i) {
          const short2 sv = *reinterpret_cast<const short2*>(x + 2 * (j + 16 * i));
          const short2 nv = *reinterpret_cast<const short2*>(nz + 2 * (j + 16 * i));
          xv[i] = v2f{mix_one(sv.x, g, nv.x), mix_one(sv.y, g, nv.y)};
        }
      } else {                 // odd window start: 2-B noise loads (every access naturally aligned)
#pragma unroll
        for (int i = 0; i < 20; ++i) {
          const short2 sv = *reinterpret_cast<const short2*>(x + 2 * (j + 16 * i));
          const short n0 = nz[2 * (j + 16 * i)], n1 = nz[2 * (j + 16 * i) + 1];
          xv[i] = v2f{mix_one(sv.x, g, n0), mix_one(sv.y, g, n1)};
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 20; ++i) xv[i] = ld2(x + 2 * (j + 16 * i));
    }
    v2f tw[19];   // pass-A twiddles, read ahead of the transpose stores
#pragma unroll
    for (int k1 = 1; k1 < 20; ++k1) tw[k1 - 1] = s_tw[k1 * 16 + j];
    v2f a[20];
    double dc = 0.0, ny = 0.0;
#pragma unroll
    for (int i = 0; i < 20; ++i) {
      const int n = j + 16 * i;
      const double2 w = *reinterpret_cast<const double2*>(s_win + 2 * n);
      double d0 = (double)xv[i].x * w.x, d1 = (double)xv[i].y * w.y;
      d0 = live ? d0 : 0.0;
      d1 = live ? d1 : 0.0;
      a[i] = v2f{(float)d0, (float)d1};
      dc += d0 + d1;
      ny += d0 - d1;
    }
    dc = group16_sum(dc);
    ny = group16_sum(ny);
    dft20v(a);
    if (fa < 3) {
#pragma unroll
      for (int k1 = 0; k1 < 20; ++k1) tb[fa * 340 + k1 * 17 + j] = k1 ? pcmul(a[k1], tw[k1 - 1]) : a[0];
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
        const v2f X = e + pcmul(oo, s_post[k]);
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

// ------------------------------------------------------------------------- K1 MFCC
template <typename T>
__device__ __forceinline__ void mfcc_load_chunk(const T* __restrict__ x, int c, int lane, v2f (&raw)[20]) {
  const int fa = lane >> 4, j = lane & 15;
  const int gf = 3 * c + (fa < 3 ? fa : 0);
  if (c > 0 && c < 16) {   // wave-uniform: frames 3..47 never touch the reflected padding
#pragma unroll
    for (int i = 0; i < 20; ++i) raw[i] = ld2(x + 320 * gf + 2 * (j + 16 * i) - 320);
  } else {
#pragma unroll
    for (int i = 0; i < 20; ++i) {
      int s0 = 320 * gf + 2 * (j + 16 * i) - 320, s1 = s0 + 1;
      s0 = s0 < 0 ? -s0 : (s0 > kPcmLen - 1 ? 2 * (kPcmLen - 1) - s0 : s0);
      s1 = s1 < 0 ? -s1 : (s1 > kPcmLen - 1 ? 2 * (kPcmLen - 1) - s1 : s1);
      raw[i] = v2f{ld1(x + s0), ld1(x + s1)};
    }
  }
}

// ------------------------------------------------------------------------- K1 MFCC (v3)
// Workgroup = 4 waves, persistent over clips, 2 workgroups per CU (67.4 KB LDS each).  Per clip the
// waves split the 17 chunks of 3 frames; per chunk and wave, all in registers except two LDS
// round trips:
//   pass A  lane (frame, j): 20-point DFT of the windowed samples, twiddle, LDS transpose;
//   pass B  lane (frame, k1): 16-point DFT -> Z[k1 + 20 k2] in registers; the packed-real untangle
//           pairs Z[k] with Z[320 - k], held by lane (frame, 20 - k1) at k2' = 15 - k2: ONE
//           ds_bpermute per float instead of an LDS spectrum write + two reads; |X[k]|^2 -> LDS;
//   mel     each lane owns a narrow (<= 3 bins) and a wide (<= 15 bins) filter: 18 taps read from LDS
//           with immediate offsets (window starts chosen bank-conflict-free, runtime.hip), weights in
//           registers; power_to_db -> the clip's dB image in LDS.
// Lane constants (window, mel weights) stay in registers for the whole kernel; the twiddles are read
// from LDS.
// After one workgroup barrier (the clip's top_db max), the DCT-II runs on the fp32 matrix cores:
// C[16 x 64] = DCT[16 x 128] . max(dB, floor)[128 x 64], one 16-frame column tile per wave
// (v_mfma_f32_16x16x4_f32, exact fp32 products), then the deltas and the store.
constexpr int kM3Waves = 4;
constexpr int kM3DbP = 132;   // dB image [frame][band] pitch (16-B rows)
constexpr int kM3CP = 53;     // coefficient image [13][53] (odd pitch: the delta reads of 13 rows spread over banks)


typedef float f32x4_ __attribute__((ext_vector_type(4)));

// Diagnostic build only (tools/build_variant.sh ... -DSRK_MFCC_STAMPS): per-wave s_memtime phase
// totals, read back by srk_debug_mfcc_stamps (tools/mfcc_stamps.py).  Never in the product build.
// Diagnostic builds only (tools/build_variant.sh ... -DSRK_MFCC_STOP=n, tools/feat_budget.sh): the chunk
// step ends after phase n (0 = the sample loads only, 1 = + window / pass A / transpose, 2 = + pass B,
// 3 = + untangle, 4 = everything), so per-phase instruction counts are differences of SQ_INSTS_* per clip.
#ifndef SRK_MFCC_STOP
#define SRK_MFCC_STOP 4
#endif

#ifdef SRK_MFCC_STAMPS
constexpr int kStampPhases = 10;
__device__ unsigned long long g_mfcc_stamps[512 * kM3Waves * kStampPhases];
#define MFCC_STAMP(p)                                                   \
  do {                                                                  \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
    st_acc[p] += t_ - st_last;                                          \
    st_last = t_;                                                       \
  } while (0)
#else
#define MFCC_STAMP(p) do { } while (0)
#endif

// Pass-B lane layout of the DPP untangle (DPP = true): the partner (frame, 20 - k1) of lane (frame, k1)
// sits at the DPP row_mirror position (lane ^ 15 within its 16-lane row), so the 16 partner values
// move by v_mov_b32 dpp row_mirror (VALU) instead of ds_bpermute (LDS pipe, 24-49 cycles a wave).
// Rows 0-2 = frames 0-2, k1 = 1..8 at p = 0..7 and 12..19 at p = 8..15.  Row 3: (f, 9) at p = f and
// (f, 11) at 15 - f; (f, 10) at 3 + f with a duplicate at 12 - f (its mirror); (f, 0) at 6 + f (own
// values, as before); p = 9 idle.  Duplicates and the idle lane write into the slice's unused tail.
__device__ __forceinline__ void mfcc_passb_lane(int lane, int& fb, int& k1, int& fbw) {
  const int r = lane >> 4, p = lane & 15;
  fbw = -1;
  if (r < 3) {
    fb = r;
    k1 = p < 8 ? p + 1 : p + 4;
  } else if (p < 3) {
    fb = p; k1 = 9;
  } else if (p >= 13) {
    fb = 15 - p; k1 = 11;
  } else if (p < 6) {
    fb = p - 3; k1 = 10;
  } else if (p >= 10) {
    fb = 12 - p; k1 = 10; fbw = 3;
  } else if (p < 9) {
    fb = p - 6; k1 = 0;
  } else {
    fb = 2; k1 = 0; fbw = 3;
  }
  if (fbw < 0) fbw = fb;
}

__device__ __forceinline__ float dpp_mirror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140 /* row_mirror */, 0xF, 0xF, false));
}

// VAR bit 0: the DPP untangle exchange; bit 1: the pass-A and untangle twiddles held in registers for
// the whole kernel (lane constants) instead of 28 LDS reads per chunk
template <int VAR, typename T>
__global__ __launch_bounds__(64 * kM3Waves, 2) void mfcc3_kernel(const T* __restrict__ pcm, float* __restrict__ out,
                                                                  int layout, int64_t n_clips, DeviceTables t) {
  __shared__ __attribute__((aligned(16))) v2f tbuf[kM3Waves][3 * 340];
  constexpr int DBP = kM3DbP;
  __shared__ __attribute__((aligned(16))) float db[51 * kM3DbP];
  __shared__ v2f s_tw[20 * 16];   // W320^(j k1) at [k1][j]
  __shared__ v2f s_post[320];     // W640^k (untangle twiddles)
  __shared__ float cbuf[2][13 * kM3CP];                         // coefficient images, alternating clips
  __shared__ __attribute__((aligned(16))) float s_dct[13 * kM3DbP];   // DCT-II rows (ortho), pitch 132: the
                                                                       // 16-B fragment reads of 16 rows hit distinct banks
  __shared__ float red[kM3Waves];
  // the wave index in an SGPR: the chunk loop and its reflect / tail branches stay scalar
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fa = lane >> 4, j = lane & 15;           // pass A
  constexpr bool DPP = (VAR & 1) != 0, TWREG = (VAR & 2) != 0;
  // pass B: lane (frame fb, k1b); bins written to frame fbw's slice (3 = the unused tail)
  int fb, k1b, fbw;
  if (DPP) {
    mfcc_passb_lane(lane, fb, k1b, fbw);
  } else {
    fb = lane / 20;                                  // fb == 3: lanes 60..63 idle
    k1b = lane - 20 * fb;
    fbw = fb;
  }
  for (int i = threadIdx.x; i < 320; i += 64 * kM3Waves)
    s_tw[i] = *reinterpret_cast<const v2f*>(t.tw320 + ((i >> 4) * (i & 15)));
  v2f win[20];
#pragma unroll
  for (int i = 0; i < 20; ++i) win[i] = *reinterpret_cast<const v2f*>(t.hann640f + 2 * (j + 16 * i));
  for (int i = threadIdx.x; i < 320; i += 64 * kM3Waves) s_post[i] = *reinterpret_cast<const v2f*>(t.post640 + i);
  for (int i = threadIdx.x; i < 13 * 128; i += 64 * kM3Waves) s_dct[(i >> 7) * kM3DbP + (i & 127)] = t.dct[i];
  const int4 mlo = t.melq_lo[lane];   // {window start a, window start b, filter a, filter b}
  float mw[18];
#pragma unroll
  for (int q = 0; q < 18; ++q) mw[q] = 0.25f * t.melq_w[q * 64 + lane];   // the LDS holds 4 |X|^2
  const int pbyte = 4 * (fb < 3 ? fb * 20 + (k1b == 0 ? 0 : 20 - k1b) : lane);
  // pin the lane constants in registers: left alone, the compiler re-loads these invariant table
  // entries from global memory inside the chunk loop and waits on them there
#pragma unroll
  for (int i = 0; i < 20; ++i) asm volatile("" : "+v"(win[i]));
#pragma unroll
  for (int q = 0; q < 18; ++q) asm volatile("" : "+v"(mw[q]));
  __syncthreads();
  v2f twr[TWREG ? 19 : 1], wpr[TWREG ? 9 : 1];   // TWREG: W320^(j k1), k1 = 1..19; W640^(k1b + 20 k2), k2 < 8, and W640^160
  if (TWREG) {
#pragma unroll
    for (int k1 = 1; k1 < 20; ++k1) twr[k1 - 1] = s_tw[k1 * 16 + j];
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) wpr[k2] = s_post[k1b + 20 * k2];
    wpr[8] = s_post[160];
#pragma unroll
    for (int i = 0; i < 19; ++i) asm volatile("" : "+v"(twr[i]));
#pragma unroll
    for (int i = 0; i < 9; ++i) asm volatile("" : "+v"(wpr[i]));
  }
  v2f* tb = tbuf[wave];
  float* pb = reinterpret_cast<float*>(tb);   // |X|^2 [3][321] over the transpose slice
#ifdef SRK_MFCC_STAMPS
  unsigned long long st_acc[kStampPhases] = {}, st_last = __builtin_amdgcn_s_memtime();
#endif

  // Chunk order: wave w takes chunks (w + 4 k + 2) mod 17, k < nsteps, so the wave with the fifth
  // chunk (wave 0) holds none of the two reflect-padded edge chunks (0 and 16, the dearer loads).
  const int nsteps = (17 - wave + kM3Waves - 1) / kM3Waves;   // 5 for wave 0, else 4 (uniform)
  auto chunk_of = [&](int k) { return (wave + kM3Waves * k + 2) % 17; };
  // One chunk of 3 frames (the wave's k-th): consumes `raw` (its samples) and, right after the
  // 20-point DFTs, re-fills it with the wave's next chunk (this clip's, else the next clip's first),
  // so those loads overlap pass B, the untangle and the mel reduction.
  auto step = [&](v2f (&raw)[20], int64_t clip, int k, float& vmax) {
    const int c = chunk_of(k);
    if (SRK_MFCC_STOP == 0) {
      const bool more = k + 1 < nsteps;
      int64_t nclip = more ? clip : clip + gridDim.x;
      nclip = nclip < n_clips ? nclip : clip;
#pragma unroll
      for (int i = 0; i < 20; ++i) asm volatile("" :: "v"(raw[i].x), "v"(raw[i].y));
      mfcc_load_chunk(pcm + nclip * kPcmLen, chunk_of(more ? k + 1 : 0), lane, raw);
      return;
    }
    v2f a[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) a[i] = raw[i] * win[i];
    // the 19 twiddles are read before the DFT: read between the transpose stores, each one would
    // wait out its own LDS round trip (the compiler keeps loads behind stores it cannot disambiguate)
    v2f tw[19];
#pragma unroll
    for (int k1 = 1; k1 < 20; ++k1) tw[k1 - 1] = TWREG ? twr[k1 - 1] : s_tw[k1 * 16 + j];
    dft20v(a);
    if (fa < 3) {
#pragma unroll
      for (int k1 = 0; k1 < 20; ++k1) tb[fa * 340 + k1 * 17 + j] = k1 ? pcmul(a[k1], tw[k1 - 1]) : a[0];
    }
    MFCC_STAMP(0);
    {  // next: this clip's next chunk, else the next clip's first (past the end: a re-read)
      const bool more = k + 1 < nsteps;
      int64_t nclip = more ? clip : clip + gridDim.x;
      nclip = nclip < n_clips ? nclip : clip;
      mfcc_load_chunk(pcm + nclip * kPcmLen, chunk_of(more ? k + 1 : 0), lane, raw);
    }
    if (SRK_MFCC_STOP == 1) return;
    wave_lds_fence();
    // lanes 60..63 (fb = 3) duplicate frame 2's reads and park their results in the unused tail
    // of the slice (3 * 321 + 303 < 2 * 1020 floats): no divergent branches in this phase
    v2f b[16];
    const int fbr = fb < 3 ? fb : 2;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) b[jj] = tb[fbr * 340 + k1b * 17 + jj];
    dft16v(b);
    if (SRK_MFCC_STOP == 2) {
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) asm volatile("" :: "v"(b[jj].x), "v"(b[jj].y));
      return;
    }
    wave_lds_fence();
    MFCC_STAMP(1);
    // untangle the packed real FFT: with A = Z[k], B = Z[320 - k], W = W640^k,
    //   2 E = (A.x + B.x, A.y - B.y) = S,  2 O = -i (A - B*) = (A.y + B.y, B.x - A.x) = U,
    //   2 X[k] = S + W U,  2 X[320 - k] = (S - W U)*,
    // so one (A, B) pair gives two bins.  Lane (frame, k1) pairs its k2 < 8 with the partner lane
    // (frame, 20 - k1) at 15 - k2 (ds_bpermute), which in turn covers the other 8; k1 = 0 and 10 pair
    // inside the lane, and k1 = 0 also takes the self-paired bin 160.  The LDS holds |2 X|^2 = 4 |X|^2;
    // the factor 1/4 is folded into the mel weights (exact).
    float Bx[8], By[8];
    v2f wpost[8];   // untangle twiddles, requested with the partner values (not between the stores)
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) wpost[k2] = TWREG ? wpr[k2] : s_post[k1b + 20 * k2];
    const v2f w160 = TWREG ? wpr[8] : s_post[160];
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      if (DPP) {
        Bx[k2] = dpp_mirror(b[15 - k2].x);
        By[k2] = dpp_mirror(b[15 - k2].y);
      } else {
        Bx[k2] = bperm(pbyte, b[15 - k2].x);
        By[k2] = bperm(pbyte, b[15 - k2].y);
      }
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the 24 requests ahead of their consumers
    float* pf = pb + fbw * 321;
    auto two_bins = [&](v2f A, v2f B, v2f w, int k) {
      const v2f p = untangle_pk(A, B, w);
      pf[320 - k] = p.y;   // first: bin 160 pairs with itself, |S + W U|^2 stands
      pf[k] = p.x;
    };
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      const float bx = k1b == 0 ? b[(16 - k2) & 15].x : Bx[k2];
      const float by = k1b == 0 ? b[(16 - k2) & 15].y : By[k2];
      two_bins(b[k2], v2f{bx, by}, wpost[k2], k1b + 20 * k2);
    }
    if (k1b == 0) two_bins(b[8], b[8], w160, 160);
    if (SRK_MFCC_STOP == 3) return;
    wave_lds_fence();
    MFCC_STAMP(2);
    // Slaney mel (the lane's narrow and wide filter) -> power_to_db(ref = 1, amin = 1e-10).  The 18
    // taps of frame ff + 1 are requested before frame ff's sums run (LDS latency off the chain).
    const int f0 = 3 * c;
    const int nf = f0 + 3 <= 51 ? 3 : 51 - f0;   // uniform
    float pv[2][18];
    auto read_taps = [&](int ff, float (&v)[18]) {
      const float* p = pb + ff * 321;
#pragma unroll
      for (int q = 0; q < 3; ++q) v[q] = p[mlo.x + q];
#pragma unroll
      for (int q = 0; q < 15; ++q) v[3 + q] = p[mlo.y + q];
    };
    read_taps(0, pv[0]);
#pragma unroll
    for (int ff = 0; ff < 3; ++ff) {
      if (ff >= nf) break;   // uniform
      if (ff + 1 < nf) read_taps(ff + 1, pv[(ff + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      const float* v = pv[ff & 1];
      float s0 = mw[0] * v[0], s1 = mw[3] * v[3], s2 = mw[4] * v[4];
      s0 = fmaf(mw[1], v[1], s0);
      s0 = fmaf(mw[2], v[2], s0);
#pragma unroll
      for (int q = 5; q < 18; q += 2) {
        s1 = fmaf(mw[q], v[q], s1);
        if (q + 1 < 18) s2 = fmaf(mw[q + 1], v[q + 1], s2);
      }
      s1 += s2;
      const float v0 = s0 > 1e-10f ? 10.0f * fast_log10(s0) : -100.0f;
      const float v1 = s1 > 1e-10f ? 10.0f * fast_log10(s1) : -100.0f;
      db[(f0 + ff) * DBP + mlo.z] = v0;
      db[(f0 + ff) * DBP + mlo.w] = v1;
      vmax = fmaxf(vmax, fmaxf(v0, v1));
    }
    wave_lds_fence();
    MFCC_STAMP(3);
  };

  // [C; dC; ddC] of one clip from its coefficient image: np.gradient (edge_order 1) twice.  Item =
  // (coefficient, block of 4 frames), 13 x 13 items over `nthr` threads; an item reads the 8 image
  // values its frames and their 2-frame neighbourhoods need.
  auto emit = [&](const float* cb, int64_t clip, int tid, int nthr) {
    float* o = out + clip * 39 * 51;
    for (int it = tid; it < 13 * 13; it += nthr) {
      int cr, fb4;
      if (layout == 0) { cr = it / 13; fb4 = it - 13 * cr; } else { fb4 = it / 13; cr = it - 13 * fb4; }
      const int f0 = 4 * fb4;
      const float* r = cb + cr * kM3CP;
      float w[8];   // frames f0 - 2 .. f0 + 5, clamped
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = r[min(max(f0 - 2 + u, 0), 50)];
      auto G = [&](int p, int u) {   // gradient at frame p = f0 - 2 + u
        return p == 0 ? w[u + 1] - w[u] : (p == 50 ? w[u] - w[u - 1] : (w[u + 1] - w[u - 1]) * 0.5f);
      };
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int f = f0 + q;
        if (f > 50) break;
        const float g0 = G(f, q + 2);
        const float g2 = f == 0 ? G(f + 1, q + 3) - g0
                                : (f == 50 ? g0 - G(f - 1, q + 1) : (G(f + 1, q + 3) - G(f - 1, q + 1)) * 0.5f);
        if (layout == 0) {
          o[cr * 51 + f] = w[q + 2];
          o[(13 + cr) * 51 + f] = g0;
          o[(26 + cr) * 51 + f] = g2;
        } else {
          o[f * 39 + cr] = w[q + 2];
          o[f * 39 + 13 + cr] = g0;
          o[f * 39 + 26 + cr] = g2;
        }
      }
    }
  };

  // Per clip: the 17 chunks (wave 0 takes 5, the others 4), then the top_db max, the DCT into
  // cbuf[clip parity] and the barrier that frees db.  The previous clip's output is written from
  // its coefficient image by waves 1..3 while wave 0 runs its fifth chunk, off the barrier.
  v2f raw[20];
  if ((int64_t)blockIdx.x < n_clips) mfcc_load_chunk(pcm + (int64_t)blockIdx.x * kPcmLen, chunk_of(0), lane, raw);
  int par = 0;
  for (int64_t clip = blockIdx.x; clip < n_clips; clip += gridDim.x, par ^= 1) {
    float vmax = -INFINITY;
    for (int k = 0; k < nsteps; ++k) step(raw, clip, k, vmax);
    if (wave > 0 && clip != (int64_t)blockIdx.x) {
      emit(cbuf[par ^ 1], clip - gridDim.x, threadIdx.x - 64, 64 * (kM3Waves - 1));
      MFCC_STAMP(8);
    }
    vmax = wave_max(vmax);
    if (lane == 0) red[wave] = vmax;
    MFCC_STAMP(4);
    __syncthreads();
    MFCC_STAMP(5);
    float mx = red[0];
#pragma unroll
    for (int w = 1; w < kM3Waves; ++w) mx = fmaxf(mx, red[w]);
    const float floor_db = mx - 80.0f;
    {  // DCT-II (ortho, 13 rows) on the matrix cores: wave = frames [16 wave, 16 wave + 16)
      const int row = lane & 15, kq = 4 * (lane >> 4);
      const int fr = min(16 * wave + row, 50);
      const float* dr = db + fr * DBP + kq;
      const float* ar = s_dct + min(row, 12) * kM3DbP + kq;
      f32x4_ acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 8; ++kb) {
        const v4f bv = *reinterpret_cast<const v4f*>(dr + 16 * kb);
        v4f av = *reinterpret_cast<const v4f*>(ar + 16 * kb);
        if (row >= 13) av = v4f{0.f, 0.f, 0.f, 0.f};
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, fmaxf(bv.x, floor_db), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, fmaxf(bv.y, floor_db), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, fmaxf(bv.z, floor_db), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, fmaxf(bv.w, floor_db), acc, 0, 0, 0);
      }
      // acc[r] = C[coef 4 (lane >> 4) + r][frame 16 wave + (lane & 15)]
      const int fo = 16 * wave + row;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int coef = kq + r;
        if (coef < 13 && fo < 51) cbuf[par][coef * kM3CP + fo] = acc[r];
      }
    }
    MFCC_STAMP(6);
    __syncthreads();   // cbuf[par] complete; db free for the next clip
    MFCC_STAMP(7);
  }
  {  // the last clip's output, all waves
    const int64_t nmine = ((int64_t)blockIdx.x < n_clips) ? (n_clips - 1 - blockIdx.x) / gridDim.x + 1 : 0;
    if (nmine > 0) emit(cbuf[par ^ 1], blockIdx.x + (nmine - 1) * gridDim.x, threadIdx.x, 64 * kM3Waves);
    MFCC_STAMP(8);
  }
#ifdef SRK_MFCC_STAMPS
  if (lane == 0) {
    unsigned long long* d = g_mfcc_stamps + ((size_t)blockIdx.x * kM3Waves + wave) * kStampPhases;
#pragma unroll
    for (int p = 0; p < kStampPhases - 1; ++p) d[p] = st_acc[p];
    d[kStampPhases - 1] = 1;
  }
#endif
}

// ------------------------------------------------------------------------- K4 noise mix
__global__ void noise_mix_kernel(const int16_t* __restrict__ pcm, const int16_t* __restrict__ bank,
                                 int64_t n_files, int64_t bank_len, const int64_t* __restrict__ file_idx,
                                 const int64_t* __restrict__ offs, const double* __restrict__ gains,
                                 int64_t n_clips, float* __restrict__ out) {
  // 8 samples per thread: 16-B int16 loads of pcm, 16-B + 16-B fp32 stores.
  const int64_t i8 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total8 = n_clips * (kPcmLen / 8);
  if (i8 >= total8) return;
  const int64_t clip = i8 / (kPcmLen / 8);
  const int s0 = (int)(i8 % (kPcmLen / 8)) * 8;
  // the host validates the draws before an eager launch; inside a captured graph it cannot read them,
  // so the file and offset are also clamped here: an invalid draw can never read outside the bank
  const int64_t f = min(max(file_idx[clip], (int64_t)0), n_files - 1);
  const int64_t off = min(max(offs[clip], (int64_t)0), bank_len - kPcmLen);
  const int16_t* nz = bank + f * bank_len + off + s0;
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

#ifdef SRK_MFCC_STAMPS
extern "C" int srk_debug_mfcc_stamps(unsigned long long* host, int64_t n) {
  const int64_t cap = 512 * srk::kM3Waves * srk::kStampPhases;
  if (n > cap) n = cap;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(srk::g_mfcc_stamps), n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
#endif

namespace srk {
namespace {

template <typename T>
int fbank_fwd(const T* pcm, int64_t n_clips, float* out, void* stream) {
  SRK_REQUIRE(n_clips >= 0 && n_clips <= INT32_MAX, SRK_ERR_INVALID, "srk_fbank_fwd: bad n_clips %lld", (long long)n_clips);
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(pcm && out, SRK_ERR_INVALID, "srk_fbank_fwd: null pointer");
  SRK_REQUIRE((uintptr_t)pcm % (2 * sizeof(T)) == 0, SRK_ERR_INVALID, "srk_fbank_fwd: pcm must be %d-byte aligned",
              (int)(2 * sizeof(T)));
  const DeviceTables* t = nullptr;
  if (int rc = get_tables(&t)) return rc;
  FbankTables ft{t->hamming400, t->tw256, t->post512, t->fbp_meta, t->fbp_w};
  const int64_t items = n_clips * kFbChunks;
  const int64_t blocks = std::min<int64_t>((items + 3) / 4, 2048);   // waves take (clip, 4-frame chunk) items
  // algorithmic bytes: the PCM in (64000 B/clip as fp32, 32000 as int16) + 47040 out
  ProfScope prof("fbank", as_stream(stream), (16000.0 * sizeof(T) + 47040.0) * (double)n_clips);
  hipLaunchKernelGGL(fbank_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), pcm, out, n_clips, ft);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

template <typename T>
int spec_fwd(const T* pcm, int64_t n_clips, float* out, int transposed, void* stream, const NoiseArgs* nm = nullptr) {
  SRK_REQUIRE(n_clips >= 0 && n_clips <= INT32_MAX, SRK_ERR_INVALID, "srk_spec_fwd: bad n_clips");
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(pcm && out, SRK_ERR_INVALID, "srk_spec_fwd: null pointer");
  SRK_REQUIRE((uintptr_t)pcm % (2 * sizeof(T)) == 0, SRK_ERR_INVALID, "srk_spec_fwd: pcm must be %d-byte aligned",
              (int)(2 * sizeof(T)));
  const DeviceTables* t = nullptr;
  if (int rc = get_tables(&t)) return rc;
  SpecTables st{t->tukey640, t->tw320, t->post640, (float)t->spec_scale};
  const int64_t items = n_clips * kSpChunks;
  const int64_t blocks = std::min<int64_t>((items + 3) / 4, 2048);
  hipStream_t s = as_stream(stream);
  if (nm) {   // K4 + K3: int16 clip + int16 noise window in, the spectrogram out (126,916 B/clip)
    ProfScope prof("spec", s, (32000.0 + 32000.0 + 62916.0) * (double)n_clips);
    prof.detail("spec_kernel<int16,noise_mix>");
    hipLaunchKernelGGL((spec_kernel<int16_t, true>), dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<const int16_t*>(pcm), out, n_clips, transposed ? 1 : 0, st, *nm);
  } else {
    ProfScope prof("spec", s, (16000.0 * sizeof(T) + 62916.0) * (double)n_clips);
    hipLaunchKernelGGL(spec_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, pcm, out, n_clips,
                       transposed ? 1 : 0, st, NoiseArgs{});
  }
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

template <typename T>
int mfcc_fwd(const T* pcm, int64_t n_clips, float* out, int layout, void* stream) {
  SRK_REQUIRE(n_clips >= 0 && n_clips <= INT32_MAX, SRK_ERR_INVALID, "srk_mfcc_fwd: bad n_clips");
  SRK_REQUIRE(layout == 0 || layout == 1, SRK_ERR_INVALID, "srk_mfcc_fwd: layout must be 0 or 1");
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(pcm && out, SRK_ERR_INVALID, "srk_mfcc_fwd: null pointer");
  SRK_REQUIRE((uintptr_t)pcm % (2 * sizeof(T)) == 0, SRK_ERR_INVALID, "srk_mfcc_fwd: pcm must be %d-byte aligned",
              (int)(2 * sizeof(T)));
  const DeviceTables* t = nullptr;
  if (int rc = get_tables(&t)) return rc;
  ProfScope prof("mfcc", as_stream(stream), (16000.0 * sizeof(T) + 7956.0) * (double)n_clips);
  const int64_t grid = std::min<int64_t>(n_clips, 256 * 2);   // persistent over clips, 2 per CU
  const dim3 g((unsigned)grid), b(64 * kM3Waves);
  hipStream_t s = as_stream(stream);
  if (sizeof(T) == 2) {   // the int16 input: the default variant only
    hipLaunchKernelGGL((mfcc3_kernel<3, T>), g, b, 0, s, pcm, out, layout, n_clips, *t);
  } else {
    switch (g_opt_mfcc_variant) {
      case 1: hipLaunchKernelGGL((mfcc3_kernel<1, T>), g, b, 0, s, pcm, out, layout, n_clips, *t); break;
      case 2: hipLaunchKernelGGL((mfcc3_kernel<2, T>), g, b, 0, s, pcm, out, layout, n_clips, *t); break;
      case 3: hipLaunchKernelGGL((mfcc3_kernel<3, T>), g, b, 0, s, pcm, out, layout, n_clips, *t); break;
      default: hipLaunchKernelGGL((mfcc3_kernel<0, T>), g, b, 0, s, pcm, out, layout, n_clips, *t);
    }
  }
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

}  // namespace
}  // namespace srk

extern "C" {

int srk_fbank_fwd(const float* pcm, int64_t n_clips, float* out, void* stream) {
  SRK_API_BEGIN
  return srk::fbank_fwd(pcm, n_clips, out, stream);
  SRK_API_END
}

int srk_fbank_fwd_i16(const int16_t* pcm, int64_t n_clips, float* out, void* stream) {
  SRK_API_BEGIN
  return srk::fbank_fwd(pcm, n_clips, out, stream);
  SRK_API_END
}

int srk_spec_fwd(const float* pcm, int64_t n_clips, float* out, int transposed, void* stream) {
  SRK_API_BEGIN
  return srk::spec_fwd(pcm, n_clips, out, transposed, stream);
  SRK_API_END
}

int srk_spec_fwd_i16(const int16_t* pcm, int64_t n_clips, float* out, int transposed, void* stream) {
  SRK_API_BEGIN
  return srk::spec_fwd(pcm, n_clips, out, transposed, stream);
  SRK_API_END
}

int srk_spec_noise_fwd(const int16_t* pcm, const int16_t* bank, int64_t n_files, int64_t bank_len,
                       const int64_t* file_idx, const int64_t* offset, const double* gain, int64_t n_clips, float* out,
                       int transposed, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n_clips >= 0, SRK_ERR_INVALID, "srk_spec_noise_fwd: bad n_clips");
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(bank && file_idx && offset && gain, SRK_ERR_INVALID, "srk_spec_noise_fwd: null pointer");
  SRK_REQUIRE(n_files > 0 && bank_len >= 16000, SRK_ERR_INVALID,
              "srk_spec_noise_fwd: bank must hold >= 1 file of >= 16000 samples");
  SRK_REQUIRE((uintptr_t)bank % 4 == 0, SRK_ERR_INVALID, "srk_spec_noise_fwd: bank must be 4-byte aligned");
  const srk::NoiseArgs nm{bank, n_files, bank_len, file_idx, offset, gain};
  return srk::spec_fwd(pcm, n_clips, out, transposed, stream, &nm);
  SRK_API_END
}

int srk_mfcc_fwd(const float* pcm, int64_t n_clips, float* out, int layout, void* stream) {
  SRK_API_BEGIN
  return srk::mfcc_fwd(pcm, n_clips, out, layout, stream);
  SRK_API_END
}

int srk_mfcc_fwd_i16(const int16_t* pcm, int64_t n_clips, float* out, int layout, void* stream) {
  SRK_API_BEGIN
  return srk::mfcc_fwd(pcm, n_clips, out, layout, stream);
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
                     n_files, bank_len, file_idx, offset, gain, n_clips, out);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
