// K1 MFCC, K2 log-mel fbank, K3 log spectrogram, K4 noise-mix — gfx950 HIP kernels.
//
// Design: one workgroup per clip, frames processed in chunks of F.
// Per chunk:
//   load   : wave-per-frame coalesced float2 loads of PCM, window applied in fp64, packed as
//            z[n] = x[2n] + i x[2n+1] (real N-point FFT via an N/2-point complex FFT); the DC and
//            Nyquist sums are accumulated in fp64 in the same pass (fp32 cancellation in the DC
//            bin costs up to 0.17 dB in fbank column 1 otherwise — SURVEY.md Appendix A).
//   fft    : mixed-radix Stockham passes (radix 4 / 5) in LDS, twiddles from a table.
//   untangle + |X|^2, then the feature-specific reduction (sparse mel, log, DCT ...).
#include "srk_internal.h"

namespace srk {
namespace {

constexpr int kPcmLen = 16000;

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }   // -i * a

template <int R>
__device__ __forceinline__ void dft(float2 (&v)[R]);

template <>
__device__ __forceinline__ void dft<4>(float2 (&v)[4]) {
  const float2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
  const float2 s13 = cadd(v[1], v[3]), d13 = mul_mi(csub(v[1], v[3]));
  v[0] = cadd(s02, s13);
  v[2] = csub(s02, s13);
  v[1] = cadd(d02, d13);
  v[3] = csub(d02, d13);
}

template <>
__device__ __forceinline__ void dft<5>(float2 (&v)[5]) {
  constexpr float c1 = 0.30901699437494745f, c2 = -0.8090169943749473f;
  constexpr float s1 = 0.9510565162951535f, s2 = 0.5877852522924732f;
  const float2 t1 = cadd(v[1], v[4]), t2 = cadd(v[2], v[3]);
  const float2 t3 = csub(v[1], v[4]), t4 = csub(v[2], v[3]);
  const float2 b1 = make_float2(v[0].x + c1 * t1.x + c2 * t2.x, v[0].y + c1 * t1.y + c2 * t2.y);
  const float2 b2 = make_float2(v[0].x + c2 * t1.x + c1 * t2.x, v[0].y + c2 * t1.y + c1 * t2.y);
  const float2 q1 = make_float2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y);   // -i*q1 for y1
  const float2 q2 = make_float2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y);
  v[0] = make_float2(v[0].x + t1.x + t2.x, v[0].y + t1.y + t2.y);
  v[1] = cadd(b1, mul_mi(q1));
  v[4] = csub(b1, mul_mi(q1));
  v[2] = cadd(b2, mul_mi(q2));
  v[3] = csub(b2, mul_mi(q2));
}

// One Stockham autosort pass of radix R over F frames of M complex points held in `buf`
// (frame-major).  Ns = product of the radices of the previous passes.  Butterfly j reads
// x[j + r*M/R], scales input r by W_{Ns*R}^{(j mod Ns)*r}, and writes y[(j/Ns)*Ns*R + j%Ns + r*Ns].
// In place: every thread keeps its butterflies in registers across the barrier.
template <int R, int NS, int M, int F, int NT>
__device__ __forceinline__ void stockham_pass(float2* buf, const float2* __restrict__ tw) {
  constexpr int MR = M / R;
  constexpr int NB = F * MR;
  constexpr int CNT = (NB + NT - 1) / NT;
  float2 v[CNT][R];
  int dst[CNT];
#pragma unroll
  for (int i = 0; i < CNT; ++i) {
    const int b = threadIdx.x + i * NT;
    dst[i] = -1;
    if (b < NB) {
      const int fr = b / MR, j = b % MR, k = j % NS;
      const int base = fr * M;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float2 a = buf[base + j + r * MR];
        if (NS > 1 && r > 0) a = cmul(a, tw[k * r * (M / (NS * R))]);
        v[i][r] = a;
      }
      dft<R>(v[i]);
      dst[i] = base + (j / NS) * NS * R + k;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < CNT; ++i) {
    if (dst[i] >= 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) buf[dst[i] + r * NS] = v[i][r];
    }
  }
  __syncthreads();
}

template <int M, int F, int NT>
__device__ __forceinline__ void fft_frames(float2* buf, const float2* __restrict__ tw);

template <>
__device__ __forceinline__ void fft_frames<256, 14, 256>(float2* buf, const float2* __restrict__ tw) {
  stockham_pass<4, 1, 256, 14, 256>(buf, tw);
  stockham_pass<4, 4, 256, 14, 256>(buf, tw);
  stockham_pass<4, 16, 256, 14, 256>(buf, tw);
  stockham_pass<4, 64, 256, 14, 256>(buf, tw);
}

template <int F, int NT>
__device__ __forceinline__ void fft320(float2* buf, const float2* __restrict__ tw) {
  stockham_pass<4, 1, 320, F, NT>(buf, tw);
  stockham_pass<4, 4, 320, F, NT>(buf, tw);
  stockham_pass<4, 16, 320, F, NT>(buf, tw);
  stockham_pass<5, 64, 320, F, NT>(buf, tw);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Untangle the packed real FFT and store |X[k]|^2 (k = 0..M) as floats over `buf`, frame
// stride M+1.  X[0] / X[M] come from the fp64 sums `dcny` instead of the fp32 FFT.
template <int M, int F, int NT>
__device__ __forceinline__ void power_spectrum(float2* buf, const float2* __restrict__ post,
                                               const double2* dcny, bool fix_dc, bool fix_nyq) {
  constexpr int NI = F * (M + 1);
  constexpr int CNT = (NI + NT - 1) / NT;
  float p[CNT];
#pragma unroll
  for (int i = 0; i < CNT; ++i) {
    const int it = threadIdx.x + i * NT;
    p[i] = 0.f;
    if (it < NI) {
      const int fr = it / (M + 1), k = it % (M + 1);
      const float2 a = buf[fr * M + (k % M)];
      const float2 bz = buf[fr * M + ((M - k) % M)];
      const float2 bc = make_float2(bz.x, -bz.y);
      const float2 e = make_float2(0.5f * (a.x + bc.x), 0.5f * (a.y + bc.y));
      const float2 o = mul_mi(make_float2(0.5f * (a.x - bc.x), 0.5f * (a.y - bc.y)));
      const float2 x = cadd(e, cmul(post[k], o));
      p[i] = x.x * x.x + x.y * x.y;
      if (k == 0 && fix_dc) p[i] = (float)(dcny[fr].x * dcny[fr].x);
      if (k == M && fix_nyq) p[i] = (float)(dcny[fr].y * dcny[fr].y);
    }
  }
  __syncthreads();
  float* pb = reinterpret_cast<float*>(buf);
#pragma unroll
  for (int i = 0; i < CNT; ++i) {
    const int it = threadIdx.x + i * NT;
    if (it < NI) pb[it] = p[i];
  }
  __syncthreads();
}

// ------------------------------------------------------------------------- per-feature loads
// Each returns the two windowed fp64 samples feeding z[n] = x[2n] + i x[2n+1] of frame gf.
struct FbankLoad {   // model_fbanks_cnn.py:21 (fp32 pre-emphasis), :36-41 (frames, Hamming)
  static constexpr int N = 512, M = 256, NFRAMES = 98;
  __device__ static __forceinline__ double emph(const float* x, int i) {
    // numpy rounds the product and the difference separately: no FMA contraction here
#pragma clang fp contract(off)
    return i == 0 ? (double)x[0] : (double)(x[i] - 0.97f * x[i - 1]);
  }
  __device__ static __forceinline__ void load(const float* x, const DeviceTables& t, int gf, int n,
                                              double& a, double& b) {
    const int m = 2 * n;
    if (m >= 400) { a = b = 0.0; return; }
    const int s = 160 * gf + m;
    a = emph(x, s) * t.hamming400[m];
    b = emph(x, s + 1) * t.hamming400[m + 1];
  }
};

struct SpecLoad {    // scipy.signal.spectrogram segments, model_spec_bgru.py:13
  static constexpr int N = 640, M = 320, NFRAMES = 49;
  __device__ static __forceinline__ void load(const float* x, const DeviceTables& t, int gf, int n,
                                              double& a, double& b) {
    const int s = 320 * gf + 2 * n;
    const float2 v = *reinterpret_cast<const float2*>(x + s);
    a = (double)v.x * t.tukey640[2 * n];
    b = (double)v.y * t.tukey640[2 * n + 1];
  }
};

// Load frames [f0, f0+F) of clip x into buf, windowed; frames past NFRAMES are zero.
template <class L, int F, int NT>
__device__ __forceinline__ void load_frames(float2* buf, double2* dcny, const float* x,
                                            const DeviceTables& t, int f0) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int fr = wave; fr < F; fr += NW) {
    const int gf = f0 + fr;
    double se = 0.0, so = 0.0;
#pragma unroll
    for (int i = 0; i < L::M / 64; ++i) {
      const int n = lane + 64 * i;
      double a = 0.0, b = 0.0;
      if (gf < L::NFRAMES) L::load(x, t, gf, n, a, b);
      buf[fr * L::M + n] = make_float2((float)a, (float)b);
      se += a;
      so += b;
    }
    se = wave_sum(se);
    so = wave_sum(so);
    if (lane == 0) dcny[fr] = make_double2(se + so, se - so);
  }
  __syncthreads();
}

// ------------------------------------------------------------------------- K2 fbank
constexpr int kFbF = 14, kFbNT = 256;
constexpr float kFbEpsDb = -313.07119549076395f;   // 20*log10(np.finfo(float).eps), :61-62

__global__ __launch_bounds__(kFbNT) void fbank_kernel(const float* __restrict__ pcm, float* __restrict__ out,
                                                      DeviceTables t) {
  __shared__ float2 buf[kFbF * 256];
  __shared__ double2 dcny[kFbF];
  const int clip = blockIdx.x;
  const float* x = pcm + (size_t)clip * kPcmLen;
  float* o = out + (size_t)clip * 98 * 120;
  for (int f0 = 0; f0 < 98; f0 += kFbF) {
    load_frames<FbankLoad, kFbF, kFbNT>(buf, dcny, x, t, f0);
    fft_frames<256, kFbF, kFbNT>(buf, t.tw256);
    power_spectrum<256, kFbF, kFbNT>(buf, t.post512, dcny, true, true);
    const float* pb = reinterpret_cast<const float*>(buf);
    for (int it = threadIdx.x; it < kFbF * 120; it += kFbNT) {
      const int fr = it / 120, m = it % 120;
      const int cnt = t.fb_cnt[m];
      float acc = 0.f;
      if (cnt > 0) {
        const int lo = t.fb_lo[m], off = t.fb_off[m];
        const float* p = pb + fr * 257 + lo;
        for (int c = 0; c < cnt; ++c) acc = fmaf(t.fb_w[off + c], p[c], acc);
      }
      // |rfft|^2 / NFFT (:44): the 1/512 is an exact power of two, applied after the sum
      acc *= (1.0f / 512.0f);
      o[(f0 + fr) * 120 + m] = acc == 0.f ? kFbEpsDb : 20.0f * log10f(acc);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------- K3 spectrogram
constexpr int kSpF = 7, kSpNT = 256;

__global__ __launch_bounds__(kSpNT) void spec_kernel(const float* __restrict__ pcm, float* __restrict__ out,
                                                     int transposed, float scale, DeviceTables t) {
  __shared__ float2 buf[kSpF * 320];
  __shared__ double2 dcny[kSpF];
  const int clip = blockIdx.x;
  const float* x = pcm + (size_t)clip * kPcmLen;
  float* o = out + (size_t)clip * 49 * 321;
  for (int f0 = 0; f0 < 49; f0 += kSpF) {
    load_frames<SpecLoad, kSpF, kSpNT>(buf, dcny, x, t, f0);
    fft320<kSpF, kSpNT>(buf, t.tw320);
    power_spectrum<320, kSpF, kSpNT>(buf, t.post640, dcny, true, true);
    const float* pb = reinterpret_cast<const float*>(buf);
    for (int it = threadIdx.x; it < kSpF * 321; it += kSpNT) {
      const int fr = it / 321, k = it % 321;
      float v = pb[it] * scale;
      if (k > 0 && k < 320) v *= 2.0f;                 // one-sided, DC/Nyquist not doubled
      v = logf(__fadd_rn(v, 1e-10f));                  // model_spec_bgru.py:14
      const int f = f0 + fr;
      if (transposed) o[f * 321 + k] = v; else o[k * 49 + f] = v;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------- register FFT (v2)
// N = 640 real = 320 complex, factored 320 = 16 (j) x 20 (i): n = j + 16 i, k = k1 + 20 k2.
//   pass A (lane per (frame, j), 16 lanes / frame): 20-point DFT over i in registers,
//                                                   then twiddle W320^(j k1)
//   LDS transpose (row pitch 17 complex: conflict-free ds_read_b64 / ds_write_b64)
//   pass B (lane per (frame, k1), 20 lanes / frame): 16-point DFT over j in registers
// A wave processes 3 frames at a time (48 lanes in pass A, 60 in pass B); no workgroup barrier
// is needed inside the frame loop (each wave owns its LDS slices).
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v2f cm2(v2f a, v2f b) { return v2f{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ v2f mi2(v2f a) { return v2f{a.y, -a.x}; }   // -i * a

__device__ constexpr float kW20[4][5][2] = {
  {{1.f, 0.f}, {1.f, 0.f}, {1.f, 0.f}, {1.f, 0.f}, {1.f, 0.f}},
  {{1.f, 0.f}, {9.510565163e-01f, -3.090169944e-01f}, {8.090169944e-01f, -5.877852523e-01f},
   {5.877852523e-01f, -8.090169944e-01f}, {3.090169944e-01f, -9.510565163e-01f}},
  {{1.f, 0.f}, {8.090169944e-01f, -5.877852523e-01f}, {3.090169944e-01f, -9.510565163e-01f},
   {-3.090169944e-01f, -9.510565163e-01f}, {-8.090169944e-01f, -5.877852523e-01f}},
  {{1.f, 0.f}, {5.877852523e-01f, -8.090169944e-01f}, {-3.090169944e-01f, -9.510565163e-01f},
   {-9.510565163e-01f, -3.090169944e-01f}, {-8.090169944e-01f, 5.877852523e-01f}}};
__device__ constexpr float kW16[4][4][2] = {
  {{1.f, 0.f}, {1.f, 0.f}, {1.f, 0.f}, {1.f, 0.f}},
  {{1.f, 0.f}, {9.238795325e-01f, -3.826834324e-01f}, {7.071067812e-01f, -7.071067812e-01f},
   {3.826834324e-01f, -9.238795325e-01f}},
  {{1.f, 0.f}, {7.071067812e-01f, -7.071067812e-01f}, {0.f, -1.f}, {-7.071067812e-01f, -7.071067812e-01f}},
  {{1.f, 0.f}, {3.826834324e-01f, -9.238795325e-01f}, {-7.071067812e-01f, -7.071067812e-01f},
   {-9.238795325e-01f, 3.826834324e-01f}}};

__device__ __forceinline__ void dft4v(v2f& a0, v2f& a1, v2f& a2, v2f& a3) {
  const v2f s02 = a0 + a2, d02 = a0 - a2, s13 = a1 + a3, d13 = mi2(a1 - a3);
  a0 = s02 + s13;
  a2 = s02 - s13;
  a1 = d02 + d13;
  a3 = d02 - d13;
}

__device__ __forceinline__ void dft5v(v2f& a0, v2f& a1, v2f& a2, v2f& a3, v2f& a4) {
  constexpr float c1 = 0.30901699437494745f, c2 = -0.8090169943749473f;
  constexpr float s1 = 0.9510565162951535f, s2 = 0.5877852522924732f;
  const v2f t1 = a1 + a4, t2 = a2 + a3, t3 = a1 - a4, t4 = a2 - a3;
  const v2f b1 = a0 + c1 * t1 + c2 * t2, b2 = a0 + c2 * t1 + c1 * t2;
  const v2f q1 = s1 * t3 + s2 * t4, q2 = s2 * t3 - s1 * t4;
  a0 = a0 + t1 + t2;
  a1 = b1 + mi2(q1);
  a4 = b1 - mi2(q1);
  a2 = b2 + mi2(q2);
  a3 = b2 - mi2(q2);
}

// in-place 20-point forward DFT, natural order in and out (i = 4p + q, k = k1 + 5 k2)
__device__ __forceinline__ void dft20v(v2f (&a)[20]) {
  v2f b[4][5];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v2f t0 = a[q], t1 = a[4 + q], t2 = a[8 + q], t3 = a[12 + q], t4 = a[16 + q];
    dft5v(t0, t1, t2, t3, t4);
    b[q][0] = t0; b[q][1] = t1; b[q][2] = t2; b[q][3] = t3; b[q][4] = t4;
#pragma unroll
    for (int k1 = 1; k1 < 5; ++k1)
      if (q > 0) b[q][k1] = cm2(b[q][k1], v2f{kW20[q][k1][0], kW20[q][k1][1]});
  }
#pragma unroll
  for (int k1 = 0; k1 < 5; ++k1) {
    v2f u0 = b[0][k1], u1 = b[1][k1], u2 = b[2][k1], u3 = b[3][k1];
    dft4v(u0, u1, u2, u3);
    a[k1] = u0; a[k1 + 5] = u1; a[k1 + 10] = u2; a[k1 + 15] = u3;
  }
}

// in-place 16-point forward DFT (j = 4p + q, k = k1 + 4 k2)
__device__ __forceinline__ void dft16v(v2f (&a)[16]) {
  v2f b[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v2f t0 = a[q], t1 = a[4 + q], t2 = a[8 + q], t3 = a[12 + q];
    dft4v(t0, t1, t2, t3);
    b[q][0] = t0; b[q][1] = t1; b[q][2] = t2; b[q][3] = t3;
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1)
      if (q > 0) b[q][k1] = cm2(b[q][k1], v2f{kW16[q][k1][0], kW16[q][k1][1]});
  }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    v2f u0 = b[0][k1], u1 = b[1][k1], u2 = b[2][k1], u3 = b[3][k1];
    dft4v(u0, u1, u2, u3);
    a[k1] = u0; a[k1 + 4] = u1; a[k1 + 8] = u2; a[k1 + 12] = u3;
  }
}

__device__ __forceinline__ void wave_lds_fence() {
  // orders this wave's LDS writes before its later LDS reads (no workgroup barrier needed)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave computes the 320-point complex FFT of 3 frames whose packed inputs z[n] it supplies
// through `a` (pass-A lanes, frame = lane >> 4, j = lane & 15, a[i] = z[j + 16 i]); on return the
// natural-order spectra are in xs[f * 320 + k] (f < 3).  tb = this wave's transpose slice.
__device__ __forceinline__ void fft320x3(v2f (&a)[20], const v2f (&tw)[20], v2f* tb, v2f* xs, int lane) {
  const int fa = lane >> 4, j = lane & 15;
  dft20v(a);
  if (fa < 3) {
#pragma unroll
    for (int k1 = 0; k1 < 20; ++k1) tb[fa * 340 + k1 * 17 + j] = k1 ? cm2(a[k1], tw[k1]) : a[0];
  }
  wave_lds_fence();
  const int fb = lane / 20, k1 = lane % 20;
  v2f b[16];
  if (fb < 3) {
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) b[jj] = tb[fb * 340 + k1 * 17 + jj];
  }
  dft16v(b);
  if (fb < 3) {
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) xs[fb * 320 + k1 + 20 * k2] = b[k2];
  }
  wave_lds_fence();
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
        const float v0 = s0 > 1e-10f ? 10.0f * log10f(s0) : -100.0f;
        const float v1 = s1 > 1e-10f ? 10.0f * log10f(s1) : -100.0f;
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
  const DeviceTables* t = nullptr;
  if (int rc = srk::get_tables(&t)) return rc;
  srk::ProfScope prof("fbank", srk::as_stream(stream), 111040.0 * (double)n_clips);   // 64000 in + 47040 out B/clip
  hipLaunchKernelGGL(srk::fbank_kernel, dim3((unsigned)n_clips), dim3(srk::kFbNT), 0, srk::as_stream(stream),
                     pcm, out, *t);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_spec_fwd(const float* pcm, int64_t n_clips, float* out, int transposed, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n_clips >= 0 && n_clips <= INT32_MAX, SRK_ERR_INVALID, "srk_spec_fwd: bad n_clips");
  if (n_clips == 0) return SRK_OK;
  SRK_REQUIRE(pcm && out, SRK_ERR_INVALID, "srk_spec_fwd: null pointer");
  const DeviceTables* t = nullptr;
  if (int rc = srk::get_tables(&t)) return rc;
  srk::ProfScope prof("spec", srk::as_stream(stream), 126916.0 * (double)n_clips);    // 64000 + 62916 B/clip
  hipLaunchKernelGGL(srk::spec_kernel, dim3((unsigned)n_clips), dim3(srk::kSpNT), 0, srk::as_stream(stream),
                     pcm, out, transposed ? 1 : 0, (float)t->spec_scale, *t);
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
