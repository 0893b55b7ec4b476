// K12 batched pitch_shifting (dataset.py:225-235): librosa.effects.pitch_shift(y, sr = 16000, n_steps)
// of the training-mode augmentation, for every clip of a batch whose draw chose it, in ONE launch.
//
// The algorithm is librosa 0.6's (parity unpinned: librosa / resampy are absent; oracle/pitch.py
// restates it with the dtypes those versions use, and states the choices):
//   rate = 2^(-n_steps / 12)
//   time_stretch: STFT (n_fft 2048, hop 512, periodic Hann, centred, reflect padding; complex64 values
//                 of a float64 FFT) -> phase vocoder (float32 magnitudes / phases, float64 phase
//                 advance, float32 phase accumulator) -> inverse STFT (float64 inverse FFT, Hann,
//                 overlap-add in frame order, window sum-square normalisation, centre trim)
//                 -> fix_length(round(16000 / rate))
//   resample:     resampy 'kaiser_best' (64 zero crossings x 512 taps, Kaiser beta 14.7697, rolloff
//                 0.9476) from 16000 / rate to 16000 Hz, resampy's interpolation loop in float64
//   int16 truncation toward zero -> float32 (Dataset items are int16-valued float32).
//
// One workgroup of 1024 threads per shifted clip; the clip's stages run back to back with workgroup
// barriers, the intermediate images in a caller-supplied HBM workspace (srk_pitch_workspace_bytes):
// magnitude / phase of the 32 STFT columns, the vocoder's complex64 columns, the windowed inverse
// frames and the stretched signal — ~1.2 MB per clip, L2-resident while the workgroup runs.
// FFTs: 2048-point complex radix-2 in LDS (fp64, 11 stages of one butterfly per thread), two real
// frames per transform (x_a + i x_b forward; two Hermitian spectra as A + i B inverse).
// Transcendentals in float64, rounded to float32 where librosa holds float32 (oracle/pitch.py).
#include <cmath>
#include <mutex>
#include <vector>

#include "srk_internal.h"

namespace srk {
namespace {

constexpr int kLen = 16000;
constexpr int kNfft = 2048;
constexpr int kHop = 512;
constexpr int kBins = kNfft / 2 + 1;        // 1025
constexpr int kCols = 1 + kLen / kHop;      // 32 STFT columns (1 + (16000 + 2048 - 2048) // 512)
constexpr int kColsPad = kCols + 2;         // the vocoder's two zero columns
constexpr int kMaxSteps = 40;               // ceil(32 / rate) <= 36 for |n_steps| <= 2
constexpr int kMaxStretch = kHop * kMaxSteps;
constexpr int kThreads = 1024;
constexpr int kNumZeros = 64, kPrecision = 9, kNumTable = 1 << kPrecision;
constexpr int kWin = kNumZeros * kNumTable + 1;   // 32769 taps of the filter's right wing
constexpr int kLevels = 4;                        // n_steps = -2, -1, 1, 2
constexpr double kBeta = 14.769656459379492, kRolloff = 0.9475937167399596;

struct Level {
  double rate;          // 2 ** (-n_steps / 12)
  int steps;            // phase-vocoder output columns = len(arange(0, 32, rate))
  int stretch_len;      // int(round(16000 / rate)) (fix_length of time_stretch)
  double sample_ratio;  // 16000 / (16000 / rate) (resampy's sr_new / sr_orig)
  double scale;         // min(1, sample_ratio)
  int index_step;       // int(scale * 512)
  int n_out;            // int(stretch_len * sample_ratio) (resampy output length)
  int n_keep;           // min(n_out, ceil(stretch_len * ratio), 16000): samples the two fix_lengths keep
  const double* win;    // interp_win (scaled by sample_ratio when < 1), [kWin]
  const double* delta;  // interp_delta, [kWin]
  const double* treg;   // the time register before each output, accumulated as resampy does, [16000]
};

struct PitchTables {
  bool ready = false;
  double2* tw = nullptr;    // exp(-2 pi i k / 2048), k < 1024
  double* hann = nullptr;   // scipy get_window('hann', 2048, fftbins=True)
  Level lv[kLevels];
};

constexpr int kMaxDevices = 64;
PitchTables g_pt[kMaxDevices];
std::mutex g_pt_mutex;

std::vector<double> np_linspace(double a, double b, int n) {   // numpy.linspace semantics
  std::vector<double> y(n);
  const double step = (b - a) / (n - 1);
  for (int i = 0; i < n; ++i) y[i] = i * step + a;
  y[n - 1] = b;
  return y;
}

double bessel_i0(double x) {   // power series, relative error ~1e-16 for |x| <= 20
  const double q = 0.25 * x * x;
  double term = 1.0, sum = 1.0;
  for (int k = 1; k < 200 && term > 1e-18 * sum; ++k) {
    term *= q / ((double)k * (double)k);
    sum += term;
  }
  return sum;
}

template <class T>
int upload_vec(T** dst, const std::vector<T>& v) {
  SRK_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(dst), v.size() * sizeof(T)));
  SRK_CHECK_HIP(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return SRK_OK;
}

int build_pitch_tables(PitchTables& t) {
  int rc;
  std::vector<double2> tw(kNfft / 2);
  for (int k = 0; k < kNfft / 2; ++k) {
    const double a = -2.0 * M_PI * (double)k / (double)kNfft;
    tw[k] = make_double2(std::cos(a), std::sin(a));
  }
  if ((rc = upload_vec(&t.tw, tw))) return rc;
  {  // scipy general_cosine(2049, [0.5, 0.5])[:2048]: 0.5 + 0.5 cos(linspace(-pi, pi, 2049))
    const std::vector<double> fac = np_linspace(-M_PI, M_PI, kNfft + 1);
    std::vector<double> h(kNfft);
    for (int n = 0; n < kNfft; ++n) h[n] = 0.5 + 0.5 * std::cos(fac[n]);
    if ((rc = upload_vec(&t.hann, h))) return rc;
  }
  // resampy sinc_window(num_zeros = 64, precision = 9, kaiser(beta), rolloff): the right wing
  const int n = kNumTable * kNumZeros;
  const std::vector<double> xs = np_linspace(0.0, (double)kNumZeros, n + 1);
  std::vector<double> base(kWin);
  const double i0b = bessel_i0(kBeta);
  const double alpha = (double)(2 * n) / 2.0;   // kaiser(2n + 1): alpha = (M - 1) / 2
  for (int i = 0; i < kWin; ++i) {
    const double u = kRolloff * xs[i];
    const double y = M_PI * (u == 0.0 ? 1.0e-20 : u);   // numpy.sinc
    const double sinc = kRolloff * (std::sin(y) / y);
    const double r = ((double)(n + i) - alpha) / alpha;
    const double taper = bessel_i0(kBeta * std::sqrt(1.0 - r * r)) / i0b;
    base[i] = taper * sinc;
  }
  static const int kSteps[kLevels] = {-2, -1, 1, 2};
  for (int l = 0; l < kLevels; ++l) {
    Level& L = t.lv[l];
    L.rate = std::pow(2.0, -(double)kSteps[l] / 12.0);
    L.steps = (int)std::ceil((double)kCols / L.rate);   // len(np.arange(0, 32, rate))
    SRK_REQUIRE(L.steps <= kMaxSteps, SRK_ERR_INTERNAL, "pitch: %d vocoder steps", L.steps);
    L.stretch_len = (int)std::nearbyint((double)kLen / L.rate);   // round half even
    const double sr_orig = 16000.0 / L.rate;
    L.sample_ratio = 16000.0 / sr_orig;
    L.scale = std::min(1.0, L.sample_ratio);
    L.index_step = (int)(L.scale * kNumTable);
    L.n_out = (int)((double)L.stretch_len * L.sample_ratio);
    const int n_samples = (int)std::ceil((double)L.stretch_len * L.sample_ratio);
    L.n_keep = std::min(std::min(L.n_out, n_samples), kLen);
    std::vector<double> w(base), d(kWin, 0.0), tr(kLen);
    if (L.sample_ratio < 1.0)
      for (double& v : w) v *= L.sample_ratio;
    for (int i = 0; i + 1 < kWin; ++i) d[i] = w[i + 1] - w[i];
    double acc = 0.0;
    const double inc = 1.0 / L.sample_ratio;
    for (int i = 0; i < kLen; ++i) {
      tr[i] = acc;
      acc += inc;
    }
    double *pw, *pd, *ptr;
    if ((rc = upload_vec(&pw, w)) || (rc = upload_vec(&pd, d)) || (rc = upload_vec(&ptr, tr))) return rc;
    L.win = pw;
    L.delta = pd;
    L.treg = ptr;
  }
  t.ready = true;
  return SRK_OK;
}

int get_pitch_tables(const PitchTables** out) {
  int dev = 0;
  SRK_CHECK_HIP(hipGetDevice(&dev));
  SRK_REQUIRE(dev >= 0 && dev < kMaxDevices, SRK_ERR_INVALID, "device %d out of range", dev);
  PitchTables& t = g_pt[dev];
  if (!t.ready) {
    std::lock_guard<std::mutex> lk(g_pt_mutex);
    if (!t.ready) {
      int rc = build_pitch_tables(t);
      if (rc) return rc;
    }
  }
  *out = &t;
  return SRK_OK;
}

// Workspace of one clip, in doubles (16-B aligned sections)
constexpr size_t kWsMag = 0;                                            // float [34][1025] (as doubles: /2)
constexpr size_t kWsAng = kWsMag + (size_t)kColsPad * kBins / 2 + 8;    // float [34][1025]
constexpr size_t kWsCol = kWsAng + (size_t)kColsPad * kBins / 2 + 8;    // float2 [40][1025]
constexpr size_t kWsFrm = kWsCol + (size_t)kMaxSteps * kBins + 8;       // double [40][2048]
constexpr size_t kWsY = kWsFrm + (size_t)kMaxSteps * kNfft;             // double [kMaxStretch + 2048]
constexpr size_t kWsPerClip = kWsY + (size_t)kMaxStretch + kNfft;

__device__ __forceinline__ int bitrev11(int i) { return (int)(__builtin_bitreverse32((unsigned)i) >> 21); }

// in-place forward 2048-point FFT of buf (loaded in bit-reversed order), 1024 threads
__device__ void fft2048(double2* buf, const double2* __restrict__ tw) {
#pragma clang fp contract(off)
  const int j = threadIdx.x;
#pragma unroll 1
  for (int s = 0; s < 11; ++s) {
    const int half = 1 << s;
    const int pos = j & (half - 1);
    const int i0 = ((j >> s) << (s + 1)) + pos, i1 = i0 + half;
    const double2 w = tw[pos << (10 - s)];
    const double2 a = buf[i0], b = buf[i1];
    const double2 bw = make_double2(b.x * w.x - b.y * w.y, b.x * w.y + b.y * w.x);
    buf[i0] = make_double2(a.x + bw.x, a.y + bw.y);
    buf[i1] = make_double2(a.x - bw.x, a.y - bw.y);
    __syncthreads();
  }
}

__device__ __forceinline__ int reflect(int s) { return s < 0 ? -s : (s > kLen - 1 ? 2 * (kLen - 1) - s : s); }

__global__ __launch_bounds__(kThreads) void pitch_shift_kernel(const int16_t* __restrict__ pcm,
                                                               const int32_t* __restrict__ clip_idx,
                                                               const int32_t* __restrict__ level_idx,
                                                               float* __restrict__ out, double* __restrict__ ws_all,
                                                               PitchTables t) {
#pragma clang fp contract(off)
  __shared__ double2 buf[kNfft];
  __shared__ double2 s_tw[kNfft / 2];
  __shared__ double s_hann[kNfft];
  const int tid = threadIdx.x;
  const int64_t clip = clip_idx[blockIdx.x];
  const int li = level_idx[blockIdx.x];
  const Level L = t.lv[li];
  const int16_t* x = pcm + clip * kLen;
  double* ws = ws_all + (size_t)blockIdx.x * kWsPerClip;
  float* mag = reinterpret_cast<float*>(ws + kWsMag);
  float* ang = reinterpret_cast<float*>(ws + kWsAng);
  float2* col = reinterpret_cast<float2*>(ws + kWsCol);
  double* frm = ws + kWsFrm;
  double* ys = ws + kWsY;
  s_tw[tid] = t.tw[tid];
  s_hann[tid] = t.hann[tid];
  s_hann[tid + 1024] = t.hann[tid + 1024];
  __syncthreads();

  // ---- STFT: two frames per transform, z = w * (frame a + i frame b); bins -> |X| and angle (float32)
  for (int p = 0; p < kCols / 2; ++p) {
    for (int i = tid; i < kNfft; i += kThreads) {
      const double w = s_hann[i];
      const double a = (double)x[reflect(kHop * 2 * p + i - kNfft / 2)];
      const double b = (double)x[reflect(kHop * (2 * p + 1) + i - kNfft / 2)];
      buf[bitrev11(i)] = make_double2(w * a, w * b);
    }
    __syncthreads();
    fft2048(buf, s_tw);
    for (int k = tid; k < kBins; k += kThreads) {
      const double2 zk = buf[k], zn = buf[(kNfft - k) & (kNfft - 1)];
      // X_a = (Z[k] + conj Z[N-k]) / 2, X_b = (Z[k] - conj Z[N-k]) / 2i; complex64 values
      const float ar = (float)(0.5 * (zk.x + zn.x)), ai = (float)(0.5 * (zk.y - zn.y));
      const float br = (float)(0.5 * (zk.y + zn.y)), bi = (float)(0.5 * (zn.x - zk.x));
      const int ca = 2 * p, cb = 2 * p + 1;
      mag[ca * kBins + k] = (float)hypot((double)ar, (double)ai);
      ang[ca * kBins + k] = (float)atan2((double)ai, (double)ar);
      mag[cb * kBins + k] = (float)hypot((double)br, (double)bi);
      ang[cb * kBins + k] = (float)atan2((double)bi, (double)br);
    }
    __syncthreads();
  }
  for (int k = tid; k < 2 * kBins; k += kThreads) {   // the two zero columns of np.pad
    mag[kCols * kBins + k] = 0.f;
    ang[kCols * kBins + k] = 0.f;
  }
  __syncthreads();

  // ---- phase vocoder: one bin per thread, the steps in order
  for (int k = tid; k < kBins; k += kThreads) {
    const double phi_adv = k == kBins - 1 ? M_PI * kHop : (double)k * (M_PI * kHop / (double)(kBins - 1));
    float phase = ang[k];
    for (int tt = 0; tt < L.steps; ++tt) {
      const double step = (double)tt * L.rate;
      const int s = (int)step;
      const double alpha = fmod(step, 1.0);
      const float m0 = mag[s * kBins + k], m1 = mag[(s + 1) * kBins + k];
      const float m = (float)(1.0 - alpha) * m0 + (float)alpha * m1;
      const double ph = (double)phase;
      col[tt * kBins + k] = make_float2(m * (float)cos(ph), m * (float)sin(ph));
      double dphase = (double)(ang[(s + 1) * kBins + k] - ang[s * kBins + k]) - phi_adv;
      dphase = dphase - 2.0 * M_PI * rint(dphase / (2.0 * M_PI));
      phase = (float)((double)phase + (phi_adv + dphase));
    }
  }
  __syncthreads();

  // ---- inverse STFT: two columns per transform (A + i B, A and B Hermitian), windowed frames
  for (int c0 = 0; c0 < L.steps; c0 += 2) {
    const bool two = c0 + 1 < L.steps;
    for (int i = tid; i < kNfft; i += kThreads) {
      // full spectra: k <= 1024 the column (imaginary part of bins 0 and 1024 dropped: it only feeds
      // the inverse's imaginary part, which istft discards), k > 1024 conj(col[2048 - k]);
      // conj(A + i B) loaded: the inverse is conj(FFT(conj(.))) / N
      const int k = i <= kNfft / 2 ? i : kNfft - i;
      const float sg = i <= kNfft / 2 ? 1.f : -1.f;
      const bool real_bin = (k == 0) || (k == kNfft / 2);
      const float2 a = col[c0 * kBins + k];
      const float2 b = two ? col[(c0 + 1) * kBins + k] : make_float2(0.f, 0.f);
      const double are = a.x, aim = real_bin ? 0.0 : (double)(sg * a.y);
      const double bre = b.x, bim = real_bin ? 0.0 : (double)(sg * b.y);
      // Z = A + i B = (are - bim) + i (aim + bre); loaded conjugated
      buf[bitrev11(i)] = make_double2(are - bim, -(aim + bre));
    }
    __syncthreads();
    fft2048(buf, s_tw);
    for (int n = tid; n < kNfft; n += kThreads) {
      const double2 z = buf[n];   // conj(z) / N = a + i b
      frm[c0 * kNfft + n] = s_hann[n] * (z.x / (double)kNfft);
      if (two) frm[(c0 + 1) * kNfft + n] = s_hann[n] * (-z.y / (double)kNfft);
    }
    __syncthreads();
  }

  // ---- overlap-add in frame order, window sum-square normalisation, centre trim, fix_length
  const int body = kHop * (L.steps - 1);   // len(y) after trimming n_fft / 2 at each end
  for (int j = tid; j < L.stretch_len; j += kThreads) {
    double v = 0.0;
    if (j < body) {
      const int sp = j + kNfft / 2;
      const int i_lo = sp >= kNfft ? (sp - kNfft) / kHop + 1 : 0;
      const int i_hi = min(sp / kHop, L.steps - 1);
      double y = 0.0, wss = 0.0;
      for (int i = i_lo; i <= i_hi; ++i) {
        const int o = sp - kHop * i;
        y = y + frm[i * kNfft + o];
        const double h = s_hann[o];
        wss = wss + h * h;
      }
      v = wss > 2.2250738585072014e-308 ? y / wss : y;
    }
    ys[j] = v;
  }
  __syncthreads();

  // ---- resampy resample_f: left wing then right wing, interpolated filter taps, float64
  float* dst = out + clip * kLen;
  const int n_orig = L.stretch_len;
  for (int tt = tid; tt < kLen; tt += kThreads) {
    double acc = 0.0;
    if (tt < L.n_keep) {
      const double tr = L.treg[tt];
      const int n = (int)tr;
      double frac = L.scale * (tr - (double)n);
      double index_frac = frac * (double)kNumTable;
      int offset = (int)index_frac;
      double eta = index_frac - (double)offset;
      const int i_max = min(n + 1, (kWin - offset) / L.index_step);
      for (int i = 0; i < i_max; ++i) {
        const int q = offset + i * L.index_step;
        const double weight = L.win[q] + eta * L.delta[q];
        acc = acc + weight * ys[n - i];
      }
      frac = L.scale - frac;
      index_frac = frac * (double)kNumTable;
      offset = (int)index_frac;
      eta = index_frac - (double)offset;
      const int k_max = min(n_orig - n - 1, (kWin - offset) / L.index_step);
      for (int k = 0; k < k_max; ++k) {
        const int q = offset + k * L.index_step;
        const double weight = L.win[q] + eta * L.delta[q];
        acc = acc + weight * ys[n + k + 1];
      }
    }
    dst[tt] = (float)(int16_t)(int)acc;
  }
}

}  // namespace
}  // namespace srk

extern "C" int64_t srk_pitch_workspace_bytes(int64_t n_shift) {
  return n_shift <= 0 ? 0 : n_shift * (int64_t)(srk::kWsPerClip * sizeof(double));
}

extern "C" int srk_pitch_shift(const int16_t* pcm, int64_t n_clips, const int32_t* clip_idx,
                               const int32_t* level_idx, int64_t n_shift, float* out, void* workspace,
                               int64_t workspace_bytes, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(n_clips >= 0 && n_clips < ((int64_t)1 << 31) && n_shift >= 0 && n_shift <= n_clips, SRK_ERR_INVALID,
              "srk_pitch_shift: bad n_clips / n_shift");
  if (n_shift == 0) return SRK_OK;
  SRK_REQUIRE(pcm && clip_idx && level_idx && out && workspace, SRK_ERR_INVALID, "srk_pitch_shift: null pointer");
  SRK_REQUIRE(workspace_bytes >= srk_pitch_workspace_bytes(n_shift), SRK_ERR_INVALID,
              "srk_pitch_shift: workspace of %lld bytes, %lld needed", (long long)workspace_bytes,
              (long long)srk_pitch_workspace_bytes(n_shift));
  SRK_REQUIRE((uintptr_t)workspace % 16 == 0, SRK_ERR_INVALID, "srk_pitch_shift: workspace must be 16-byte aligned");
  const srk::PitchTables* t = nullptr;
  int rc = srk::get_pitch_tables(&t);
  if (rc) return rc;
  hipStream_t s = srk::as_stream(stream);
  srk::ProfScope prof("pitch_shift", s, 96000.0 * (double)n_shift);   // 32000 in + 64000 out per clip
  hipLaunchKernelGGL(srk::pitch_shift_kernel, dim3((unsigned)n_shift), dim3(srk::kThreads), 0, s, pcm, clip_idx,
                     level_idx, out, static_cast<double*>(workspace), *t);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}
