// libsrk runtime: error reporting, per-device constant tables, srk_init.
//
// The tables are built on the host in double precision from the same closed forms the
// reference evaluates with numpy/scipy/librosa, then uploaded once per device:
//  * fbank triangles       models/model_fbanks_cnn.py:46-59 (rebuilt per call there)
//  * Slaney mel (norm=1)   librosa.filters.mel as called by model_mfcc_bgru.py:13
//  * DCT-II ortho [:13]    librosa.filters.dct / scipy.fftpack.dct(norm='ortho')
//  * windows               np.hamming(400) (model_fbanks_cnn.py:41), periodic Hann(640)
//                          (librosa stft), periodic Tukey(640, 0.25) (scipy spectrogram)
#include <atomic>
#include <functional>
#include <cmath>
#include <cstdarg>
#include <mutex>
#include <vector>

#include "gru_internal.h"
#include "srk_internal.h"

namespace srk {

int g_opt_gru_persistent = 1;
int g_opt_gemm16_kernel = 0;
int g_opt_conv16_sources = 1;
int g_opt_conv_fused_db = 1;
int g_opt_conv_unpool_gather = 1;
int g_opt_conv_tile = 128;
int g_opt_conv_ring = 0x77;
int g_opt_conv_unpool16 = 1;
int g_opt_conv_colsum16 = 1;
int g_opt_conv_ring_qs = 6;
int g_opt_conv_fast16 = 1;
int g_opt_conv_row16 = 1;
int g_opt_conv_row32 = 1;
int g_opt_conv_fw_gemm = 1;
int g_opt_conv_row16_dgrad = 2;
int g_opt_bn_tree = 0;
int g_opt_mfcc_variant = 3;
int g_opt_gemm_streamk = 1;
int g_opt_gemm32_kernel = 0;
static std::atomic<int> g_opt_matmul_prec{kPrecF32};
thread_local int t_prec_override = -1;
int matmul_prec() { return t_prec_override >= 0 ? t_prec_override : g_opt_matmul_prec.load(std::memory_order_relaxed); }
int g_opt_conv_fwd_fp32 = 0;
unsigned long long* g_opt_gru_trace = nullptr;
unsigned g_opt_gru_spin_limit = 0;
int g_opt_gru_xcd_local = 1;
int g_opt_gru_lp2 = 1;
int g_opt_gru_lp_wide = 1;
int g_opt_gru_dc = 1;
unsigned g_opt_gru_dc_offset = 200;
int g_opt_gru_fast_cell = 1;
int g_opt_gru_dc_prio = 0;
int g_opt_gru_dwhh_fused = 1;
int g_opt_gru_fwd_worker = 0;
int g_opt_gru_dwhh_batched = 1;
int g_opt_gemm_skinny = 1;
std::atomic<int64_t> g_scratch_gen{0};

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

namespace {

constexpr int kMaxDevices = 64;
DeviceTables g_tables[kMaxDevices];
std::mutex g_mutex;

template <class T>
int upload(T** dst, const std::vector<T>& src) {
  SRK_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(dst), src.size() * sizeof(T)));
  SRK_CHECK_HIP(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return SRK_OK;
}

std::vector<double> linspace(double a, double b, int n) {   // numpy.linspace semantics
  std::vector<double> y(n);
  const double step = (b - a) / (n - 1);
  for (int i = 0; i < n; ++i) y[i] = i * step + a;
  y[n - 1] = b;
  return y;
}

std::vector<float2> twiddles(int m, int count) {
  std::vector<float2> t(count);
  for (int k = 0; k < count; ++k) {
    const double a = -2.0 * M_PI * (double)k / (double)m;
    t[k] = make_float2((float)std::cos(a), (float)std::sin(a));
  }
  return t;
}

// Dense [nf][nbins] -> fixed-width windows: lo[m] (clamped so lo + width <= nbins) and
// w[m][q] = dense[m][lo + q] (zero outside the filter).  Every filter here spans <= 15 bins.
int to_windows(const std::vector<double>& w, int nf, int nbins, int width, std::vector<int>& lo,
               std::vector<float>& vals) {
  lo.assign(nf, 0);
  vals.assign((size_t)nf * width, 0.f);
  for (int m = 0; m < nf; ++m) {
    int first = -1, last = -1;
    for (int k = 0; k < nbins; ++k)
      if (w[(size_t)m * nbins + k] != 0.0) { if (first < 0) first = k; last = k; }
    if (first < 0) continue;
    SRK_REQUIRE(last - first + 1 <= width, SRK_ERR_INTERNAL, "filter %d wider than %d bins", m, width);
    const int l = std::min(first, nbins - width);
    lo[m] = l;
    for (int k = first; k <= last; ++k) vals[(size_t)m * width + (k - l)] = (float)w[(size_t)m * nbins + k];
  }
  return SRK_OK;
}

// Dense [nf][nbins] matrix -> CSR by filter (each filter is one contiguous run of bins).
void to_csr(const std::vector<double>& w, int nf, int nbins, std::vector<int>& lo,
            std::vector<int>& cnt, std::vector<int>& off, std::vector<float>& vals) {
  lo.assign(nf, 0); cnt.assign(nf, 0); off.assign(nf, 0); vals.clear();
  for (int m = 0; m < nf; ++m) {
    int first = -1, last = -1;
    for (int k = 0; k < nbins; ++k)
      if (w[(size_t)m * nbins + k] != 0.0) { if (first < 0) first = k; last = k; }
    off[m] = (int)vals.size();
    if (first < 0) continue;
    lo[m] = first; cnt[m] = last - first + 1;
    for (int k = first; k <= last; ++k) vals.push_back((float)w[(size_t)m * nbins + k]);
  }
}

// Dense [nf][nbins] -> lane pairs (filter l, filter nf-1-l), l < ceil(nf/2): meta {lo_a, cnt_a,
// lo_b, cnt_b} and the two weight runs back to back, zero padded to `taps`.
int to_pairs(const std::vector<double>& w, int nf, int nbins, int taps, std::vector<int4>& meta,
             std::vector<float>& vals) {
  const int np = (nf + 1) / 2;
  meta.assign(np, int4{0, 0, 0, 0});
  vals.assign((size_t)np * taps, 0.f);
  auto run = [&](int m, int& lo, int& cnt) {
    int first = -1, last = -1;
    for (int k = 0; k < nbins; ++k)
      if (w[(size_t)m * nbins + k] != 0.0) { if (first < 0) first = k; last = k; }
    lo = first < 0 ? 0 : first;
    cnt = first < 0 ? 0 : last - first + 1;
  };
  for (int l = 0; l < np; ++l) {
    int la, ca, lb = 0, cb = 0;
    run(l, la, ca);
    if (nf - 1 - l != l) run(nf - 1 - l, lb, cb);
    SRK_REQUIRE(ca + cb <= taps, SRK_ERR_INTERNAL, "filter pair %d spans %d > %d taps", l, ca + cb, taps);
    meta[l] = int4{la, ca, lb, cb};
    for (int q = 0; q < ca; ++q) vals[(size_t)l * taps + q] = (float)w[(size_t)l * nbins + la + q];
    for (int q = 0; q < cb; ++q) vals[(size_t)l * taps + ca + q] = (float)w[(size_t)(nf - 1 - l) * nbins + lb + q];
  }
  return SRK_OK;
}

// models/model_fbanks_cnn.py:46-59
std::vector<double> fbank_matrix() {
  const int nfilt = 120, nfft = 512, sr = 16000, nb = nfft / 2 + 1;
  const double high = 2595.0 * std::log10(1.0 + (sr / 2.0) / 700.0);
  std::vector<double> mel = linspace(0.0, high, nfilt + 2), bin(nfilt + 2);
  for (int i = 0; i < nfilt + 2; ++i)
    bin[i] = std::floor((nfft + 1) * (700.0 * (std::pow(10.0, mel[i] / 2595.0) - 1.0)) / sr);
  std::vector<double> fb((size_t)nfilt * nb, 0.0);
  for (int m = 1; m <= nfilt; ++m) {
    const int fl = (int)bin[m - 1], fc = (int)bin[m], fr = (int)bin[m + 1];
    for (int k = fl; k < fc; ++k) fb[(size_t)(m - 1) * nb + k] = (k - bin[m - 1]) / (bin[m] - bin[m - 1]);
    for (int k = fc; k < fr; ++k) fb[(size_t)(m - 1) * nb + k] = (bin[m + 1] - k) / (bin[m + 1] - bin[m]);
  }
  return fb;
}

double hz_to_mel(double f) {   // Slaney (htk=False)
  const double f_sp = 200.0 / 3.0, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = std::log(6.4) / 27.0;
  return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
double mel_to_hz(double m) {
  const double f_sp = 200.0 / 3.0, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = std::log(6.4) / 27.0;
  return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}

// librosa.filters.mel(16000, 640, n_mels=128, norm=1)
std::vector<double> slaney_mel() {
  const int nmel = 128, nb = 321;
  std::vector<double> fft = linspace(0.0, 8000.0, nb);
  std::vector<double> mels = linspace(hz_to_mel(0.0), hz_to_mel(8000.0), nmel + 2), mf(nmel + 2);
  for (int i = 0; i < nmel + 2; ++i) mf[i] = mel_to_hz(mels[i]);
  std::vector<double> w((size_t)nmel * nb, 0.0);
  for (int i = 0; i < nmel; ++i) {
    const double fd0 = mf[i + 1] - mf[i], fd1 = mf[i + 2] - mf[i + 1];
    const double enorm = 2.0 / (mf[i + 2] - mf[i]);
    for (int k = 0; k < nb; ++k) {
      const double lower = -(mf[i] - fft[k]) / fd0, upper = (mf[i + 2] - fft[k]) / fd1;
      w[(size_t)i * nb + k] = std::max(0.0, std::min(lower, upper)) * enorm;
    }
  }
  return w;
}

int build_tables(DeviceTables& t) {
  int rc;
  if ((rc = upload(&t.tw256, twiddles(256, 256)))) return rc;
  if ((rc = upload(&t.tw320, twiddles(320, 320)))) return rc;
  if ((rc = upload(&t.post512, twiddles(512, 257)))) return rc;
  if ((rc = upload(&t.post640, twiddles(640, 321)))) return rc;

  std::vector<double> ham(400), hann(640), tuk(641);
  for (int n = 0; n < 400; ++n) ham[n] = 0.54 - 0.46 * std::cos(2.0 * M_PI * n / 399.0);
  for (int n = 0; n < 640; ++n) hann[n] = 0.5 - 0.5 * std::cos(2.0 * M_PI * n / 640.0);
  {  // scipy tukey(641, 0.25, sym=True)[:640]
    const int m = 641;
    const double alpha = 0.25;
    const int width = (int)std::floor(alpha * (m - 1) / 2.0);
    for (int n = 0; n < m; ++n) tuk[n] = 1.0;
    for (int n = 0; n <= width; ++n)
      tuk[n] = 0.5 * (1.0 + std::cos(M_PI * (-1.0 + 2.0 * n / alpha / (m - 1))));
    for (int n = m - width - 1; n < m; ++n)
      tuk[n] = 0.5 * (1.0 + std::cos(M_PI * (-2.0 / alpha + 1.0 + 2.0 * n / alpha / (m - 1))));
    tuk.resize(640);
  }
  double s2 = 0.0;
  for (double v : tuk) s2 += v * v;
  t.spec_scale = 1.0 / (16000.0 * s2);
  if ((rc = upload(&t.hamming400, ham))) return rc;
  {
    std::vector<float> hf(hann.begin(), hann.end()), tf(tuk.begin(), tuk.end()), mf(ham.begin(), ham.end());
    if ((rc = upload(&t.hann640f, hf)) || (rc = upload(&t.tukey640f, tf)) || (rc = upload(&t.hamming400f, mf)))
      return rc;
  }
  if ((rc = upload(&t.hann640, hann))) return rc;
  if ((rc = upload(&t.tukey640, tuk))) return rc;

  {
    std::vector<int4> meta;
    std::vector<float> pv;
    if ((rc = to_pairs(fbank_matrix(), 120, 257, 12, meta, pv)) || (rc = upload(&t.fbp_meta, meta)) ||
        (rc = upload(&t.fbp_w, pv)))
      return rc;
    std::vector<int> wl;
    std::vector<float> wv;
    if ((rc = to_windows(slaney_mel(), 128, 321, 16, wl, wv)) || (rc = upload(&t.mel16_lo, wl)) ||
        (rc = upload(&t.mel16_w, wv)))
      return rc;
    std::vector<float> wt(16 * 128);
    for (int m = 0; m < 128; ++m)
      for (int q = 0; q < 16; ++q) wt[q * 128 + m] = wv[m * 16 + q];
    if ((rc = upload(&t.mel16_wt, wt))) return rc;
    // lane pairs for mfcc3_kernel.  Lane l owns one narrow filter (0..63, <= 3 bins) read as a 3-bin
    // window and one wide filter (64..127, <= 15 bins) read as a 15-bin window.  ds_read_b32 serves
    // lanes 0-31 and 32-63 as two groups over 32 banks: the narrow filters go to the groups by halves,
    // the wide ones alternately, and each wide window's start (free within [last - 14, first]) is
    // matched so that the 32 starts of a group are distinct mod 32 — every tap read conflict-free
    // (a plain lane = filter layout costs 3x on those 15 reads).
    const std::vector<double> mel = slaney_mel();
    int first[128], last[128];
    for (int m = 0; m < 128; ++m) {
      first[m] = last[m] = -1;
      for (int k = 0; k < 321; ++k)
        if (mel[(size_t)m * 321 + k] != 0.0) { if (first[m] < 0) first[m] = k; last[m] = k; }
      SRK_REQUIRE(first[m] >= 0 && last[m] - first[m] < (m < 64 ? 3 : 15), SRK_ERR_INTERNAL,
                  "mel filter %d does not fit its lane window", m);
    }
    std::vector<int4> qlo(64);
    std::vector<float> qw(18 * 64, 0.f);
    for (int g = 0; g < 2; ++g) {
      int wide[32], start[32], owner[32];
      for (int i = 0; i < 32; ++i) { wide[i] = 64 + 2 * i + g; start[i] = first[wide[i]]; }
      for (int r = 0; r < 32; ++r) owner[r] = -1;
      // Kuhn's augmenting paths: filter i -> a start s in [max(0, last - 14), min(first, 306)], residue s % 32
      std::vector<int> seen(32);
      std::function<bool(int)> assign = [&](int i) {
        const int f = wide[i];
        for (int s0 = std::max(0, last[f] - 14); s0 <= std::min(first[f], 321 - 15); ++s0) {
          const int r = s0 % 32;
          if (seen[r]) continue;
          seen[r] = 1;
          if (owner[r] < 0 || assign(owner[r])) { owner[r] = i; start[i] = s0; return true; }
        }
        return false;
      };
      bool ok = true;
      for (int i = 0; i < 32 && ok; ++i) { std::fill(seen.begin(), seen.end(), 0); ok = assign(i); }
      if (!ok)   // still correct, only slower: plain starts
        for (int i = 0; i < 32; ++i) start[i] = first[wide[i]];
      for (int i = 0; i < 32; ++i) {
        const int l = 32 * g + i, fa = 32 * g + i, fb = wide[i];
        qlo[l] = int4{first[fa], start[i], fa, fb};
        for (int q = 0; q < 3; ++q)
          if (first[fa] + q <= last[fa]) qw[q * 64 + l] = (float)mel[(size_t)fa * 321 + first[fa] + q];
        for (int q = 0; q < 15; ++q) {
          const int k = start[i] + q;
          if (k >= first[fb] && k <= last[fb]) qw[(3 + q) * 64 + l] = (float)mel[(size_t)fb * 321 + k];
        }
      }
    }
    if ((rc = upload(&t.melq_lo, qlo)) || (rc = upload(&t.melq_w, qw))) return rc;
  }

  std::vector<float> dct(13 * 128);
  for (int k = 0; k < 128; ++k) dct[k] = (float)(1.0 / std::sqrt(128.0));
  for (int i = 1; i < 13; ++i)
    for (int k = 0; k < 128; ++k)
      dct[i * 128 + k] = (float)(std::cos(i * (2 * k + 1) * M_PI / 256.0) * std::sqrt(2.0 / 128.0));
  if ((rc = upload(&t.dct, dct))) return rc;
  t.ready = true;
  return SRK_OK;
}

}  // namespace

int get_tables(const DeviceTables** out) {
  int dev = 0;
  SRK_CHECK_HIP(hipGetDevice(&dev));
  SRK_REQUIRE(dev >= 0 && dev < kMaxDevices, SRK_ERR_INVALID, "device %d out of range", dev);
  DeviceTables& t = g_tables[dev];
  if (!t.ready) {
    std::lock_guard<std::mutex> lk(g_mutex);
    if (!t.ready) {
      int rc = build_tables(t);
      if (rc) return rc;
    }
  }
  *out = &t;
  return SRK_OK;
}

}  // namespace srk

extern "C" {

int srk_version(void) { return SRK_ABI_VERSION; }

const char* srk_last_error(void) { return srk::g_last_error.c_str(); }

int srk_init(int device) {
  SRK_API_BEGIN
  int prev = 0;
  SRK_CHECK_HIP(hipGetDevice(&prev));
  SRK_CHECK_HIP(hipSetDevice(device));
  const srk::DeviceTables* t = nullptr;
  int rc = srk::get_tables(&t);
  SRK_CHECK_HIP(hipSetDevice(prev));
  return rc;
  SRK_API_END
}

int srk_set_option(const char* name, int64_t value) {
  SRK_API_BEGIN
  SRK_REQUIRE(name, SRK_ERR_INVALID, "set_option: null name");
  const std::string n(name);
  if (n == "release_scratch") {   // free the library's grow-only scratch buffers (invalidates captured graphs)
    if (int rc = srk::release_gemm_scratch()) return rc;
    if (int rc = srk::release_conv_scratch()) return rc;
    if (int rc = srk::release_gru_scratch()) return rc;
    return srk::release_bn_scratch();
  }
  if (n == "gru_persistent") {
    srk::g_opt_gru_persistent = value != 0;
    return SRK_OK;
  }
  if (n == "conv_fwd_fp32") {   // 16-bit modes: conv forward passes on fp32 operands (1), or 16-bit (0)
    srk::g_opt_conv_fwd_fp32 = value != 0;
    return SRK_OK;
  }
  if (n == "matmul_precision") {   // 0 fp32, 1 bf16, 2 fp16 matrix-core operands (fp32 accumulate)
    SRK_REQUIRE(value >= 0 && value <= 2, SRK_ERR_INVALID, "matmul_precision must be 0, 1 or 2");
    srk::g_opt_matmul_prec.store((int)value);
    return SRK_OK;
  }
  if (n == "gemm16_kernel") {   // 0 by shape, 1 register-staged, 2 LDS-DMA ping-pong (16-bit operands)
    SRK_REQUIRE(value >= 0 && value <= 2, SRK_ERR_INVALID, "gemm16_kernel must be 0, 1 or 2");
    srk::g_opt_gemm16_kernel = (int)value;
    return SRK_OK;
  }
  if (n == "gemm_streamk") {   // fp32 ping-pong GEMM: stream-K over a partial round of tiles (1) or not (0)
    srk::g_opt_gemm_streamk = value != 0;
    return SRK_OK;
  }
  if (n == "mfcc_variant") {   // K1: bit 0 DPP untangle exchange, bit 1 twiddles in registers (bitwise the same)
    SRK_REQUIRE(value >= 0 && value <= 3, SRK_ERR_INVALID, "mfcc_variant must be 0..3");
    srk::g_opt_mfcc_variant = (int)value;
    return SRK_OK;
  }
  if (n == "bn_tree") {   // BatchNorm statistics: chunk partials combined as a pairwise tree (1) or in order (0)
    SRK_REQUIRE(value >= 0 && value <= 2, SRK_ERR_INVALID, "bn_tree must be 0, 1 or 2");
    srk::g_opt_bn_tree = (int)value;
    return SRK_OK;
  }
  if (n == "conv_ring_qs") {   // 16-bit ring convs: whole K-tiles per MFMA section, mask by width (64, 128, 256)
    SRK_REQUIRE(value >= 0 && value <= 7, SRK_ERR_INVALID, "conv_ring_qs is a 3-bit mask");
    srk::g_opt_conv_ring_qs = (int)value;
    return SRK_OK;
  }
  if (n == "conv_row16_dgrad") {   // row-staged conv2 data gradient (1, 2) or the implicit GEMM (0)
    SRK_REQUIRE(value >= 0 && value <= 2, SRK_ERR_INVALID,
                "conv_row16_dgrad must be 0, 1 (3 / 3 / 2 / 2 row blocks per wave) or 2 (5 units per wave)");
    srk::g_opt_conv_row16_dgrad = (int)value;
    return SRK_OK;
  }
  if (n == "conv_row16") {   // fbanks conv2 + pool, 16-bit: row-staged kernel (1) or implicit GEMM (0)
    SRK_REQUIRE(value >= 0 && value <= 2, SRK_ERR_INVALID, "conv_row16 must be 0, 1 (8 waves) or 2 (4 waves)");
    srk::g_opt_conv_row16 = (int)value;
    return SRK_OK;
  }
  if (n == "conv_row32") {   // fbanks conv2 on fp32 operands: row-staged kernels (1) or the implicit GEMM (0)
    srk::g_opt_conv_row32 = value != 0;
    return SRK_OK;
  }
  if (n == "conv_fw_gemm") {   // full-width "valid" conv forward as a plain GEMM (1) or the implicit GEMM (0)
    srk::g_opt_conv_fw_gemm = value != 0;
    return SRK_OK;
  }
  if (n == "conv_fast16") {   // 16-bit-source register-staged convs: uniform-tap fast gathers (1) or generic (0)
    srk::g_opt_conv_fast16 = value != 0;
    return SRK_OK;
  }
  if (n == "conv_colsum16") {   // 16-bit modes: conv bias gradients fused into dY's 16-bit conversion (1) or not (0)
    srk::g_opt_conv_colsum16 = value != 0;
    return SRK_OK;
  }
  if (n == "conv_unpool16") {   // 16-bit modes: pooled-conv backward writes dY's 16-bit copy directly (1) or not (0)
    srk::g_opt_conv_unpool16 = value != 0;
    return SRK_OK;
  }
  if (n == "conv_ring") {   // ring conv kernels where the shape qualifies: bits 0-2 fp32 fwd / dgrad / wgrad, 4-6 16-bit,
                            // 7 the pooled forward too
    SRK_REQUIRE(value >= 0 && value <= 0xf7, SRK_ERR_INVALID,
                "conv_ring is a mask of 1 / 2 / 4 (fp32 fwd / dgrad / wgrad), 16 / 32 / 64 (16-bit) and 128 "
                "(the pooled forward too)");
    srk::g_opt_conv_ring = (int)value;
    return SRK_OK;
  }
  if (n == "conv_tile") {   // 128: 128-row conv tiles (4 waves); 256: 256-row tiles (8 waves) on tall convs
    SRK_REQUIRE(value == 128 || value == 256, SRK_ERR_INVALID, "conv_tile must be 128 or 256");
    srk::g_opt_conv_tile = (int)value;
    return SRK_OK;
  }
  if (n == "conv_unpool_gather") {   // pooled conv backward: gathers unpool (1) or a dense scratch gradient (0)
    srk::g_opt_conv_unpool_gather = value != 0;
    return SRK_OK;
  }
  if (n == "conv_fused_db") {   // conv bias gradients fused into the weight-gradient kernel (1) or a column sum (0)
    srk::g_opt_conv_fused_db = value != 0;
    return SRK_OK;
  }
  if (n == "conv16_sources") {   // bf16 / fp16 convs gather from a pre-rounded 16-bit copy (1) or round in LDS (0)
    srk::g_opt_conv16_sources = value != 0;
    return SRK_OK;
  }
  if (n == "gemm32_kernel") {   // 0 by shape, 1 register-staged, 2 LDS-DMA ping-pong (fp32 operands)
    SRK_REQUIRE(value >= 0 && value <= 2, SRK_ERR_INVALID, "gemm32_kernel must be 0, 1 or 2");
    srk::g_opt_gemm32_kernel = (int)value;
    return SRK_OK;
  }
  if (n == "gru_spin_limit") {   // test hook: polls before a persistent wait gives up (0 = ~2 s default)
    SRK_REQUIRE(value >= 0 && value <= 0xffffffffLL, SRK_ERR_INVALID, "gru_spin_limit out of range");
    srk::g_opt_gru_spin_limit = (unsigned)value;
    return SRK_OK;
  }
  if (n == "gru_xcd_local") {   // persistent GRU: XCD-local hand-off when every XCD hosts one (dir, group)
    srk::g_opt_gru_xcd_local = value != 0;
    return SRK_OK;
  }
  if (n == "gru_fp32_dual_chain") {   // fp32 recurrence: 8-wave workgroups running two row chains (1) or the 4-wave form (0)
    srk::g_opt_gru_dc = value != 0;
    return SRK_OK;
  }
  if (n == "gru_dc_offset_ns") {   // fp32 two-chain kernels: delay chain 1's start (phase offset between the chains)
    SRK_REQUIRE(value >= 0 && value <= 1000000, SRK_ERR_INVALID, "gru_dc_offset_ns out of range");
    srk::g_opt_gru_dc_offset = (unsigned)(value / 10);
    return SRK_OK;
  }
  if (n == "gru_fwd_worker") {   // 16-bit forward: y / gate stores and the gi fetch on extra worker waves (1) or not (0)
    srk::g_opt_gru_fwd_worker = value != 0;
    return SRK_OK;
  }
  if (n == "gru_dwhh_fused") {   // 16-bit backward: dW_hh accumulated in the recurrence kernel (bit 0) or by a GEMM (0);
                                  // bit 1: h_prev fetched after the next exchange barrier, bit 2: recurrence waves at s_setprio 1
    SRK_REQUIRE(value >= 0 && value <= 7, SRK_ERR_INVALID, "gru_dwhh_fused must be 0..7");
    srk::g_opt_gru_dwhh_fused = (value & 1) ? (int)value : 0;
    return SRK_OK;
  }
  if (n == "gru_dc_prio") {   // fp32 two-chain kernels: 0 equal priority, 1 / 2 chain 0 / 1 at s_setprio 1 (static)
    SRK_REQUIRE(value >= 0 && value <= 2, SRK_ERR_INVALID, "gru_dc_prio must be 0, 1 or 2");
    srk::g_opt_gru_dc_prio = (int)value;
    return SRK_OK;
  }
  if (n == "gru_fp32_fast_cell") {   // fp32 two-chain forward: v_exp_f32 / v_rcp_f32 cell nonlinearities
    srk::g_opt_gru_fast_cell = value != 0;
    return SRK_OK;
  }
  if (n == "gru_lp_wide") {   // 16-bit recurrence over > 256 rows: 64-row workgroups in one launch (1) or 256-row chunks (0)
    srk::g_opt_gru_lp_wide = value != 0;
    return SRK_OK;
  }
  if (n == "gemm_skinny") {   // GEMMs with a dimension <= 16 on the VALU kernels (1) or the matrix-core tiles (0)
    srk::g_opt_gemm_skinny = value != 0;
    return SRK_OK;
  }
  if (n == "gru_dwhh_batched") {   // 16-bit GRU backward: both directions' dW_hh in one batched GEMM (1) or two (0)
    srk::g_opt_gru_dwhh_batched = value != 0;
    return SRK_OK;
  }
  if (n == "gru_lp_32x32") {   // 16-bit recurrence: 32 x 32 workgroups (1) or 64 rows x 16 units (0)
    srk::g_opt_gru_lp2 = value != 0;
    return SRK_OK;
  }
  if (n == "gru_trace_ptr") {   // diagnostics: device buffer of 8 x u64 per (workgroup, step), 0 = off
    srk::g_opt_gru_trace = reinterpret_cast<unsigned long long*>(value);
    return SRK_OK;
  }
  SRK_REQUIRE(false, SRK_ERR_INVALID, "set_option: unknown option '%s'", name);
  SRK_API_END
}

}  // extern "C"

extern "C" int64_t srk_scratch_generation(void) { return srk::g_scratch_gen.load(); }
