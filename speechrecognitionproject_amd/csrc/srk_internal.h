// Internal helpers shared by every translation unit of libsrk.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/srk.h"

namespace srk {

// Thread-local last-error text, read back through srk_last_error() (include/srk.h).
void set_error(const char* fmt, ...);

#define SRK_CHECK_HIP(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      ::srk::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
      return SRK_ERR_HIP;                                                                \
    }                                                                                    \
  } while (0)

#define SRK_REQUIRE(cond, code, ...)     \
  do {                                   \
    if (!(cond)) {                       \
      ::srk::set_error(__VA_ARGS__);     \
      return (code);                     \
    }                                    \
  } while (0)

// Wraps the body of every extern "C" entry point: C++ exceptions never cross the C ABI.
#define SRK_API_BEGIN try {
#define SRK_API_END                                              \
  }                                                              \
  catch (const std::exception& e) {                              \
    ::srk::set_error("exception: %s", e.what());                 \
    return SRK_ERR_INTERNAL;                                     \
  }                                                              \
  catch (...) {                                                  \
    ::srk::set_error("unknown exception");                       \
    return SRK_ERR_INTERNAL;                                     \
  }

// Per-device constant tables (twiddles, windows, filterbanks, DCT), uploaded once by srk_init.
struct DeviceTables {
  bool ready = false;
  // FFT twiddles exp(-2*pi*i*t/M), float2 interleaved
  float2* tw256 = nullptr;     // M = 256 (fbank, N = 512)
  float2* tw320 = nullptr;     // M = 320 (mfcc / spec, N = 640)
  float2* post512 = nullptr;   // exp(-2*pi*i*k/512), k = 0..256
  float2* post640 = nullptr;   // exp(-2*pi*i*k/640), k = 0..320
  double* hamming400 = nullptr;
  double* tukey640 = nullptr;
  double* hann640 = nullptr;
  float* hann640f = nullptr;   // fp32 copies for the register-FFT kernels
  float* tukey640f = nullptr;
  float* hamming400f = nullptr;
  // filter banks as lane pairs (filter l and nf - 1 - l, balancing narrow and wide triangles):
  // meta {lo_a, cnt_a, lo_b, cnt_b}, weights of a then b, zero padded to a fixed tap count
  int4* fbp_meta = nullptr; float* fbp_w = nullptr;     // fbank: 60 pairs x 12 taps
  float* dct = nullptr;        // [13][128] orthonormal DCT-II
  // Slaney mel as fixed 16-tap windows (zero-padded, start clamped so lo+16 <= bins)
  int* mel16_lo = nullptr; float* mel16_w = nullptr;   // [128], [128][16]
  float* mel16_wt = nullptr;                           // [16][128] (lane-coalesced)
  // Slaney mel as 64 lane pairs (a narrow filter <= 3 bins, a wide one <= 15 bins, bank-conflict-free
  // window starts; runtime.hip): {start_a, start_b, filter_a, filter_b} and [18][64] weights
  // (taps 0..2 from start_a, taps 3..17 from start_b)
  int4* melq_lo = nullptr; float* melq_w = nullptr;
  double spec_scale = 0.0;     // 1 / (fs * sum(w^2)) for the Tukey window
};

// Returns the tables for the current HIP device, building them on first use.
int get_tables(const DeviceTables** out);

// Matrix-core operand precision of the GEMM-shaped kernels (srk_set_option "matmul_precision"):
// 0 = fp32 (exact fp32 MFMA, the reference's arithmetic), 1 = bf16, 2 = fp16 operands (rounded to
// nearest-even when staged into LDS) with fp32 accumulation and fp32 inputs / outputs.
enum MatmulPrec { kPrecF32 = 0, kPrecBF16 = 1, kPrecF16 = 2 };
int matmul_prec();
// Scoped override of matmul_prec() on this host thread (p < 0: no override): the conv forward passes under
// "conv_fwd_fp32" run their whole dispatch at fp32.
extern thread_local int t_prec_override;
struct PrecScope {
  int saved;
  explicit PrecScope(int p) : saved(t_prec_override) {
    if (p >= 0) t_prec_override = p;
  }
  ~PrecScope() { t_prec_override = saved; }
};
// 16-bit modes: every convolution FORWARD pass on fp32 operands, the data / weight gradients on 16-bit ones
// ("conv_fwd_fp32", default 0).  resnet_bgru's training-mode BatchNorm chain amplifies the forward's operand
// rounding into 4-39 % norm-wise gradient errors, while 16-bit gradients alone stay <= 0.9 %
// (tools/bf16_policy_resnet.py): the faithful 16-bit training mode of the BatchNorm models.
extern int g_opt_conv_fwd_fp32;

// Kernel of the 16-bit-operand GEMM (srk_set_option "gemm16_kernel", A/B measurements and tests):
// 0 = by shape, 1 = register-staged gemm_h16_kernel, 2 = LDS-DMA ping-pong gemm_g16_kernel.
// Bumped whenever a library scratch buffer is (re)allocated: a captured HIP graph that refers to the
// old buffer must not be replayed (srk_scratch_generation; graphs.GraphedStep checks it).
extern std::atomic<int64_t> g_scratch_gen;
// Free every grow-only scratch buffer of one pool (device-synchronizing; bumps g_scratch_gen).
int release_gemm_scratch();
int release_conv_scratch();
int release_bn_scratch();
int release_gru_scratch();
extern int g_opt_gemm16_kernel;
// Kernel of the fp32 GEMM (srk_set_option "gemm32_kernel"): 0 = by shape, 1 = register-staged
// gemm_f32_kernel, 2 = LDS-DMA ping-pong gemm_p32_kernel.
extern int g_opt_gemm32_kernel;
extern int g_opt_gru_dwhh_batched;
extern int g_opt_gemm_skinny;   // GEMMs with a dimension <= 16 on the VALU skinny kernels   // 16-bit GRU backward: one batched dW_hh GEMM for both directions
// 16-bit conv operand sources (srk_set_option "conv16_sources", default 1): bf16 / fp16 convolutions
// gather from one pre-rounded 16-bit copy of x / dY / the weights (0 = round at LDS-store time).
extern int g_opt_conv16_sources;
// conv bias gradients as column sums fused into the weight-gradient kernel ("conv_fused_db", default
// 1; 0 = the separate column-sum kernel over dY)
extern int g_opt_conv_fused_db;
// the pooled conv's backward gathers the pooled gradient through the argmax ("conv_unpool_gather",
// default 1; 0 = unpool into library scratch first)
extern int g_opt_conv_unpool_gather;
// 16-bit-source modes: the pooled conv's backward writes the dense dY straight as its 16-bit copy
// ("conv_unpool16", default 1; 0 = dense fp32 dY, then the 16-bit conversion and column sums)
extern int g_opt_conv_unpool16;
// 16-bit-source modes: the conv bias gradient (column sums of dY) fused into the pass that rounds dY (or
// unpools it) to its 16-bit copy ("conv_colsum16", default 1; 0 = a separate column-sum pass over dY)
extern int g_opt_conv_colsum16;
// 16-bit ring convs: whole 32-deep K-tiles per MFMA section (QS 2) by tile width, a mask ("conv_ring_qs": bit 1
// BN 128, bit 2 BN 256; default 6)
extern int g_opt_conv_ring_qs;
// register-staged 16-bit-source convs (fwd / dgrad): uniform-tap gathers with per-row bases and zero-filling
// buffer loads where the channels are a multiple of the K-tile ("conv_fast16", default 1)
extern int g_opt_conv_fast16;
// fbanks_cnn conv2 + maxpool2 in 16-bit modes on the row-staged kernel (weights resident in LDS, image rows staged
// once per tile) ("conv_row16", default 1; 0 = the implicit-GEMM kernels)
extern int g_opt_conv_row16;
// fbanks_cnn conv2 (+ maxpool2) on fp32 operands on the row-staged kernels (x rows staged once per tile, the weights
// streamed one tap at a time) ("conv_row32", default 1; 0 = the implicit-GEMM kernels)
extern int g_opt_conv_row32;
// a full-width "valid" conv's forward (fbanks_cnn conv3, (1, 10) over width 10) as the plain GEMM x . Wt + bias
// ("conv_fw_gemm", default 1; 0 = the implicit GEMM)
extern int g_opt_conv_fw_gemm;
// the row-staged data gradient of the same conv ("conv_row16_dgrad", default 2 = 5 units per wave; 1 = 3 / 3 / 2 / 2
// row blocks per wave, 418 vs 475-485 us, r05p; 0 = the implicit GEMM)
extern int g_opt_conv_row16_dgrad;
// BatchNorm training statistics: the <= 256 chunk partials combined in chunk order, the count ratios off the
// dependent chain ("bn_tree" 0, default); 1 = a fixed pairwise tree, one wave per channel (more accurate, but
// other bits than the reference's in-order arithmetic: ReLU decisions on values within roundoff of 0 move —
// tests/test_conv_gpu.py golden resnet_bgru at B = 2); 2 = in order with the divides in the chain (form 0's
// bitwise reference)
extern int g_opt_bn_tree;
// conv tile shape ("conv_tile": 128 = 128-row tiles of 4 waves, 256 = 256-row tiles of 8 waves on
// tall convolutions)
extern int g_opt_conv_tile;
// LDS-DMA ring implicit-GEMM convolutions where the shape qualifies ("conv_ring": a mask of
// 1 / 2 / 4 = fp32 forward / data gradient / weight gradient, 16 / 32 / 64 = the same on 16-bit
// operands, 128 = the forward with the pooled epilogue and the fp32 forward at K < 3072 too; default
// 0x77 — measured, r04ab / r04ab3 / r04ab6: the pooled ring forward slower in both precisions, the fp32
// ring forward faster on the deep-K ResNet layers only)
extern int g_opt_conv_ring;
// K1 MFCC variant ("mfcc_variant", bitwise-identical outputs): bit 0 = the untangle's partner exchange
// by DPP row_mirror instead of ds_bpermute, bit 1 = twiddles in registers instead of LDS (default 3)
extern int g_opt_mfcc_variant;
// stream-K for fp32 ping-pong GEMMs whose 256 x 256 grid covers 1/2 .. 1 round of CUs ("gemm_streamk",
// default 1)
extern int g_opt_gemm_streamk;

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// RAII event pair around one kernel launch (prof.hip); inert unless srk_prof_enable(1).
// `work` = the launch's ALGORITHMIC flops (matrix kernels) or bytes (streaming kernels).
class ProfScope {
 public:
  ProfScope(const char* name, hipStream_t s, double work = 0.0);
  ~ProfScope();
  ProfScope(const ProfScope&) = delete;
  ProfScope& operator=(const ProfScope&) = delete;
  // The launch's kernel and shape ("gemm_f32_kernel<NT,256x128> 13056x3072x1024"), printf-style;
  // srk_prof_kernels groups records by (name, detail).  No-op (no formatting) when profiling is off.
  void detail(const char* fmt, ...) __attribute__((format(printf, 2, 3)));
  // The launch's ALGORITHMIC HBM bytes (matrix kernels, whose `work` is flops): each operand tensor read
  // once + the output written once — what PMC traffic is priced against.
  void bytes(double b) { bytes_ = b; }

 private:
  const char* name_;
  hipStream_t s_;
  void* a_;
  double work_;
  double bytes_ = 0.0;
  unsigned long long opened_ = 0;   // this scope's number among the thread's scopes (innermost-wins nesting)
  char detail_[96];
};

}  // namespace srk
