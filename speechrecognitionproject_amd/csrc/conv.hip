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
#include <type_traits>

#include "gemm.h"
#include "mfma_tile.h"

namespace srk {
namespace {

using namespace tile;

enum { kFwd = 0, kDgrad = 1, kWgrad = 2 };

// Division by a launch-invariant divisor as multiply-high + add + shift (Granlund & Montgomery,
// "Division by invariant integers using multiplication", 1994): the gathers split staged k / m
// indices into (pixel, tap, channel) every k-tile, and integer division is a long software
// sequence on the VALU.  Exact for n < 2^31 (run_conv_gemm checks M, K < 2^31).
struct FastDiv {
  unsigned d = 1, m = 1, l = 0;
  FastDiv() = default;
  __host__ explicit FastDiv(unsigned dv) : d(dv) {
    while ((1ull << l) < dv) ++l;
    m = (unsigned)(((1ull << 32) * ((1ull << l) - dv)) / dv + 1);
  }
  __device__ __forceinline__ unsigned div(unsigned n) const { return (__umulhi(n, m) + n) >> l; }
};

struct ConvArgs {
  int N, H, W, Ci, Ho, Wo, Co, KH, KW, ph, pw, sh, sw;
  const float* x;      // [N][H][W][Ci]
  const float* dy;     // [N][Ho][Wo][Co]
  const float* wmat;   // fwd: Wt [KH*KW*Ci][Co]; dgrad: Wd [KH*KW*Co][Ci]
  float* out;          // fwd: Y [N*Ho*Wo][Co]; dgrad: dX [N*H*W][Ci]; wgrad: dWt [KH*KW*Ci][Co]
  const float* bias;   // fwd only, [Co]
  int64_t M, Nn, K;    // GEMM dims
  int tiles_m, tiles_n, tiles, nblk, group_m;
  int64_t kchunk;
  float* partial;      // split-K slabs
  // 16-bit operand sources (matmul_precision bf16 / fp16, 8-aligned channel counts): the A source
  // (x or dy) and B (the weight matrix, or dy for wgrad) pre-rounded once per call, so a gather
  // moves 8 elements per 16-B load and the LDS store needs no conversion.  Null = fp32 sources.
  const unsigned short* a16;
  const unsigned short* b16;
  // divisors of the gathers (host-set): pixel grid (cols, rows), channels, KW, strides (dgrad)
  FastDiv fd_w, fd_h, fd_c, fd_kw, fd_sh, fd_sw;
  // fwd: max-pool the output over windows of pool_w consecutive output columns in the epilogue
  // (0 = off): out becomes [M / pool_w][Co], pool_arg the uint8 window argmax
  int pool_w;
  uint8_t* pool_arg;
  // wgrad: column sums of B = dY over this split's pixels (the conv bias gradient), written by the
  // tiles of the first m row as [split][Co] (null = off)
  float* colsum_part;
  float* db;           // host side only: where run_conv_gemm<kWgrad> reduces colsum_part to
  // dgrad / wgrad of a (1, 4)-pooled conv (UNPOOL kernels): dy holds the POOLED gradient
  // [N*Ho*Wo/4][Co] and dy_arg its window argmax; the gathers rebuild the dense gradient
  // dY[pixel][co] = dy_arg[pixel/4][co] == pixel % 4 ? dy[pixel/4][co] : 0 at LDS-store time
  const uint8_t* dy_arg;
  // 16-bit sources, fwd / dgrad (host-set, run_conv_gemm): the gathered operand's channel count is a multiple
  // of the K-tile (one tap per K-tile, uniform over the workgroup), dgrad stride 1, and both 16-bit operands
  // under 2^30 elements — the gathers then use per-row base offsets fixed for the whole k loop, 32-bit buffer
  // loads whose out-of-range offset returns zeros (no masks, no selects at LDS-store time)
  int fast16;
};

// Implicit-GEMM operand gathers.  Each returns the ELEMENT OFFSET of the value (clamped to 0 when
// the position is outside the image / problem) and whether it is valid; the caller loads
// unconditionally and zeroes invalid values at LDS-store time (after the stage's MFMAs), so no load
// is exec-masked and no select waits on a load in front of the MFMAs.
//   fwd   A[m = pixel (n,ho,wo)][k = (kh,kw,ci)] = X[n, ho*sh+kh-ph, wo*sw+kw-pw, ci]
//   dgrad A[m = pixel (n,h,w)][k = (kh,kw,co)]   = dY[n, (h+ph-kh)/sh, (w+pw-kw)/sw, co] (exact division only)
//   wgrad A[m = (kh,kw,ci)][k = pixel (n,ho,wo)] = X[n, ho*sh+kh-ph, wo*sw+kw-pw, ci]
struct Pix { int n, a, b; bool ok; };   // pixel (n, row, col) + "row index < rows"

__device__ __forceinline__ Pix split_pix(int64_t p, int64_t rows, const FastDiv& fw, const FastDiv& fh) {
  Pix q;
  q.ok = p < rows;
  const unsigned pc = q.ok ? (unsigned)p : 0u;
  const unsigned u = fw.div(pc), v = fh.div(u);
  q.b = (int)(pc - u * fw.d);
  q.a = (int)(u - v * fh.d);
  q.n = (int)v;
  return q;
}
struct Tap { int kh, kw, ch; };   // k (or wgrad m) = (kh, kw, channel)
__device__ __forceinline__ Tap split_tap(int64_t k, const FastDiv& fc, const FastDiv& fkw) {
  const unsigned kk = (unsigned)k, u = fc.div(kk), v = fkw.div(u);
  Tap t;
  t.ch = (int)(kk - u * fc.d);
  t.kw = (int)(u - v * fkw.d);
  t.kh = (int)v;
  return t;
}

template <int MODE>
__device__ __forceinline__ int64_t a_offset(const ConvArgs& c, const Pix& p, const Tap& t, bool& ok) {
  if (MODE == kDgrad) {
    const int ht = p.a + c.ph - t.kh, wt = p.b + c.pw - t.kw;
    const int ho = (int)c.fd_sh.div(ht > 0 ? (unsigned)ht : 0u), wo = (int)c.fd_sw.div(wt > 0 ? (unsigned)wt : 0u);
    ok = ok && p.ok && ht >= 0 && wt >= 0 && ho * c.sh == ht && wo * c.sw == wt && ho < c.Ho && wo < c.Wo;
    return ok ? (((int64_t)p.n * c.Ho + ho) * c.Wo + wo) * c.Co + t.ch : 0;
  }
  const int hi = p.a * c.sh + t.kh - c.ph, wi = p.b * c.sw + t.kw - c.pw;
  ok = ok && p.ok && hi >= 0 && hi < c.H && wi >= 0 && wi < c.W;
  return ok ? (((int64_t)p.n * c.H + hi) * c.W + wi) * c.Ci + t.ch : 0;
}

// ------------------------------------------------------------------ 16-bit operand images
// (matmul_precision bf16 / fp16): the staged fp32 float4s are rounded to 4 x 16 bit and stored as
// ONE 8-B write each, in the orientation they were gathered:
//   k-contiguous A (fwd / dgrad):  [row][BK + 8]       fragment = ds_read_b128 (8 consecutive k)
//   row-contiguous A (wgrad), B:   [k][kTrPitch]       fragment = 2 x ds_read_b64_tr_b16 (the
//       hardware transpose read: lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3;
//       lane i receives column i of the 4 rows), pitch 160 = 32 (mod 128) elements, so each
//       32-lane half reads 4 rows x 64 B on 64 distinct banks.
typedef float v8f_ __attribute__((ext_vector_type(8)));
typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
constexpr int kTrPitch = 160;

template <int LP> struct ConvLp;
template <> struct ConvLp<1> {
  typedef __bf16 e8 __attribute__((ext_vector_type(8)));
  typedef __bf16 e4 __attribute__((ext_vector_type(4)));
  __device__ static __forceinline__ f32x16 mma(u32x4_ a, u32x4_ b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(e8, a), __builtin_bit_cast(e8, b), c, 0, 0, 0);
  }
};
template <> struct ConvLp<2> {
  typedef _Float16 e8 __attribute__((ext_vector_type(8)));
  typedef _Float16 e4 __attribute__((ext_vector_type(4)));
  __device__ static __forceinline__ f32x16 mma(u32x4_ a, u32x4_ b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(e8, a), __builtin_bit_cast(e8, b), c, 0, 0, 0);
  }
};

// 16-bit image of one operand: element offset of a staged float4 (same walk as Img::store_off) and
// the 32x32x16 MFMA fragment of operand rows c0 + (lane & 31), k = kk + 8 (lane >> 5) + 0..7.
template <bool KC, int ROWS, int BK>
struct Img16 {
  static constexpr int P = KC ? BK + 8 : (ROWS <= 128 ? kTrPitch : ROWS + 32);   // 32 (mod 128) elements
  static constexpr int ELEMS = KC ? ROWS * P : BK * P;
  __device__ static __forceinline__ int store_off(int vi) {
    return KC ? (vi / (BK / 4)) * P + (vi % (BK / 4)) * 4 : (vi / (ROWS / 4)) * P + (vi % (ROWS / 4)) * 4;
  }
  // the same for a staged unit of 8 elements (16-bit sources)
  __device__ static __forceinline__ int store_off8(int vi) {
    return KC ? (vi / (BK / 8)) * P + (vi % (BK / 8)) * 8 : (vi / (ROWS / 8)) * P + (vi % (ROWS / 8)) * 8;
  }
  __device__ static __forceinline__ u32x4_ frag(const unsigned short* img, int c0, int kk, int lane) {
    if (KC) return *reinterpret_cast<const u32x4_*>(img + (c0 + (lane & 31)) * P + kk + 8 * (lane >> 5));
    const int q = (lane >> 2) & 3, p = lane & 3;
    const unsigned short* a = img + (kk + 8 * (lane >> 5) + q) * P + c0 + 16 * ((lane >> 4) & 1) + 4 * p;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * P));
    const u32x2_ l2 = __builtin_bit_cast(u32x2_, lo), h2 = __builtin_bit_cast(u32x2_, hi);
    return u32x4_{l2.x, l2.y, h2.x, h2.y};
  }
};

// VEC: the 4 elements of a staged A float4 share one pixel and one (kh, kw) — channel count % 4 == 0
// (fwd / wgrad: Ci, dgrad: Co).  VECB: the B operand's N % 4 == 0 (16-B loads along n).
// LP: 0 = fp32 operands (v_mfma_f32_32x32x2_f32), 1 / 2 = bf16 / fp16 operands rounded at LDS-store
// time (v_mfma_f32_32x32x16_{bf16,f16}, Img16 images), fp32 gathers, masks and epilogue alike.
// S16: 16-bit sources (ConvArgs::a16 / b16, rounded by the same conversion as the LDS-store path,
// so the MFMA operands are bit-identical): a staged unit is 8 elements = one 16-B load and one
// 16-B LDS store (needs VEC and VECB with 8-aligned channel counts / N).
// UNPOOL: dY is the (1, 4)-pooled gradient + argmax (ConvArgs::dy_arg; dgrad / wgrad, fp32 sources)
// NW: waves per workgroup — 4 (2 x 2, each (BM/2) x (BN/2)) or 8 (BM = 256: 4 x 2, each 64 x (BN/2);
// one 8-wave workgroup per CU holds a 256-row tile: half the L2 -> CU operand bytes per flop of two
// 128-row workgroups)
template <int MODE, int BM, int BN, int BK, bool VEC, bool VECB, int LP = 0, bool S16 = false, bool UNPOOL = false,
          int NW = 4>
__global__ __launch_bounds__(NW * 64) void conv_gemm_kernel(ConvArgs c) {
  constexpr int NT = NW * 64;
  constexpr int WM = NW == 8 ? 4 : 2, WN = NW / WM;
  constexpr bool AKC = MODE != kWgrad;   // A k-contiguous (channels along k) for fwd / dgrad
  using IA = Img<AKC, BM, BK>;
  using IB = Img<false, BN, BK>;         // B = row-major [K][N] (Wt / Wd / dY)
  using JA = Img16<AKC, BM, BK>;
  using JB = Img16<false, BN, BK>;
  static_assert(!S16 || (LP != 0 && VEC && VECB), "16-bit sources need the vector gathers");
  static_assert(!UNPOOL || (MODE != kFwd && !S16 && VEC && VECB), "unpooling gathers: dgrad / wgrad, fp32 sources");
  constexpr int EU = S16 ? 8 : 4;        // elements per staged unit
  constexpr int VA = BM * BK / EU / NT, VB = BN * BK / EU / NT;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(VA >= 1 && VB >= 1 && TM >= 1 && TN >= 1 && VA * 4 <= 32, "bad tile");
  static_assert(NT % (BN / 4) == 0 && (AKC || NT % (BM / EU) == 0), "a staging thread keeps its columns / taps");
  constexpr int STAGE_FLOATS = LP ? (JA::ELEMS + JB::ELEMS + 1) / 2 : IA::FLOATS + IB::FLOATS;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE_FLOATS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int split, tm, tn;
  map_tile(c.nblk, c.tiles, c.tiles_m, c.tiles_n, c.group_m, true, split, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kb0 = split * c.kchunk;
  const int64_t ke = (kb0 + c.kchunk < c.K) ? kb0 + c.kchunk : c.K;
  const int wm0 = (wave / WN) * (BM / WM), wn0 = (wave % WN) * (BN / WN);
  const float* __restrict__ Asrc = MODE == kDgrad ? c.dy : c.x;
  const float* __restrict__ Bsrc = MODE == kWgrad ? c.dy : c.wmat;
  // pixel / tap splits by the host-set divisors: fd_w, fd_h = the pixel grid of A's rows (fwd / dgrad)
  // or k (wgrad); fd_c = the channel count along A's k (fwd / dgrad) or m (wgrad); fd_kw = KW

  // fwd / dgrad: this thread's A rows are fixed for the whole k loop (decomposed once);
  // wgrad: its A "rows" (= taps m) are fixed instead.
  Pix prow[VA];
  Tap mtap[4];   // wgrad: the taps m0 + aq + e of this thread (fixed for the whole k loop)
  int aq;        // fwd/dgrad: k offset of this thread's float4 in a stage; wgrad: m offset
  if (AKC) {
    aq = (tid % (BK / EU)) * EU;
#pragma unroll
    for (int i = 0; i < VA; ++i) prow[i] = split_pix(m0 + (tid + i * NT) / (BK / EU), c.M, c.fd_w, c.fd_h);
  } else {
    aq = (tid % (BM / EU)) * EU;
#pragma unroll
    for (int e = 0; e < 4; ++e) mtap[e] = split_tap(m0 + aq + e < c.M ? m0 + aq + e : 0, c.fd_c, c.fd_kw);
  }

  // fast16 gathers (ConvArgs::fast16): per A row, the element offset of tap (0, 0) channel 0 relative to the
  // row's pixel and the row's first valid tap row / column as (lo, hi) windows the uniform tap is checked against
  int rbase[AKC && S16 ? VA : 1], rh[AKC && S16 ? VA : 1], rw[AKC && S16 ? VA : 1];
  if constexpr (AKC && S16) {
    if (c.fast16) {
#pragma unroll
      for (int i = 0; i < VA; ++i) {
        const Pix& q = prow[i];
        if (MODE == kFwd) {   // hi = a sh - ph + kh, wi = b sw - pw + kw
          rh[i] = q.ok ? q.a * c.sh - c.ph : -(1 << 20);
          rw[i] = q.b * c.sw - c.pw;
          rbase[i] = ((q.n * c.H + rh[i]) * c.W + rw[i]) * c.Ci;
        } else {              // stride 1: ho = a + ph - kh, wo = b + pw - kw
          rh[i] = q.ok ? q.a + c.ph : -(1 << 20);
          rw[i] = q.b + c.pw;
          rbase[i] = ((q.n * c.Ho + rh[i]) * c.Wo + rw[i]) * c.Co;
        }
      }
    }
  }

  v4f ra[VA], rb[VB];   // fp32 staged units (unused, and eliminated, when S16)
  // UNPOOL: the argmax bytes of each staged dY unit and its pixel's window position (2 bits per unit)
  unsigned parg[UNPOOL ? (MODE == kDgrad ? VA : VB) : 1];
  unsigned psub = 0;
  u32x4_ ha[S16 ? VA : 1], hb[S16 ? VB : 1];   // S16 staged units (8 x 16 bit)
  unsigned amask = 0, bmask = 0;   // bit = element valid (4 per staged float4; S16: 1 per unit)
  auto load_tile = [&](int64_t k0) {
    amask = 0;
    bmask = 0;
    if constexpr (S16) {
      if constexpr (AKC) {
        if (c.fast16) {   // one tap per K-tile (uniform), buffer loads: out of range -> 16 zero bytes
          const auto rsA16 = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(c.a16), (short)0, 0x7ffffff0,
                                                               0x00020000);
          const auto rsB16 = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(c.b16), (short)0, 0x7ffffff0,
                                                               0x00020000);
          const int chans = MODE == kDgrad ? c.Co : c.Ci;
          const int tap = __builtin_amdgcn_readfirstlane((int)((unsigned)k0 / (unsigned)chans));
          const int ch = (int)k0 - tap * chans + aq;
          const int kh = __builtin_amdgcn_readfirstlane(tap / c.KW), kw = tap - kh * c.KW;
          const bool kin = k0 + aq < ke;
#pragma unroll
          for (int i = 0; i < VA; ++i) {
            bool ok;
            int off;
            if (MODE == kFwd) {
              const int hi = rh[i] + kh, wi = rw[i] + kw;
              ok = kin && (unsigned)hi < (unsigned)c.H && (unsigned)wi < (unsigned)c.W;
              off = rbase[i] + (kh * c.W + kw) * c.Ci + ch;
            } else {
              const int ho = rh[i] - kh, wo = rw[i] - kw;
              ok = kin && (unsigned)ho < (unsigned)c.Ho && (unsigned)wo < (unsigned)c.Wo;
              off = rbase[i] - (kh * c.Wo + kw) * c.Co + ch;
            }
            ha[i] = __builtin_bit_cast(u32x4_, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rsA16, ok ? (int)((unsigned)off * 2u) : (int)0x80000000u, 0, 0));
          }
#pragma unroll
          for (int i = 0; i < VB; ++i) {
            const int vi = tid + i * NT;
            const int k = (int)k0 + vi / (BN / EU), n = (int)n0 + (vi % (BN / EU)) * EU;
            const bool ok = k < ke && n < c.Nn;
            hb[i] = __builtin_bit_cast(u32x4_, __builtin_amdgcn_raw_buffer_load_b128(
                                                   rsB16, ok ? (int)((unsigned)(k * (int)c.Nn + n) * 2u) : (int)0x80000000u,
                                                   0, 0));
          }
          amask = (1u << VA) - 1u;
          bmask = (1u << VB) - 1u;
          return;
        }
      }
      // every unit shares one pixel and one tap (channel counts % 8 == 0) and never straddles ke
      // (K and the split chunks are multiples of 8)
      if (AKC) {
        const int64_t k = k0 + aq;
        const Tap t = split_tap(k < ke ? k : 0, c.fd_c, c.fd_kw);
#pragma unroll
        for (int i = 0; i < VA; ++i) {
          bool ok = k < ke;
          const int64_t off = a_offset<MODE>(c, prow[i], t, ok);
          ha[i] = *reinterpret_cast<const u32x4_*>(c.a16 + off);
          amask |= (ok ? 1u : 0u) << i;
        }
      } else {
#pragma unroll
        for (int i = 0; i < VA; ++i) {
          const int64_t k = k0 + (tid + i * NT) / (BM / EU);
          const Pix p = split_pix(k < ke ? k : 0, c.K, c.fd_w, c.fd_h);
          bool ok = k < ke && m0 + aq < c.M;
          const int64_t off = a_offset<MODE>(c, p, mtap[0], ok);
          ha[i] = *reinterpret_cast<const u32x4_*>(c.a16 + off);
          amask |= (ok ? 1u : 0u) << i;
        }
      }
#pragma unroll
      for (int i = 0; i < VB; ++i) {
        const int vi = tid + i * NT;
        const int64_t k = k0 + vi / (BN / EU), n = n0 + (vi % (BN / EU)) * EU;
        const unsigned short* q = c.b16 + (k < ke ? k : ke - 1) * c.Nn;
        hb[i] = *reinterpret_cast<const u32x4_*>(q + (n < c.Nn ? n : c.Nn - 8));
        bmask |= (k < ke ? 1u : 0u) << i;
      }
      return;
    }
    if (AKC) {   // 4 consecutive k = (kh, kw, ch .. ch+3) of one pixel row
      const int64_t k = k0 + aq;
      if (VEC) {
        const Tap t = split_tap(k < ke ? k : 0, c.fd_c, c.fd_kw);
        if constexpr (UNPOOL) psub = 0;
#pragma unroll
        for (int i = 0; i < VA; ++i) {
          bool ok = k < ke;
          const int64_t off = a_offset<MODE>(c, prow[i], t, ok);
          if constexpr (UNPOOL) {
            // the dY pixel of this tap (stride 1: ho = h + ph - kh, wo = w + pw - kw), its pooled row
            // pixel / 4 and window slot pixel % 4
            const int64_t pix =
                ok ? ((int64_t)prow[i].n * c.Ho + (prow[i].a + c.ph - t.kh)) * c.Wo + (prow[i].b + c.pw - t.kw) : 0;
            const int64_t po = (pix >> 2) * c.Co + t.ch;
            ra[i] = ld4(Asrc + po);
            parg[i] = *reinterpret_cast<const unsigned*>(c.dy_arg + po);
            psub |= (unsigned)(pix & 3) << (2 * i);
          } else {
            ra[i] = ld4(Asrc + off);
          }
          (void)off;
          amask |= (ok ? 0xFu : 0u) << (4 * i);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t ke_ = k + e;
          const Tap t = split_tap(ke_ < ke ? ke_ : 0, c.fd_c, c.fd_kw);
#pragma unroll
          for (int i = 0; i < VA; ++i) {
            bool ok = ke_ < ke;
            const int64_t off = a_offset<MODE>(c, prow[i], t, ok);
            ra[i][e] = Asrc[off];
            amask |= (ok ? 1u : 0u) << (4 * i + e);
          }
        }
      }
    } else {     // wgrad: 4 consecutive taps m (channels ch .. ch+3) at pixel k
#pragma unroll
      for (int i = 0; i < VA; ++i) {
        const int64_t k = k0 + (tid + i * NT) / (BM / 4);
        const Pix p = split_pix(k < ke ? k : 0, c.K, c.fd_w, c.fd_h);
        if (VEC) {
          bool ok = k < ke && m0 + aq < c.M;
          const int64_t off = a_offset<MODE>(c, p, mtap[0], ok);
          ra[i] = ld4(Asrc + off);
          amask |= (ok ? 0xFu : 0u) << (4 * i);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            bool ok = k < ke && m0 + aq + e < c.M;
            const int64_t off = a_offset<MODE>(c, p, mtap[e], ok);
            ra[i][e] = Asrc[off];
            amask |= (ok ? 1u : 0u) << (4 * i + e);
          }
        }
      }
    }
    // B [K][N] row-major, float4 along n: rows clamped (k >= ke zeroed at store), columns clamped
    // (columns >= N only feed output columns that are never stored)
    if constexpr (UNPOOL && MODE == kWgrad) {
      psub = 0;
#pragma unroll
      for (int i = 0; i < VB; ++i) {
        const int vi = tid + i * NT;
        const int64_t k = k0 + vi / (BN / 4), n = n0 + (vi % (BN / 4)) * 4;
        const int64_t kk = k < ke ? k : ke - 1;   // the dY pixel
        const int64_t po = (kk >> 2) * c.Nn + (n < c.Nn ? n : c.Nn - 4);
        rb[i] = ld4(Bsrc + po);
        parg[i] = *reinterpret_cast<const unsigned*>(c.dy_arg + po);
        psub |= (unsigned)(kk & 3) << (2 * i);
        bmask |= (k < ke ? 1u : 0u) << i;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < VB; ++i) {
      const int vi = tid + i * NT;
      const int64_t k = k0 + vi / (BN / 4), n = n0 + (vi % (BN / 4)) * 4;
      const float* q = Bsrc + (k < ke ? k : ke - 1) * c.Nn;
      if (VECB) {
        rb[i] = ld4(q + (n < c.Nn ? n : c.Nn - 4));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) rb[i][e] = q[n + e < c.Nn ? n + e : c.Nn - 1];
      }
      bmask |= (k < ke ? 1u : 0u) << i;
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // wgrad bias gradient: every staged B unit of a thread sits at the same 4 columns
  // n0 + (tid % (BN / 4)) * 4 (NT is a multiple of BN / 4); one m row of tiles sums them
  const bool csum_on = MODE == kWgrad && !S16 && c.colsum_part != nullptr && tm == 0;
  v4f csum = {0.f, 0.f, 0.f, 0.f};

  auto store_tile = [&](int buf) {
    if constexpr (UNPOOL) {   // rebuild the dense dY values: keep element e where its window argmax is this pixel
      if constexpr (MODE == kDgrad) {
#pragma unroll
        for (int i = 0; i < VA; ++i) {
          const unsigned sub = (psub >> (2 * i)) & 3u;
#pragma unroll
          for (int e = 0; e < 4; ++e) ra[i][e] = ((parg[i] >> (8 * e)) & 0xFFu) == sub ? ra[i][e] : 0.f;
        }
      } else {
#pragma unroll
        for (int i = 0; i < VB; ++i) {
          const unsigned sub = (psub >> (2 * i)) & 3u;
#pragma unroll
          for (int e = 0; e < 4; ++e) rb[i][e] = ((parg[i] >> (8 * e)) & 0xFFu) == sub ? rb[i][e] : 0.f;
        }
      }
    }
    if constexpr (S16) {
      unsigned short* As = reinterpret_cast<unsigned short*>(smem + buf * STAGE_FLOATS);
      unsigned short* Bs = As + JA::ELEMS;
      const u32x4_ z = {0u, 0u, 0u, 0u};
      if (AKC && c.fast16) {   // zeros came from the loads
#pragma unroll
        for (int i = 0; i < VA; ++i) *reinterpret_cast<u32x4_*>(As + JA::store_off8(tid + i * NT)) = ha[i];
#pragma unroll
        for (int i = 0; i < VB; ++i) *reinterpret_cast<u32x4_*>(Bs + JB::store_off8(tid + i * NT)) = hb[i];
        return;
      }
#pragma unroll
      for (int i = 0; i < VA; ++i)
        *reinterpret_cast<u32x4_*>(As + JA::store_off8(tid + i * NT)) = (amask >> i) & 1u ? ha[i] : z;
#pragma unroll
      for (int i = 0; i < VB; ++i)
        *reinterpret_cast<u32x4_*>(Bs + JB::store_off8(tid + i * NT)) = (bmask >> i) & 1u ? hb[i] : z;
      return;
    }
    if constexpr (LP != 0) {
      using E4 = typename ConvLp<LP>::e4;
      unsigned short* As = reinterpret_cast<unsigned short*>(smem + buf * STAGE_FLOATS);
      unsigned short* Bs = As + JA::ELEMS;
#pragma unroll
      for (int i = 0; i < VA; ++i) {
        v4f v = ra[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (amask >> (4 * i + e)) & 1u ? v[e] : 0.f;
        *reinterpret_cast<u32x2_*>(As + JA::store_off(tid + i * NT)) =
            __builtin_bit_cast(u32x2_, __builtin_convertvector(v, E4));
      }
#pragma unroll
      for (int i = 0; i < VB; ++i) {
        const v4f v = (bmask >> i) & 1u ? rb[i] : v4f{0.f, 0.f, 0.f, 0.f};
        if (csum_on) csum += v;   // the unrounded fp32 values, as the GEMMs' fused row sums
        *reinterpret_cast<u32x2_*>(Bs + JB::store_off(tid + i * NT)) =
            __builtin_bit_cast(u32x2_, __builtin_convertvector(v, E4));
      }
      return;
    }
    float* As = smem + buf * (IA::FLOATS + IB::FLOATS);
    float* Bs = As + IA::FLOATS;
#pragma unroll
    for (int i = 0; i < VA; ++i) {
      v4f v = ra[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (amask >> (4 * i + e)) & 1u ? v[e] : 0.f;
      st4(As + IA::store_off(tid + i * NT), v);
    }
#pragma unroll
    for (int i = 0; i < VB; ++i) {
      const v4f v = (bmask >> i) & 1u ? rb[i] : v4f{0.f, 0.f, 0.f, 0.f};
      if (csum_on) csum += v;
      st4(Bs + IB::store_off(tid + i * NT), v);
    }
  };
  // 16-bit stage: BK / 16 k-steps, fragments of the next step read ahead of this step's MFMAs
  auto mma_lp = [&](int buf) {
    const unsigned short* As = reinterpret_cast<const unsigned short*>(smem + buf * STAGE_FLOATS);
    const unsigned short* Bs = As + JA::ELEMS;
    u32x4_ fa[2][TM], fb[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[0][i] = JA::frag(As, wm0 + i * 32, 0, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[0][j] = JB::frag(Bs, wn0 + j * 32, 0, lane);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int cb = ks & 1;
      if (ks + 1 < BK / 16) {
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[cb ^ 1][i] = JA::frag(As, wm0 + i * 32, 16 * (ks + 1), lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[cb ^ 1][j] = JB::frag(Bs, wn0 + j * 32, 16 * (ks + 1), lane);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = ConvLp<LP == 0 ? 1 : LP>::mma(fa[cb][i], fb[cb][j], acc[i][j]);
    }
  };

  const int64_t nk = ke > kb0 ? (ke - kb0 + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tile(kb0);
    store_tile(0);
  }
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = (int)(kt & 1);
    if (kt + 1 < nk) load_tile(kb0 + (kt + 1) * BK);
    if constexpr (LP != 0) {
      mma_lp(cur);
    } else {
      const float* As = smem + cur * (IA::FLOATS + IB::FLOATS);
      mma_stage<IA, IB, TM, TN, BK>(As, As + IA::FLOATS, acc, wm0, wn0, lane);
    }
    asm volatile("" ::: "memory");      // keep the stage-k+1 LDS store (and its vmcnt wait)
    __builtin_amdgcn_sched_barrier(0);   // after this stage's MFMAs
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  if (csum_on) {
    // the 256 / (BN / 4) threads of each column quad, added through LDS in thread order (fixed)
    constexpr int Q = BN / 4, G = NT / Q;
    float* red = smem;   // the k loop ended with a barrier: the stage buffers are free
    *reinterpret_cast<v4f*>(red + 4 * tid) = csum;
    __syncthreads();
    if (tid < Q) {
      v4f t = *reinterpret_cast<const v4f*>(red + 4 * tid);
#pragma unroll
      for (int g = 1; g < G; ++g) t += *reinterpret_cast<const v4f*>(red + 4 * (tid + g * Q));
      const int64_t n = n0 + 4 * tid;
      if (n < c.Nn) *reinterpret_cast<v4f*>(c.colsum_part + split * c.Nn + n) = t;
    }
  }

  const int lh = lane >> 5, lc = lane & 31;
  if (MODE == kFwd && c.pool_w == 4) {
    // pooled epilogue (no split-K): the 4 rows (r & 3) = 0..3 of an accumulator group are 4
    // consecutive output columns of one output row (rows m0 + wm0 + 32 i + 8 (r >> 2) + 4 lh are
    // multiples of 4 and Wo % 4 == 0) — the window max and its first-maximum argmax in registers
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int64_t col = n0 + wn0 + j * 32 + lc;
        if (col >= c.Nn) continue;
        const float bv = c.bias ? c.bias[col] : 0.f;
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
          const int64_t row = m0 + wm0 + i * 32 + 8 * rq + 4 * lh;
          if (row >= c.M) continue;
          float best = acc[i][j][4 * rq] + bv;
          int arg = 0;
#pragma unroll
          for (int p = 1; p < 4; ++p) {
            const float v = acc[i][j][4 * rq + p] + bv;
            if (v > best || (v != v && best == best)) { best = v; arg = p; }
          }
          c.out[(row >> 2) * c.Nn + col] = best;
          c.pool_arg[(row >> 2) * c.Nn + col] = (uint8_t)arg;
        }
      }
    }
    return;
  }
  // epilogue.  32x32 accumulator: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t col = n0 + wn0 + j * 32 + lc;
      if (col >= c.Nn) continue;
      const float bv = (MODE == kFwd && c.bias && !c.partial) ? c.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= c.M) continue;
        if (c.partial) c.partial[((int64_t)split * c.M + row) * c.Nn + col] = acc[i][j][r];
        else c.out[row * c.Nn + col] = acc[i][j][r] + bv;
      }
    }
  }
}

__global__ void splitk_sum_kernel(const float* __restrict__ partial, int splits, int64_t n, int64_t ncol,
                                  const float* __restrict__ bias, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
#pragma unroll 8   // loads ahead of the in-order adds: the weight-gradient slabs are few threads x many splits
  for (int k = 0; k < splits; ++k) s += partial[(int64_t)k * n + i];
  out[i] = bias ? s + bias[i % ncol] : s;
}

// The same reduction for many splits (the weight gradients' deep split-K: up to 256 slabs of a few hundred
// thousand outputs, where one thread per output walking every split is latency-bound — cfg3 bf16: 218 us per
// step over 5 launches, r05u): a block = 8 waves x 64 lanes over 256 outputs (a float4 per lane), wave w adds
// the splits [w S / 8, (w + 1) S / 8) in order, then the 8 wave partials are added in wave order through LDS.
// Deterministic; n % 4 == 0 and 16-B aligned slabs (the host checks).
__global__ __launch_bounds__(512) void splitk_sum8_kernel(const float* __restrict__ partial, int splits, int64_t n,
                                                          int64_t ncol, const float* __restrict__ bias,
                                                          float* __restrict__ out) {
  __shared__ v4f red[8][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i4 = ((int64_t)blockIdx.x * 64 + lane) * 4;
  const int per = (splits + 7) / 8, k0 = min(splits, w * per), k1 = min(splits, k0 + per);
  v4f s = {0.f, 0.f, 0.f, 0.f};
  if (i4 < n) {
#pragma unroll 8
    for (int k = k0; k < k1; ++k) s += *reinterpret_cast<const v4f*>(partial + (int64_t)k * n + i4);
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && i4 < n) {
    v4f t = red[0][lane];
#pragma unroll
    for (int q = 1; q < 8; ++q) t += red[q][lane];
    if (bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] += bias[(i4 + e) % ncol];
    }
    *reinterpret_cast<v4f*>(out + i4) = t;
  }
}

// splitk_sum_kernel or, for >= 16 splits of a 4-aligned slab, splitk_sum8_kernel
void launch_splitk_sum(const float* partial, int splits, int64_t n, int64_t ncol, const float* bias, float* out,
                       hipStream_t s) {
  if (splits >= 16 && n % 4 == 0 && (uintptr_t)partial % 16 == 0 && (uintptr_t)out % 16 == 0)
    hipLaunchKernelGGL(splitk_sum8_kernel, dim3((unsigned)((n / 4 + 63) / 64)), dim3(512), 0, s, partial, splits, n,
                       ncol, bias, out);
  else
    hipLaunchKernelGGL(splitk_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, partial, splits, n,
                       ncol, bias, out);
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
// accumulate: dw += (the parameter's .grad, autograd's accumulation fused here) instead of dw =
__global__ void weight_grad_layout_kernel(const float* __restrict__ dwt, int Co, int Ci, int KH, int KW,
                                          float* __restrict__ dw, int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)Co * Ci * KH * KW;
  if (i >= n) return;
  const int kw = (int)(i % KW);
  int64_t t = i / KW;
  const int kh = (int)(t % KH);
  t /= KH;
  const int ci = (int)(t % Ci), co = (int)(t / Ci);
  const float v = dwt[(((int64_t)kh * KW + kw) * Ci + ci) * Co + co];
  dw[i] = accumulate ? dw[i] + v : v;
}

// ------------------------------------------------------------------ max pooling (NHWC)
// window = stride = (kh, kw), floor mode (nn.MaxPool2d((1,3)), MaxPool1d(98) as (98,1)).
// Backward routes each output gradient to the FIRST maximum of its window (PyTorch's rule); a
// NaN wins its window.  One thread = 4 consecutive channels of one output pixel (16-B accesses;
// C % 4 == 0 — every pooled layer of the reference models).
__device__ __forceinline__ bool takes(float v, float m, bool first) { return first || v > m || (v != v && m == m); }

__global__ void maxpool_fwd_kernel(const float* __restrict__ x, int N, int H, int W, int C, int kh, int kw,
                                   float* __restrict__ y) {
  const int Ho = H / kh, Wo = W / kw, C4 = C / 4;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n_out = (int64_t)N * Ho * Wo * C4;
  if (i >= n_out) return;
  const int c = (int)(i % C4) * 4;
  int64_t t = i / C4;
  const int wo = (int)(t % Wo);
  t /= Wo;
  const int ho = (int)(t % Ho), n = (int)(t / Ho);
  v4f m = {0.f, 0.f, 0.f, 0.f};
  bool first = true;
  for (int a = 0; a < kh; ++a)
    for (int b = 0; b < kw; ++b) {
      const v4f v = ld4(x + (((int64_t)n * H + ho * kh + a) * W + wo * kw + b) * C + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = takes(v[e], m[e], first) ? v[e] : m[e];
      first = false;
    }
  st4(y + i * 4, m);
}

__global__ void maxpool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, int N, int H, int W,
                                   int C, int kh, int kw, float* __restrict__ dx) {
  const int Ho = H / kh, Wo = W / kw, C4 = C / 4;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n_out = (int64_t)N * Ho * Wo * C4;
  if (i >= n_out) return;
  const int c = (int)(i % C4) * 4;
  int64_t t = i / C4;
  const int wo = (int)(t % Wo);
  t /= Wo;
  const int ho = (int)(t % Ho), n = (int)(t / Ho);
  v4f m = {0.f, 0.f, 0.f, 0.f};
  int arg[4] = {0, 0, 0, 0};
  bool first = true;
  for (int a = 0; a < kh; ++a)
    for (int b = 0; b < kw; ++b) {
      const v4f v = ld4(x + (((int64_t)n * H + ho * kh + a) * W + wo * kw + b) * C + c);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (takes(v[e], m[e], first)) { m[e] = v[e]; arg[e] = a * kw + b; }
      first = false;
    }
  const v4f g = ld4(dy + i * 4);
  for (int a = 0; a < kh; ++a)
    for (int b = 0; b < kw; ++b) {
      const int q = a * kw + b;
      v4f o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = arg[e] == q ? g[e] : 0.f;
      st4(dx + (((int64_t)n * H + ho * kh + a) * W + wo * kw + b) * C + c, o);
    }
}

// db[n] = sum over splits (in order) of the wgrad kernel's column-sum partials
__global__ void colsum_splits_kernel(const float* __restrict__ part, int splits, int64_t n, float* __restrict__ db) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
#pragma unroll 8   // loads ahead of the in-order adds (not one dependent load latency per split)
  for (int k = 0; k < splits; ++k) s += part[(int64_t)k * n + i];
  db[i] = s;
}

// window (1, kw) max + first-maximum argmax of a dense NHWC activation (the pooled conv's split-K
// path; the argmax matches the fused epilogue's and maxpool_bwd_kernel's rule)
__global__ void maxpool_arg_kernel(const float* __restrict__ x, int64_t rows_out, int C, int kw, float* __restrict__ y,
                                   uint8_t* __restrict__ arg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows_out * C) return;
  const int64_t r = i / C;
  const int c = (int)(i - r * C);
  float m = 0.f;
  int a = 0;
  for (int b = 0; b < kw; ++b) {
    const float v = x[(r * kw + b) * C + c];
    if (takes(v, m, b == 0)) { m = v; a = b; }
  }
  y[i] = m;
  arg[i] = (uint8_t)a;
}

// dense gradient of a (1, kw) max-pool from the pooled gradient and the window argmax:
// dx[(r, b), c] = arg[r, c] == b ? dy[r, c] : 0 (4 channels per thread)
__global__ void unpool_kernel(const float* __restrict__ dy, const uint8_t* __restrict__ arg, int64_t rows_out, int C,
                              int kw, float* __restrict__ dx) {
  const int C4 = C / 4;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows_out * C4) return;
  const int64_t r = i / C4;
  const int c = (int)(i - r * C4) * 4;
  const v4f g = ld4(dy + r * C + c);
  const unsigned a = *reinterpret_cast<const unsigned*>(arg + r * C + c);
  for (int b = 0; b < kw; ++b) {
    v4f o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = ((a >> (8 * e)) & 0xFFu) == (unsigned)b ? g[e] : 0.f;
    st4(dx + (r * kw + b) * C + c, o);
  }
}

// 16-bit modes: the dense data gradient of a pooled conv written straight as the 16-bit operand copy
// the S16 gathers read (8 channels per thread: one 16-B store per window position), rounded by the
// same conversion as to16_kernel — so the operands are bitwise those of unpool + to16, without the
// dense fp32 gradient (N Ho Wo Co x 4 B written and read back twice: conversion and bias sums)
template <int LP>
__global__ void unpool16_kernel(const float* __restrict__ dy, const uint8_t* __restrict__ arg, int64_t rows_out, int C,
                                int kw, unsigned short* __restrict__ dx16) {
  const int C8 = C / 8;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows_out * C8) return;
  const int64_t r = i / C8;
  const int c = (int)(i - r * C8) * 8;
  const v4f g0 = ld4(dy + r * C + c), g1 = ld4(dy + r * C + c + 4);
  typedef unsigned u32x2a __attribute__((ext_vector_type(2)));
  const u32x2a a = *reinterpret_cast<const u32x2a*>(arg + r * C + c);
  using E4 = typename ConvLp<LP>::e4;
  for (int b = 0; b < kw; ++b) {
    v4f o0, o1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o0[e] = ((a.x >> (8 * e)) & 0xFFu) == (unsigned)b ? g0[e] : 0.f;
      o1[e] = ((a.y >> (8 * e)) & 0xFFu) == (unsigned)b ? g1[e] : 0.f;
    }
    const u32x2_ lo = __builtin_bit_cast(u32x2_, __builtin_convertvector(o0, E4));
    const u32x2_ hi = __builtin_bit_cast(u32x2_, __builtin_convertvector(o1, E4));
    *reinterpret_cast<u32x4_*>(dx16 + (r * kw + b) * C + c) = u32x4_{lo.x, lo.y, hi.x, hi.y};
  }
}

__global__ void zero_kernel(float* __restrict__ p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

// fp32 -> 16-bit operand copy, 8 elements per thread, by the same conversion the LDS-store path
// applies (so S16 operands are bit-identical to the fp32-source LP path's)
template <int LP>
__global__ void to16_kernel(const float* __restrict__ x, int64_t n8, unsigned short* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  using E4 = typename ConvLp<LP>::e4;
  const u32x2_ lo = __builtin_bit_cast(u32x2_, __builtin_convertvector(ld4(x + 8 * i), E4));
  const u32x2_ hi = __builtin_bit_cast(u32x2_, __builtin_convertvector(ld4(x + 8 * i + 4), E4));
  *reinterpret_cast<u32x4_*>(y + 8 * i) = u32x4_{lo.x, lo.y, hi.x, hi.y};
}

// Column sums of a [rows, C] fp32 matrix (C % 8 == 0, 256 % (C / 8) == 0) fused into the one pass that
// already reads it — the conv bias gradient db = sum over pixels of dY (model_fbanks_cnn.py's conv
// biases) in 16-bit modes, where the weight-gradient GEMM reads only dY's 16-bit copy.  Thread = (row
// lane, 8-channel octet): 16-B loads, four rows' loads issued before their adds, each thread adding its
// rows in row order; the row lanes of an octet are then added through LDS in lane order and one partial
// row [C] per block goes to `part`; colsum_blocks_kernel adds the blocks in block order (deterministic).
// KIND 0: the sums only; 1: + the 16-bit operand copy y16 = round(x) (to16_kernel's conversion);
// 2: x is a (1, kw)-pooled gradient: + its unpooled dense 16-bit copy through the argmax (unpool16_kernel's
// stores; each pooled value sits once in the dense gradient, so its column sums are the bias gradient).
template <int LP, int KIND>
__global__ __launch_bounds__(256) void colsum8_kernel(const float* __restrict__ x, const uint8_t* __restrict__ arg,
                                                      int64_t rows, int C, int kw, int64_t rows_per_block,
                                                      unsigned short* __restrict__ y16, float* __restrict__ part) {
  __shared__ float red[256 * 8];
  const int C8 = C >> 3, RL = 256 / C8;
  const int q = threadIdx.x % C8, rl = threadIdx.x / C8;
  const int c = q * 8;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
  using E4 = typename ConvLp<LP == 0 ? 1 : LP>::e4;
  typedef unsigned u32x2a __attribute__((ext_vector_type(2)));
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto body = [&](int64_t r, const v4f& g0, const v4f& g1) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[e] += g0[e];
      acc[4 + e] += g1[e];
    }
    if (KIND == 1) {
      const u32x2_ lo = __builtin_bit_cast(u32x2_, __builtin_convertvector(g0, E4));
      const u32x2_ hi = __builtin_bit_cast(u32x2_, __builtin_convertvector(g1, E4));
      *reinterpret_cast<u32x4_*>(y16 + r * C + c) = u32x4_{lo.x, lo.y, hi.x, hi.y};
    } else if (KIND == 2) {
      const u32x2a a = *reinterpret_cast<const u32x2a*>(arg + r * C + c);
      for (int b = 0; b < kw; ++b) {
        v4f o0, o1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o0[e] = ((a.x >> (8 * e)) & 0xFFu) == (unsigned)b ? g0[e] : 0.f;
          o1[e] = ((a.y >> (8 * e)) & 0xFFu) == (unsigned)b ? g1[e] : 0.f;
        }
        const u32x2_ lo = __builtin_bit_cast(u32x2_, __builtin_convertvector(o0, E4));
        const u32x2_ hi = __builtin_bit_cast(u32x2_, __builtin_convertvector(o1, E4));
        *reinterpret_cast<u32x4_*>(y16 + (r * kw + b) * C + c) = u32x4_{lo.x, lo.y, hi.x, hi.y};
      }
    }
  };
  int64_t r = r0 + rl;
  for (; r + 3 * RL < r1; r += 4 * RL) {   // four rows' loads in flight, then their adds in row order
    v4f g[4][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      g[u][0] = ld4(x + (r + u * RL) * C + c);
      g[u][1] = ld4(x + (r + u * RL) * C + c + 4);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) body(r + u * RL, g[u][0], g[u][1]);
  }
  for (; r < r1; r += RL) body(r, ld4(x + r * C + c), ld4(x + r * C + c + 4));
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl * C + c + e] = acc[e];
  __syncthreads();
  for (int cc = threadIdx.x; cc < C; cc += 256) {
    float t = 0.f;
    for (int l = 0; l < RL; ++l) t += red[l * C + cc];
    part[(int64_t)blockIdx.x * C + cc] = t;
  }
}

// out[c] = sum over the nblk partial rows, in a fixed order: workgroup = 64 columns (lane = column) x 16
// waves, wave w adds its contiguous run of blocks with 8 loads in flight, then the 16 wave sums are added in
// wave order.  (One lane walking ~2,000 blocks one dependent load at a time took 400-700 us: r05c, cfg3 bf16.)
constexpr int kCsWaves = 16;
__global__ __launch_bounds__(64 * kCsWaves) void colsum_blocks_kernel(const float* __restrict__ part, int nblk, int C,
                                                                      float* __restrict__ out) {
  __shared__ float red[kCsWaves][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int run = (nblk + kCsWaves - 1) / kCsWaves;
  const int b0 = wave * run, b1 = min(nblk, b0 + run);
  float t = 0.f;
  if (c < C) {
    int b = b0;
    for (; b + 8 <= b1; b += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(b + u) * C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) t += v[u];
    }
    for (; b < b1; ++b) t += part[(int64_t)b * C + c];
  }
  red[wave][lane] = t;
  __syncthreads();
  if (wave == 0 && c < C) {
    float a = red[0][lane];
#pragma unroll
    for (int w = 1; w < kCsWaves; ++w) a += red[w][lane];
    out[c] = a;
  }
}

struct ConvScratch {
  float* p = nullptr;
  size_t floats = 0;
};
ConvScratch g_cs[64];     // split-K slabs
ConvScratch g_cs16[64];   // 16-bit operand sources
ConvScratch g_csb[64];    // wgrad bias column-sum partials
ConvScratch g_csd[64];    // dense activation / gradient of the pooled conv (split-K forward, backward dY)
ConvScratch g_csy[64];    // conv_bwd: dY's 16-bit copy made with the bias sums (dY itself may sit in g_csd)
std::mutex g_cs_mu;

int conv_scratch(size_t floats, float** out, ConvScratch* pool = g_cs) {
  int dev = 0;
  SRK_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_cs_mu);
  ConvScratch& s = pool[dev & 63];
  if (s.floats < floats) {
    if (s.p) {
      SRK_CHECK_HIP(hipDeviceSynchronize());
      SRK_CHECK_HIP(hipFree(s.p));
    }
    s.floats = floats + floats / 4;
    SRK_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&s.p), s.floats * sizeof(float)));
    g_scratch_gen.fetch_add(1);
  }
  *out = s.p;
  return SRK_OK;
}

// 16-bit sources (ConvArgs::a16 / b16) for matmul_precision bf16 / fp16 when every channel count is
// a multiple of 8 and the fp32 tensors are 16-B aligned (option "conv16_sources", default on).
bool s16_ok(int prec, int64_t Ci, int64_t Co, std::initializer_list<const void*> ptrs) {
  if (!g_opt_conv16_sources || prec == kPrecF32 || Ci % 8 || Co % 8) return false;
  for (const void* p : ptrs)
    if (reinterpret_cast<uintptr_t>(p) % 16) return false;
  return true;
}

// rounds cnt fp32 tensors (n[i] % 8 == 0 elements each) into 16-bit copies, on s.  dst[i] null on
// entry: a slice of one scratch allocation; preset: caller storage, converted into unless ready[i]
// (it already holds this tensor's copy, e.g. the one srk_conv2d_nhwc_fwd16 kept for the backward).
int to16_all(int prec, const float* const* src, const int64_t* n, int cnt, unsigned short** dst, hipStream_t s,
             const bool* ready = nullptr) {
  size_t off[4], total = 0;
  double bytes = 0;
  for (int i = 0; i < cnt; ++i) {
    off[i] = total;
    if (!dst[i]) total += (size_t)((n[i] + 63) / 64 * 64);
    if (!(ready && ready[i])) bytes += 6.0 * (double)n[i];
  }
  float* base = nullptr;
  if (total) {
    if (int rc = conv_scratch((total + 1) / 2, &base, g_cs16)) return rc;
  }
  ProfScope prof("conv_to16", s, bytes);
  for (int i = 0; i < cnt; ++i) {
    if (ready && ready[i]) continue;
    if (!dst[i]) dst[i] = reinterpret_cast<unsigned short*>(base) + off[i];
    const int64_t n8 = n[i] / 8;
    SRK_REQUIRE(n[i] % 8 == 0 && (n8 + 255) / 256 < INT32_MAX, SRK_ERR_INTERNAL, "conv: bad 16-bit source size");
    const dim3 grid((unsigned)((n8 + 255) / 256));
    if (prec == kPrecBF16) hipLaunchKernelGGL(to16_kernel<1>, grid, dim3(256), 0, s, src[i], n8, dst[i]);
    else hipLaunchKernelGGL(to16_kernel<2>, grid, dim3(256), 0, s, src[i], n8, dst[i]);
  }
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

bool colsum8_ok(int64_t C) { return g_opt_conv_colsum16 && C % 8 == 0 && C <= 2048 && 256 % (C / 8) == 0; }

// out[C] = column sums of x [rows, C] (colsum8_kernel; colsum8_ok(C)), fused with the 16-bit copy (kind 1) or
// the unpooled 16-bit copy through arg (kind 2) at precision prec
int colsum8(int kind, int prec, const float* x, const uint8_t* arg, int64_t rows, int C, int kw, unsigned short* y16,
            float* out, hipStream_t s) {
  const int RL = 256 / (C / 8);
  int64_t nblk = std::min<int64_t>((rows + RL - 1) / RL, 2048);
  int64_t per = (rows + nblk - 1) / nblk;
  per = (per + RL - 1) / RL * RL;
  nblk = (rows + per - 1) / per;
  float* part = nullptr;
  if (int rc = conv_scratch((size_t)nblk * C, &part, g_csb)) return rc;
  const double bytes = (double)rows * C * (4.0 + (kind == 1 ? 2.0 : kind == 2 ? 1.0 + 2.0 * kw : 0.0));
  ProfScope prof(kind == 0 ? "conv_colsum" : kind == 1 ? "conv_to16_colsum" : "conv_unpool16_colsum", s, bytes);
  const dim3 grid((unsigned)nblk), block(256);
#define SRK_CS8(LP_, K_) hipLaunchKernelGGL((colsum8_kernel<LP_, K_>), grid, block, 0, s, x, arg, rows, C, kw, per, y16, part)
  if (kind == 0) SRK_CS8(0, 0);
  else if (prec == kPrecBF16) { if (kind == 1) SRK_CS8(1, 1); else SRK_CS8(1, 2); }
  else { if (kind == 1) SRK_CS8(2, 1); else SRK_CS8(2, 2); }
#undef SRK_CS8
  hipLaunchKernelGGL(colsum_blocks_kernel, dim3((unsigned)((C + 63) / 64)), dim3(64 * kCsWaves), 0, s, part, (int)nblk,
                     C, out);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

template <int MODE, int BM, int BN, int BK, int LP, int NW>
void launch_conv_p(const ConvArgs& c, dim3 grid, hipStream_t s, bool vec, bool vecb) {
  const dim3 block(NW * 64);
  if constexpr (MODE != kFwd) {
    if (c.dy_arg) {   // run_conv_gemm checked vec / vecb and fp32 sources
      hipLaunchKernelGGL((conv_gemm_kernel<MODE, BM, BN, BK, true, true, LP, false, true, NW>), grid, block, 0, s, c);
      return;
    }
  }
  if constexpr (LP != 0) {
    if (c.a16) {
      hipLaunchKernelGGL((conv_gemm_kernel<MODE, BM, BN, BK, true, true, LP, true, false, NW>), grid, block, 0, s, c);
      return;
    }
  }
  if constexpr (NW == 8) {   // 8-wave tiles are only chosen with vector gathers (run_conv_gemm)
    hipLaunchKernelGGL((conv_gemm_kernel<MODE, BM, BN, BK, true, true, LP, false, false, NW>), grid, block, 0, s, c);
  } else {
    if (vec && vecb) hipLaunchKernelGGL((conv_gemm_kernel<MODE, BM, BN, BK, true, true, LP>), grid, block, 0, s, c);
    else if (vecb) hipLaunchKernelGGL((conv_gemm_kernel<MODE, BM, BN, BK, false, true, LP>), grid, block, 0, s, c);
    else hipLaunchKernelGGL((conv_gemm_kernel<MODE, BM, BN, BK, false, false, LP>), grid, block, 0, s, c);
  }
}

template <int MODE, int BM, int BN, int NW = 4>
void launch_conv(const ConvArgs& c, dim3 grid, hipStream_t s, bool vec, bool vecb, int prec) {
  if constexpr (NW == 8) {   // the 8-wave 256-row tiles: fp32 operands only (run_conv_gemm)
    launch_conv_p<MODE, BM, BN, 32, 0, NW>(c, grid, s, vec, vecb);
  } else {
    if (prec == kPrecBF16) launch_conv_p<MODE, BM, BN, 64, 1, NW>(c, grid, s, vec, vecb);
    else if (prec == kPrecF16) launch_conv_p<MODE, BM, BN, 64, 2, NW>(c, grid, s, vec, vecb);
    else launch_conv_p<MODE, BM, BN, 32, 0, NW>(c, grid, s, vec, vecb);
  }
}

// ------------------------------------------------------------------ fp32 LDS-DMA ring conv (option conv_ring)
// The implicit GEMMs of stride-1 / channel-aligned convolutions on the structure of gemm_p32_kernel
// (gemm.hip): 256 x BN tiles (BN = 256 or 128), 8 waves in two groups running one section apart
// behind raw barriers, a ring of four 16-deep K-tiles filled by inline-asm buffer_load ... lds.  The
// only conv-specific part is the DMA source address: with the gathered operand's channel count a
// multiple of 16, a K-tile lies inside one tap (kh, kw), so per K-tile each lane recomputes its unit's
// source offset from its pixel (decomposed once per tile) and the uniform tap; a unit outside the
// image, past the problem or past the split's k end is read past num_records, i.e. as zeros.
//   fwd   A = X[n, a + kh - ph, b + kw - pw, ch..ch+3]       (KC: 4 channels of one pixel per unit)
//   dgrad A = dY[n, a + ph - kh, b + pw - kw, ch..ch+3]      (KC, stride 1)
//   wgrad A^T unit = X[pixel k (+ tap), ci..ci+3]           (TR: 4 channels at one pixel per unit)
//   B = the re-laid-out weights [K][N] (fwd / dgrad) or dY [pixels][Co] (wgrad): plain row-major
// Epilogue straight from the accumulators (the 96-KB ring of BN = 128 leaves no room to stage),
// with the (1, 4) pooled variant of conv_gemm_kernel (fwd) and the fused bias column sums (wgrad).
constexpr int kRBK = 16;
constexpr unsigned kROOB = 0x80000000u;

template <int MODE, int BN>
__global__ __launch_bounds__(512, 1) void conv_ring_kernel(ConvArgs c) {
  constexpr int BK = kRBK, NST = 4;
  constexpr bool AKC = MODE != kWgrad;
  constexpr int HALF = 128 * BK;                     // 8 KB of fp32 per 128-row half image
  constexpr int NBH = BN / 128;                      // B half images
  constexpr int STAGE = (2 + NBH) * HALF;
  constexpr int NDMA = 2 + NBH;                      // DMA instructions per wave per K-tile
  // wave layout in a group of 4: BN 256 -> 1 x 4 (128 x 64 each), BN 128 -> 2 x 2 (64 x 64 each)
  constexpr int WR = BN == 256 ? 1 : 2, WC = 4 / WR;
  constexpr int TM = 128 / WR / 32, TN = BN / WC / 32;
  __shared__ __attribute__((aligned(1024))) float smem[NST * STAGE];
  typedef __attribute__((address_space(3))) void* lds_ptr;
  typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
  auto bar = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, grp = wave >> 2, w4 = wave & 3;
  const int wr = w4 / WC, wc = w4 % WC;
  int split, tm, tn;
  map_tile(c.nblk, c.tiles, c.tiles_m, c.tiles_n, c.group_m, true, split, tm, tn);
  const int64_t m0 = (int64_t)tm * 256, n0 = (int64_t)tn * BN;
  const int64_t kb0 = split * c.kchunk;
  const int64_t ke = (kb0 + c.kchunk < c.K) ? kb0 + c.kchunk : c.K;
  const int nk = ke > kb0 ? (int)((ke - kb0 + BK - 1) / BK) : 0;
  const float* Asrc = MODE == kDgrad ? c.dy : c.x;
  const float* Bsrc = MODE == kWgrad ? c.dy : c.wmat;
  auto rsrc = [](const float* p) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    return u32x4s{(unsigned)__builtin_amdgcn_readfirstlane((unsigned)a),
                  (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)), 0x7ffffff0u, 0x00020000u};
  };
  const u32x4s rsA = rsrc(Asrc), rsB = rsrc(Bsrc);
  const int chans = MODE == kDgrad ? c.Co : c.Ci;   // channels of the gathered operand

  // this wave's piece of each A half: the unit (row or m group, k offset) it brings in
  const int p = wave * 64 + lane;
  int arow[2], akk[2];
  Pix apix[2];      // fwd / dgrad: the unit's pixel
  Tap atap[2];      // wgrad: the unit's (kh, kw, ci)
  bool aok[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (AKC) {   // p = row * 4 + slot, k = 4 (slot ^ swz(row))
      arow[h] = p >> 2;
      akk[h] = ((p & 3) ^ ((arow[h] >> 2) & 3)) * 4;
      apix[h] = split_pix(m0 + h * 128 + arow[h], c.M, c.fd_w, c.fd_h);
      aok[h] = apix[h].ok;
    } else {     // p = k * 32 + unit of 4 rows
      akk[h] = p >> 5;
      arow[h] = (p & 31) * 4;
      const int64_t m = m0 + h * 128 + arow[h];
      aok[h] = m < c.M;
      atap[h] = split_tap(aok[h] ? m : 0, c.fd_c, c.fd_kw);
    }
  }
  // B halves: p = k * 32 + unit of 4 columns (plain [K][N])
  unsigned bvo[NBH];
  bool bok[NBH];
  const int bkk = p >> 5;
#pragma unroll
  for (int h = 0; h < NBH; ++h) {
    const int64_t n = n0 + h * 128 + (p & 31) * 4;
    bok[h] = n < c.Nn;
    bvo[h] = (unsigned)(((int64_t)bkk * c.Nn + (bok[h] ? n : 0)) * 4);
  }
  const unsigned lds0 =
      (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ptr)smem + (unsigned)wave * 1024u);
  auto issue = [&](unsigned v, const u32x4s& rs, unsigned ldsa, unsigned soff) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(v), "s"(rs), "s"(ldsa), "s"(soff)
                 : "memory");
  };
  auto dma_a = [&](int t) {
    const int64_t k0 = kb0 + (int64_t)t * BK;
    const unsigned ldst = lds0 + (unsigned)((t % NST) * STAGE * 4);
    // fwd / dgrad: the K-tile's tap and channel base (uniform: chans % 16 == 0, k0 % 16 == 0)
    const unsigned tap = AKC ? (unsigned)__builtin_amdgcn_readfirstlane(c.fd_c.div((unsigned)k0)) : 0u;
    const int ch0 = (int)((unsigned)k0 - tap * (unsigned)chans);
    const int kh = (int)c.fd_kw.div(tap), kw = (int)(tap - (unsigned)kh * c.KW);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      unsigned v = kROOB;
      if (AKC) {
        const Pix& q = apix[h];
        int64_t off;
        bool ok;
        if (MODE == kFwd) {
          const int hi = q.a * c.sh + kh - c.ph, wi = q.b * c.sw + kw - c.pw;
          ok = hi >= 0 && hi < c.H && wi >= 0 && wi < c.W;
          off = (((int64_t)q.n * c.H + hi) * c.W + wi) * c.Ci + ch0 + akk[h];
        } else {
          const int ho = q.a + c.ph - kh, wo = q.b + c.pw - kw;
          ok = ho >= 0 && ho < c.Ho && wo >= 0 && wo < c.Wo;
          off = (((int64_t)q.n * c.Ho + ho) * c.Wo + wo) * c.Co + ch0 + akk[h];
        }
        if (aok[h] && ok && k0 + akk[h] < ke) v = (unsigned)(off * 4);
      } else {
        const int64_t k = k0 + akk[h];    // the unit's pixel (output grid)
        const Pix q = split_pix(k < ke ? k : 0, c.K, c.fd_w, c.fd_h);
        const Tap& t4 = atap[h];
        const int hi = q.a * c.sh + t4.kh - c.ph, wi = q.b * c.sw + t4.kw - c.pw;
        const bool ok = aok[h] && k < ke && hi >= 0 && hi < c.H && wi >= 0 && wi < c.W;
        if (ok) v = (unsigned)(((((int64_t)q.n * c.H + hi) * c.W + wi) * c.Ci + t4.ch) * 4);
      }
      issue(v, rsA, ldst + (unsigned)(h * HALF * 4), 0u);
    }
  };
  auto dma_b = [&](int t) {
    const int64_t k0 = kb0 + (int64_t)t * BK;
    const unsigned ldst = lds0 + (unsigned)((t % NST) * STAGE * 4);
    const unsigned soff = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(k0 * c.Nn * 4));
#pragma unroll
    for (int h = 0; h < NBH; ++h) {
      const unsigned v = (bok[h] && k0 + bkk < ke) ? bvo[h] : kROOB;
      issue(v, rsB, ldst + (unsigned)((2 + h) * HALF * 4), soff);
    }
  };
  auto retire_keep = [](int tiles_in_flight) {   // all but the youngest tiles (NDMA DMAs each)
    if (tiles_in_flight >= 2) {
      if (NDMA == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else if (tiles_in_flight == 1) {
      if (NDMA == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // wgrad bias sums: column sums of B from the B fragments of group 0 in the first tile row
  const bool do_cs = MODE == kWgrad && c.colsum_part != nullptr && tm == 0 && grp == 0 && wr == 0;
  float cs[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) cs[j] = 0.f;

  for (int t = 0; t < NST - 1; ++t)
    if (t < nk) {
      dma_a(t);
      dma_b(t);
    }
  retire_keep(min(nk - 1, NST - 2));
  bar();
  if (grp == 1) bar();

  // fragments: A rows grp * 128 + wr * (128 / WR) + i * 32 of half grp; B columns wc * (BN / WC) + j * 32
  const int ar0 = wr * (128 / WR);
  const int bh = (wc * (BN / WC)) / 128, bc0 = (wc * (BN / WC)) % 128;
  auto fragA = [&](const float* img, int r0, int kb) -> v4f {
    const int row = r0 + (lane & 31), h = lane >> 5;
    if (AKC) return *reinterpret_cast<const v4f*>(img + row * BK + (((2 * kb + h) ^ ((row >> 2) & 3)) << 2));
    const float* q = img + (8 * kb + 4 * h) * 128 + row;
    return v4f{q[0], q[128], q[256], q[384]};
  };
  auto fragB = [&](const float* img, int r0, int kb) -> v4f {
    const float* q = img + (8 * kb + 4 * (lane >> 5)) * 128 + r0 + (lane & 31);
    return v4f{q[0], q[128], q[256], q[384]};
  };
  for (int kt = 0; kt < nk; ++kt) {
    const float* S = smem + (kt % NST) * STAGE;
    const float* As = S + grp * HALF;
    const float* Bs = S + (2 + bh) * HALF;
    const int tn_ = kt + NST - 1;
#pragma unroll
    for (int q = 0; q < BK / 8; ++q) {
      v4f fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = fragA(As, ar0 + i * 32, q);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = fragB(Bs, bc0 + j * 32, q);
      if (tn_ < nk) {
        if (q == 0) dma_a(tn_);
        else dma_b(tn_);
      }
      if (q == BK / 8 - 1) retire_keep(min(nk - 1 - (kt + 1), NST - 2));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ss = 0; ss < 4; ++ss)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][ss], fb[j][ss], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (do_cs) {
#pragma unroll
        for (int j = 0; j < TN; ++j) cs[j] += (fb[j][0] + fb[j][1]) + (fb[j][2] + fb[j][3]);
      }
      bar();
    }
  }
  if (grp == 0) bar();

  // ---- epilogue from the accumulators (32x32: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5))
  const int lh = lane >> 5, lc = lane & 31;
  const int64_t rbase = m0 + grp * 128 + ar0;
  const int64_t cbase = n0 + bh * 128 + bc0;
  if (MODE == kFwd && c.pool_w == 4 && !c.partial) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int64_t col = cbase + j * 32 + lc;
        if (col >= c.Nn) continue;
        const float bv = c.bias ? c.bias[col] : 0.f;
#pragma unroll
        for (int rq = 0; rq < 4; ++rq) {
          const int64_t row = rbase + i * 32 + 8 * rq + 4 * lh;
          if (row >= c.M) continue;
          float best = acc[i][j][4 * rq] + bv;
          int arg = 0;
#pragma unroll
          for (int pp = 1; pp < 4; ++pp) {
            const float v = acc[i][j][4 * rq + pp] + bv;
            if (v > best || (v != v && best == best)) { best = v; arg = pp; }
          }
          c.out[(row >> 2) * c.Nn + col] = best;
          c.pool_arg[(row >> 2) * c.Nn + col] = (uint8_t)arg;
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int64_t col = cbase + j * 32 + lc;
        if (col >= c.Nn) continue;
        const float bv = (MODE == kFwd && c.bias && !c.partial) ? c.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t row = rbase + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (row >= c.M) continue;
          if (c.partial) c.partial[((int64_t)split * c.M + row) * c.Nn + col] = acc[i][j][r];
          else c.out[row * c.Nn + col] = acc[i][j][r] + bv;
        }
      }
  }
  if (do_cs) {   // lanes l and l + 32 hold the two k halves of column (l & 31)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float t = cs[j] + __shfl_xor(cs[j], 32);
      const int64_t col = cbase + j * 32 + lc;
      if (lane < 32 && col < c.Nn) c.colsum_part[(int64_t)split * c.Nn + col] = t;
    }
  }
}

// 16-bit form of the ring conv (bf16 / fp16 matmul precision with the 16-bit operand copies of the
// S16 path): gemm_g16_kernel's structure — 32-deep K-tiles of 16-bit units (8 elements = 16 B), KC
// images [128 rows][4 units] read by ds_read_b128, TR images [32 k][16 units] read by
// ds_read_b64_tr_b16, v_mfma_f32_32x32x16_{bf16,f16} — with the same per-K-tile conv gathers (the
// gathered operand's channel count a multiple of 32: a K-tile inside one tap).
constexpr int kR16BK = 32;
template <bool KC>
__device__ __forceinline__ int r16_off(int row, int k) {
  if (KC) return row * kR16BK + ((((k >> 3) ^ ((row >> 2) & 3))) << 3) + (k & 7);
  return k * 128 + ((((row >> 3) ^ ((k & 3) << 2))) << 3) + (row & 7);
}
template <bool KC>
__device__ __forceinline__ u32x4_ r16_frag(const unsigned short* img, int r0, int kk, int lane) {
  if (KC) return *reinterpret_cast<const u32x4_*>(img + r16_off<true>(r0 + (lane & 31), kk + 8 * (lane >> 5)));
  const int q = (lane >> 2) & 3, pp = lane & 3;
  const int k = kk + 8 * (lane >> 5) + q, row = r0 + 16 * ((lane >> 4) & 1) + 4 * pp;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + r16_off<false>(row, k)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + r16_off<false>(row, k + 4)));
  const u32x2_ l2 = __builtin_bit_cast(u32x2_, lo), h2 = __builtin_bit_cast(u32x2_, hi);
  return u32x4_{l2.x, l2.y, h2.x, h2.y};
}

// QS: k-steps (16 deep) per MFMA section: 1 = a barrier pair per k-step (BN / 32 MFMAs per wave
// between barriers), 2 = the whole 32-deep K-tile per section (twice the
// MFMAs per barrier pair, both DMAs issued in the one load section) — option conv_ring_qs
// NST: ring stages (4; up to 160 KB of LDS: 5 at BN = 256, 6 at BN <= 128).  Deeper rings measured slower on the
// cfg3 / cfg4 shapes (r05c: rn_l4 wgrad 486 -> 587 us at 5 stages), so only NST = 4 is instantiated.
template <int VM>
__device__ __forceinline__ void wait_vm() {
  static_assert(VM >= 0 && VM < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");
}
// Measured and dropped in round 5 (git history keeps them): a persistent tile loop running the ring across
// tiles, and 256 x 64 tiles for N = 64.
template <int MODE, int BN, int LP, int QS = 1, int NST = 4>
__global__ __launch_bounds__(512, 1) void conv_ring16_kernel(ConvArgs c) {
  constexpr int BK = kR16BK;
  constexpr bool AKC = MODE != kWgrad;
  constexpr int HALF = 128 * BK;                     // 8 KB of 16-bit elements per half image
  static_assert(BN == 128 || BN == 256, "ring16: 128- or 256-wide tiles");
  constexpr int NBH = BN / 128;
  constexpr int STAGE = (2 + NBH) * HALF;
  constexpr int NDMA = 2 + NBH;
  constexpr int WR = BN == 256 ? 1 : 2, WC = 4 / WR;
  constexpr int TM = 128 / WR / 32, TN = BN / WC / 32;
  __shared__ __attribute__((aligned(1024))) unsigned short smem[NST * STAGE];
  typedef __attribute__((address_space(3))) void* lds_ptr;
  typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
  auto bar = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, grp = wave >> 2, w4 = wave & 3;
  const int wr = w4 / WC, wc = w4 % WC;
  auto rsrc = [](const unsigned short* p) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    return u32x4s{(unsigned)__builtin_amdgcn_readfirstlane((unsigned)a),
                  (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)), 0x7ffffff0u, 0x00020000u};
  };
  const u32x4s rsA = rsrc(c.a16), rsB = rsrc(c.b16);
  const int chans = MODE == kDgrad ? c.Co : c.Ci;

  // this lane's DMA slots (fixed): A rows / k of the two half images, B k and columns
  const int p = wave * 64 + lane;
  int arow[2], akk[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (AKC) {   // p = row * 4 + slot: 8 k at 8 (slot ^ swz(row))
      arow[h] = p >> 2;
      akk[h] = ((p & 3) ^ ((arow[h] >> 2) & 3)) * 8;
    } else {     // p = k * 16 + slot: rows 8 (slot ^ ((k & 3) << 2)) .. +8
      akk[h] = p >> 4;
      arow[h] = ((p & 15) ^ ((akk[h] & 3) << 2)) * 8;
    }
  }
  const int bkk = p >> 4;
  // one tile's coordinates: its origin, K range and this lane's gather coordinates there
  struct TileC {
    int64_t m0, n0, kb0, ke;
    int nk, split;
    Pix apix[2];
    Tap atap[2];
    bool aok[2];
    unsigned bvo[NBH];
    bool bok[NBH];
  };
  auto coords = [&](int v, TileC& T) {
    int tm, tn;
    map_tile_at(v, c.nblk, c.tiles, c.tiles_m, c.tiles_n, c.group_m, true, T.split, tm, tn);
    T.m0 = (int64_t)tm * 256;
    T.n0 = (int64_t)tn * BN;
    T.kb0 = T.split * c.kchunk;
    T.ke = (T.kb0 + c.kchunk < c.K) ? T.kb0 + c.kchunk : c.K;
    T.nk = T.ke > T.kb0 ? (int)((T.ke - T.kb0 + BK - 1) / BK) : 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (AKC) {
        T.apix[h] = split_pix(T.m0 + h * 128 + arow[h], c.M, c.fd_w, c.fd_h);
        T.aok[h] = T.apix[h].ok;
      } else {
        const int64_t m = T.m0 + h * 128 + arow[h];
        T.aok[h] = m < c.M;
        T.atap[h] = split_tap(T.aok[h] ? m : 0, c.fd_c, c.fd_kw);
      }
    }
#pragma unroll
    for (int h = 0; h < NBH; ++h) {
      const int64_t n = T.n0 + h * 128 + ((p & 15) ^ ((bkk & 3) << 2)) * 8;
      T.bok[h] = n < c.Nn && n < T.n0 + BN;
      T.bvo[h] = (unsigned)(((int64_t)bkk * c.Nn + (T.bok[h] ? n : 0)) * 2);
    }
  };
  const unsigned lds0 =
      (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ptr)smem + (unsigned)wave * 1024u);
  auto issue = [&](unsigned v, const u32x4s& rs, unsigned ldsa, unsigned soff) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(v), "s"(rs), "s"(ldsa), "s"(soff)
                 : "memory");
  };
  // K-tile t of tile T into ring stage g % NST (g: the ring's running K-tile count)
  auto dma_a = [&](const TileC& T, int t, int g) {
    const int64_t k0 = T.kb0 + (int64_t)t * BK;
    const unsigned ldst = lds0 + (unsigned)((g % NST) * STAGE * 2);
    const unsigned tap = AKC ? (unsigned)__builtin_amdgcn_readfirstlane(c.fd_c.div((unsigned)k0)) : 0u;
    const int ch0 = (int)((unsigned)k0 - tap * (unsigned)chans);
    const int kh = (int)c.fd_kw.div(tap), kw = (int)(tap - (unsigned)kh * c.KW);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      unsigned v = kROOB;
      if (AKC) {
        const Pix& q = T.apix[h];
        int64_t off;
        bool ok;
        if (MODE == kFwd) {
          const int hi = q.a * c.sh + kh - c.ph, wi = q.b * c.sw + kw - c.pw;
          ok = hi >= 0 && hi < c.H && wi >= 0 && wi < c.W;
          off = (((int64_t)q.n * c.H + hi) * c.W + wi) * c.Ci + ch0 + akk[h];
        } else {
          const int ho = q.a + c.ph - kh, wo = q.b + c.pw - kw;
          ok = ho >= 0 && ho < c.Ho && wo >= 0 && wo < c.Wo;
          off = (((int64_t)q.n * c.Ho + ho) * c.Wo + wo) * c.Co + ch0 + akk[h];
        }
        if (T.aok[h] && ok && k0 + akk[h] < T.ke) v = (unsigned)(off * 2);
      } else {
        const int64_t k = k0 + akk[h];
        const Pix q = split_pix(k < T.ke ? k : 0, c.K, c.fd_w, c.fd_h);
        const Tap& t4 = T.atap[h];
        const int hi = q.a * c.sh + t4.kh - c.ph, wi = q.b * c.sw + t4.kw - c.pw;
        const bool ok = T.aok[h] && k < T.ke && hi >= 0 && hi < c.H && wi >= 0 && wi < c.W;
        if (ok) v = (unsigned)(((((int64_t)q.n * c.H + hi) * c.W + wi) * c.Ci + t4.ch) * 2);
      }
      issue(v, rsA, ldst + (unsigned)(h * HALF * 2), 0u);
    }
  };
  auto dma_b = [&](const TileC& T, int t, int g) {
    const int64_t k0 = T.kb0 + (int64_t)t * BK;
    const unsigned ldst = lds0 + (unsigned)((g % NST) * STAGE * 2);
    const unsigned soff = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(k0 * c.Nn * 2));
#pragma unroll
    for (int h = 0; h < NBH; ++h) {
      const unsigned v = (T.bok[h] && k0 + bkk < T.ke) ? T.bvo[h] : kROOB;
      issue(v, rsB, ldst + (unsigned)((2 + h) * HALF * 2), soff);
    }
  };
  static_assert(NST >= 4 && NST * STAGE * 2 <= 160 * 1024, "ring16: 4+ stages within 160 KB of LDS");
  auto retire_keep = [](int tiles_in_flight) {   // at most NST - 2 K-tiles (NDMA instructions each) left in flight
    if (NST >= 6 && tiles_in_flight >= 4) wait_vm<4 * NDMA>();
    else if (NST >= 5 && tiles_in_flight >= 3) wait_vm<3 * NDMA>();
    else if (tiles_in_flight >= 2) wait_vm<2 * NDMA>();
    else if (tiles_in_flight == 1) wait_vm<NDMA>();
    else wait_vm<0>();
  };

  TileC cur;
  coords(blockIdx.x, cur);
  for (int t = 0; t < NST - 1; ++t)
    if (t < cur.nk) {
      dma_a(cur, t, t);
      dma_b(cur, t, t);
    }
  retire_keep(min(cur.nk - 1, NST - 2));
  bar();
  if (grp == 1) bar();

  const int ar0 = wr * (128 / WR);
  const int bh = (wc * (BN / WC)) / 128, bc0 = (wc * (BN / WC)) % 128;
  const int lh = lane >> 5, lc = lane & 31;
  const int g0 = 0;   // the ring's K-tile count at this tile's first K-tile
  {
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = cur.nk;
    for (int kt = 0; kt < nk; ++kt) {
      const unsigned short* S = smem + ((g0 + kt) % NST) * STAGE;
      const unsigned short* As = S + grp * HALF;
      const unsigned short* Bs = S + (2 + bh) * HALF;
      const int tn_ = kt + NST - 1;   // the K-tile issued now
      static_assert(QS == 1 || QS == 2, "ring16: 1 or 2 k-steps per section");
#pragma unroll
      for (int q = 0; q < BK / 16; q += QS) {
        u32x4_ fa[QS][TM], fb[QS][TN];
#pragma unroll
        for (int e = 0; e < QS; ++e) {
#pragma unroll
          for (int i = 0; i < TM; ++i) fa[e][i] = r16_frag<AKC>(As, ar0 + i * 32, 16 * (q + e), lane);
#pragma unroll
          for (int j = 0; j < TN; ++j) fb[e][j] = r16_frag<false>(Bs, bc0 + j * 32, 16 * (q + e), lane);
        }
        if (tn_ < nk) {
          const TileC& T = cur;
          const int tt = tn_;
          if (QS == 2) {
            dma_a(T, tt, g0 + tn_);
            dma_b(T, tt, g0 + tn_);
          } else if (q == 0) {
            dma_a(T, tt, g0 + tn_);
          } else {
            dma_b(T, tt, g0 + tn_);
          }
        }
        // K-tile kt + 1 (of the ring) landed, this wave's part
        if (q + QS == BK / 16) retire_keep(min(nk - 1 - (kt + 1), NST - 2));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int e = 0; e < QS; ++e)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = ConvLp<LP>::mma(fa[e][i], fb[e][j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
        bar();
      }
    }

    // epilogue straight from the accumulators
    const int64_t rbase = cur.m0 + grp * 128 + ar0;
    const int64_t cbase = cur.n0 + bh * 128 + bc0;
    if (MODE == kFwd && c.pool_w == 4 && !c.partial) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int64_t col = cbase + j * 32 + lc;
          if (col >= c.Nn) continue;
          const float bv = c.bias ? c.bias[col] : 0.f;
#pragma unroll
          for (int rq = 0; rq < 4; ++rq) {
            const int64_t row = rbase + i * 32 + 8 * rq + 4 * lh;
            if (row >= c.M) continue;
            float best = acc[i][j][4 * rq] + bv;
            int arg = 0;
#pragma unroll
            for (int pp = 1; pp < 4; ++pp) {
              const float v = acc[i][j][4 * rq + pp] + bv;
              if (v > best || (v != v && best == best)) { best = v; arg = pp; }
            }
            c.out[(row >> 2) * c.Nn + col] = best;
            c.pool_arg[(row >> 2) * c.Nn + col] = (uint8_t)arg;
          }
        }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int64_t col = cbase + j * 32 + lc;
          if (col >= c.Nn) continue;
          const float bv = (MODE == kFwd && c.bias && !c.partial) ? c.bias[col] : 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int64_t row = rbase + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (row >= c.M) continue;
            if (c.partial) c.partial[((int64_t)cur.split * c.M + row) * c.Nn + col] = acc[i][j][r];
            else c.out[row * c.Nn + col] = acc[i][j][r] + bv;
          }
        }
    }
  }
  if (grp == 0) bar();
}

// ------------------------------------------------------------------ row-staged (1, KW) conv + (1, 4) pool
// fbanks_cnn conv2 + maxpool2 in 16-bit modes (model_fbanks_cnn.py:74-75, 91-92: Conv2d(64, 128, (1, 7),
// padding (0, 3)) over W = 40, then MaxPool2d((1, 4))), option conv_row16.  The implicit GEMM re-gathers every
// input pixel once per tap (7 x) from L2 with per-unit index math; PMC put the register-staged kernel at
// ~22 VALU instructions per MFMA and 18 % MFMA-busy (profiles/r05/r05e_pmc_fbconv2.txt).  Here a persistent
// workgroup keeps the whole 16-bit weight matrix [(kw, ci)][co] (448 x 128, 112 KB) in LDS for its lifetime and
// stages R = 8 image rows of x16 ONCE per tile (8 x 46 padded positions x 64 channels, 46 KB, halo zeros written
// once); the 7 taps are then 7 shifted reads of the staged rows.  The next tile's rows are prefetched into
// registers during this tile's MFMAs.  Tile = 8 rows x 40 pixels = 320 GEMM rows (10 blocks of 32) x 128
// columns; wave w owns column block w & 3 and row blocks 5 (w >> 2) .. +4 (5 accumulators, one B fragment per
// k-step for five A fragments).  The epilogue is conv_gemm_kernel's pooled one: bias, the (1, 4) window max and
// its first-maximum argmax in registers (r & 3 = the 4 window columns), pooled fp32 out + uint8 argmax.
// Same MFMA operands and k order as the ring / register-staged kernels (k = (kw, ci) ascending, 16 per MFMA), so
// results equal theirs up to nothing (tests/test_lowprec_gpu.py test_conv_row16_equals_gemm: bitwise).
struct RowArgs {
  const unsigned short* x16;   // [rows][W][CI] 16-bit
  const unsigned short* w16;   // [(kw, ci)][CO] 16-bit (the fwd weight matrix Wt)
  const float* bias;           // [CO] or null
  float* y;                    // pooled [rows][W / 4][CO]
  uint8_t* arg;                // [rows][W / 4][CO]
  int rows, groups;
};
// NW: 8 waves (wave = 1 column block x 5 row blocks: 6 fragment reads per 5 MFMAs) or 4 waves (wave = 2 column
// blocks x 5 row blocks, 160 accumulator registers: 7 fragment reads per 10 MFMAs — half the LDS traffic per MFMA;
// at 8 waves the operand reads, ~150 B per clock per CU, sit above the LDS array's 128) — option conv_row16 = 1 / 2.
template <int LP, int KW, int PW, int WD, int CI, int CO, int R, int NW = 8>
__global__ __launch_bounds__(NW * 64, 1) void conv_row16_pool_kernel(RowArgs a) {
  static_assert(CO == 128 && CI % 16 == 0 && WD % 4 == 0 && (R * WD) % 32 == 0 && CI * 2 == 128, "row16 geometry");
  constexpr int NT = NW * 64;
  constexpr int WP = WD + 2 * PW;               // padded positions per staged row
  constexpr int K = KW * CI;                    // GEMM depth
  constexpr int MB = R * WD / 32;               // row blocks of 32 (10)
  constexpr int RB = MB / 2;                    // row blocks per wave (5)
  constexpr int CB = NW == 8 ? 1 : 2;           // column blocks per wave
  constexpr int XCH = R * WD * (CI / 8);        // 16-B chunks of one tile's rows (2560)
  constexpr int XPT = XCH / NT;                 // per thread (5 / 10)
  static_assert(XCH % NT == 0 && MB % 2 == 0 && (NW == 8 || NW == 4), "row16 tile split");
  __shared__ __attribute__((aligned(16))) unsigned short Wl[K * CO];        // TR image [k][co] (r16_off<false>)
  __shared__ __attribute__((aligned(16))) unsigned short Xl[R * WP * CI];   // [row][pos][ci], 16-B chunks swizzled
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = NW == 8 ? (wave & 3) : (wave & 1) * 2, rb0 = (NW == 8 ? (wave >> 2) : (wave >> 1)) * RB;
  // the weights, once: 16-B chunks of 8 columns into the TR image
  for (int c = tid; c < K * CO / 8; c += NT) {
    const int k = c / (CO / 8), col = (c % (CO / 8)) * 8;
    *reinterpret_cast<u32x4_*>(Wl + r16_off<false>(col, k)) = *reinterpret_cast<const u32x4_*>(a.w16 + (size_t)k * CO + col);
  }
  // the halo positions (never overwritten by the staging)
  for (int c = tid; c < R * 2 * PW * (CI / 8); c += NT) {
    const int rl = c / (2 * PW * (CI / 8)), rem = c % (2 * PW * (CI / 8));
    const int pp = rem / (CI / 8), ch = rem % (CI / 8);
    const int q = pp < PW ? pp : WD + pp;   // 0 .. PW - 1 and WD + PW .. WD + 2 PW - 1
    *reinterpret_cast<u32x4_*>(Xl + (rl * WP + q) * CI + ((ch ^ (q & 7)) * 8)) = u32x4_{0u, 0u, 0u, 0u};
  }
  u32x4_ xr[XPT];
  auto fetch = [&](int g) {   // tile g's rows into registers (zeros past the last row)
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT, rl = c / (WD * (CI / 8)), rem = c % (WD * (CI / 8));
      const int row = g * R + rl;
      xr[i] = row < a.rows ? *reinterpret_cast<const u32x4_*>(a.x16 + ((size_t)row * WD) * CI + (size_t)rem * 8)
                           : u32x4_{0u, 0u, 0u, 0u};
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT, rl = c / (WD * (CI / 8)), rem = c % (WD * (CI / 8));
      const int px = rem / (CI / 8), ch = rem % (CI / 8), q = px + PW;
      *reinterpret_cast<u32x4_*>(Xl + (rl * WP + q) * CI + ((ch ^ (q & 7)) * 8)) = xr[i];
    }
  };
  // this lane's A rows: row block rb0 + i, pixel (lane & 31) of it -> staged row and position (tap 0)
  // (the chunk swizzle keys on the position within the staged row, as the staging and the halo writes do)
  int arow[RB], apos[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    const int p = (rb0 + i) * 32 + (lane & 31);
    arow[i] = (p / WD) * WP;
    apos[i] = p % WD;
  }
  const int khalf = lane >> 5;   // which 8 of the 16 k of a step this lane supplies
  const int lh = lane >> 5, lc = lane & 31;
  float bv[CB];
#pragma unroll
  for (int j = 0; j < CB; ++j) bv[j] = a.bias ? a.bias[(wc + j) * 32 + lc] : 0.f;
  int g = blockIdx.x;
  if (g < a.groups) fetch(g);
  __syncthreads();
  while (g < a.groups) {
    stage();
    __syncthreads();
    const int gn = g + (int)gridDim.x;
    if (gn < a.groups) fetch(gn);   // lands during the MFMAs below
    f32x16 acc[RB][CB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int j = 0; j < CB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    constexpr int CU = NW == 4 ? 1 : 4;   // the 4-wave form: one k-step's fragments live at a time (registers)
#pragma unroll 1
    for (int kw = 0; kw < KW; ++kw) {
#pragma unroll CU
      for (int c0 = 0; c0 < CI; c0 += 16) {
        u32x4_ bf[CB];
#pragma unroll
        for (int j = 0; j < CB; ++j) bf[j] = r16_frag<false>(Wl, (wc + j) * 32, kw * CI + c0, lane);
        const int ch = (c0 >> 3) + khalf;
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int q = apos[i] + kw;   // position in the staged row
          const u32x4_ af = *reinterpret_cast<const u32x4_*>(Xl + (arow[i] + q) * CI + ((ch ^ (q & 7)) * 8));
#pragma unroll
          for (int j = 0; j < CB; ++j) acc[i][j] = ConvLp<LP>::mma(af, bf[j], acc[i][j]);
        }
      }
    }
    // pooled epilogue: rows 8 rq + 4 lh + 0..3 of a block are one (1, 4) window
#pragma unroll
    for (int i = 0; i < RB; ++i) {
#pragma unroll
      for (int rq = 0; rq < 4; ++rq) {
        const int p0 = (rb0 + i) * 32 + 8 * rq + 4 * lh;   // tile pixel, a multiple of 4
        const int row = g * R + p0 / WD;
        if (row >= a.rows) continue;
#pragma unroll
        for (int j = 0; j < CB; ++j) {
          float best = acc[i][j][4 * rq] + bv[j];
          int am = 0;
#pragma unroll
          for (int pp = 1; pp < 4; ++pp) {
            const float v = acc[i][j][4 * rq + pp] + bv[j];
            if (v > best || (v != v && best == best)) { best = v; am = pp; }
          }
          const size_t o = ((size_t)g * R * WD + p0) / 4 * CO + (wc + j) * 32 + lc;
          a.y[o] = best;
          a.arg[o] = (uint8_t)am;
        }
      }
    }
    __syncthreads();   // every wave is done reading Xl before the next tile is staged
    g = gn;
  }
}

// The same conv + (1, 4) pool on fp32 operands (cfg3 at the reference's precision; option conv_row32): the fp32
// weight matrix (448 x 128 x 4 B = 224 KB) does not fit in LDS beside the staged rows, so the workgroup stages 8
// image rows of x ONCE per tile ([8][46 padded positions][64 ci] fp32, 92 KB, 16-B chunks XOR-swizzled by position)
// and streams Wt one tap at a time ([64 ci][128 co], 32 KB, double-buffered, the next tap's loads in flight during
// this tap's MFMAs; the whole matrix stays in L2).  8 waves over the 320 x 128 tile: wave = column block w & 3 x
// row blocks 5 (w >> 2) .. +4, v_mfma_f32_32x32x2_f32 with the k-permuted 8-deep blocks of the tile core
// (mfma_tile.h: sub-step s of block b pairs k = 8 b + s and 8 b + 4 + s, A by one ds_read_b128, B by 4 ds_read_b32
// whose halves the column swizzle puts on disjoint banks).  k = (kw, ci) ascending in 8-deep blocks — the
// implicit GEMM's sequence per accumulator, and the same pooled epilogue: bitwise its result
// (tests/test_conv_gpu.py test_conv_row32_equals_gemm).
struct Row32Args {
  const float* x;      // [rows][WD][CI] fp32
  const float* wt;     // [(kw, ci)][CO] fp32 (the fwd weight matrix Wt)
  const float* bias;   // [CO] or null
  float* y;            // pooled [rows][WD / 4][CO]
  uint8_t* arg;        // [rows][WD / 4][CO]
  int rows, groups;
};
template <int KW, int PW, int WD, int CI, int CO, int R>
__global__ __launch_bounds__(512, 1) void conv_row32_pool_kernel(Row32Args a) {
  static_assert(CO == 128 && CI == 64 && WD % 4 == 0 && (R * WD) % 32 == 0, "row32 geometry");
  constexpr int NT = 512;
  constexpr int WP = WD + 2 * PW;               // padded positions per staged row
  constexpr int MB = R * WD / 32;               // row blocks of 32 (10)
  constexpr int RB = MB / 2;                    // row blocks per wave (5)
  constexpr int XCH = R * WD * (CI / 4);        // 16-B chunks of one tile's rows (5120)
  constexpr int XPT = XCH / NT;                 // per thread (10)
  constexpr int TCH = CI * CO / 4;              // 16-B chunks of one tap's weights (2048)
  constexpr int TPT = TCH / NT;                 // per thread (4)
  static_assert(XCH % NT == 0 && TCH % NT == 0 && MB % 2 == 0, "row32 tile split");
  __shared__ __attribute__((aligned(16))) float Xl[R * WP * CI];   // [row][pos][ci], chunk ch at ch ^ (pos & 15)
  __shared__ __attribute__((aligned(16))) float Wl[2][CI * CO];    // one tap [k][co], co ^ (((k >> 2) & 1) << 5)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave & 3, rb0 = (wave >> 2) * RB;
  for (int c = tid; c < R * 2 * PW * (CI / 4); c += NT) {   // the halo positions, once
    const int rl = c / (2 * PW * (CI / 4)), rem = c % (2 * PW * (CI / 4));
    const int pp = rem / (CI / 4), ch = rem % (CI / 4);
    const int q = pp < PW ? pp : WD + pp;
    *reinterpret_cast<v4f*>(Xl + (rl * WP + q) * CI + ((ch ^ (q & 15)) * 4)) = v4f{0.f, 0.f, 0.f, 0.f};
  }
  v4f xr[XPT], wr[TPT];
  const auto rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), (short)0, 0x7ffffff0, 0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.wt), (short)0, 0x7ffffff0, 0x00020000);
  auto fetch_x = [&](int g) {   // tile g's rows into registers (past the last row: 16 zero bytes)
    const int last = (a.rows - g * R) * WD * (CI / 4);
    const int sbase = __builtin_amdgcn_readfirstlane(g * R * WD * CI * 4);
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT;
      xr[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rsX, c < last ? sbase + c * 16 : (int)0x80000000u,
                                                                             0, 0));
    }
  };
  auto stage_x = [&]() {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT, rl = c / (WD * (CI / 4)), rem = c % (WD * (CI / 4));
      const int px = rem / (CI / 4), ch = rem % (CI / 4), q = px + PW;
      *reinterpret_cast<v4f*>(Xl + (rl * WP + q) * CI + ((ch ^ (q & 15)) * 4)) = xr[i];
    }
  };
  auto fetch_w = [&](int kw) {
    const int sbase = __builtin_amdgcn_readfirstlane(kw * CI * CO * 4);
#pragma unroll
    for (int i = 0; i < TPT; ++i)
      wr[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rsW, sbase + (tid + i * NT) * 16, 0, 0));
  };
  auto stage_w = [&](int buf) {
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int c = tid + i * NT, k = c / (CO / 4), col = (c % (CO / 4)) * 4;
      *reinterpret_cast<v4f*>(&Wl[buf][k * CO + (col ^ (((k >> 2) & 1) << 5))]) = wr[i];
    }
  };
  int arow[RB], apos[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    const int p = (rb0 + i) * 32 + (lane & 31);
    arow[i] = (p / WD) * WP;
    apos[i] = p % WD;
  }
  const int lh = lane >> 5, lc = lane & 31;
  const int bcol = (wc * 32 + lc) ^ (lh << 5);   // this lane's B column in the swizzled tap image (k >> 2 & 1 = lh)
  const float bv = a.bias ? a.bias[wc * 32 + lc] : 0.f;
  int g = blockIdx.x;
  if (g < a.groups) fetch_x(g);
  fetch_w(0);
  while (g < a.groups) {
    stage_x();
    stage_w(0);
    __syncthreads();
    const int gn = g + (int)gridDim.x;
    f32x16 acc[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll 1
    for (int kw = 0; kw < KW; ++kw) {
      fetch_w(kw + 1 < KW ? kw + 1 : 0);   // the next tap (tap 0 again for the next tile)
      const float* Ws = Wl[kw & 1];
      // one 8-deep block's fragments at a time (a double-buffered prefetch spilled at 2 waves per SIMD, and a 4-wave
      // form with it — 512 registers, 10 row blocks per wave — measured slower, 2.35 vs 2.08 ms per cfg3 step, r06g:
      // the other wave of the SIMD covers the LDS latency)
#pragma unroll 1
      for (int kb = 0; kb < CI / 8; ++kb) {
        const float* q0 = Ws + (kb * 8 + 4 * lh) * CO + bcol;
        const v4f fb = v4f{q0[0], q0[CO], q0[2 * CO], q0[3 * CO]};
        const int ch = 2 * kb + lh;
        v4f fa[RB];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int q = apos[i] + kw;   // position in the staged row
          fa[i] = *reinterpret_cast<const v4f*>(Xl + (arow[i] + q) * CI + ((ch ^ (q & 15)) * 4));
        }
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
          for (int i = 0; i < RB; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s2], fb[s2], acc[i], 0, 0, 0);
      }
      if (kw + 1 < KW) stage_w((kw + 1) & 1);   // that buffer was last read in tap kw - 1 (behind the barrier)
      __syncthreads();
    }
    // pooled epilogue (the implicit GEMM's): rows 8 rq + 4 lh + 0..3 of a block are one (1, 4) window
#pragma unroll
    for (int i = 0; i < RB; ++i) {
#pragma unroll
      for (int rq = 0; rq < 4; ++rq) {
        const int p0 = (rb0 + i) * 32 + 8 * rq + 4 * lh;   // tile pixel, a multiple of 4
        const int row = g * R + p0 / WD;
        if (row >= a.rows) continue;
        float best = acc[i][4 * rq] + bv;
        int am = 0;
#pragma unroll
        for (int pp = 1; pp < 4; ++pp) {
          const float v = acc[i][4 * rq + pp] + bv;
          if (v > best || (v != v && best == best)) { best = v; am = pp; }
        }
        const size_t o = ((size_t)g * R * WD + p0) / 4 * CO + wc * 32 + lc;
        a.y[o] = best;
        a.arg[o] = (uint8_t)am;
      }
    }
    if (gn < a.groups) fetch_x(gn);
    __syncthreads();   // every wave is done reading Xl before the next tile is staged
    g = gn;
  }
}

// The fp32 data gradient of the same conv (option conv_row32): dX[w][ci] = sum over (kw, co) of dY[w + PW - kw][co]
// Wd[(kw, co)][ci].  8 staged rows of dY in fp32 are 184 KB, so the workgroup stages them one 64-channel HALF at a
// time ([8][46][64] fp32, 92 KB, 16-B chunks XOR-swizzled by position) and streams Wd one (tap, half) slice at a
// time ([64 co][64 ci], 16 KB, double-buffered); the next half's (or the next tile's) dY rows load into registers
// during the current half's MFMAs.  POOLED: dY arrives as fbanks_cnn's pooled gradient + its uint8 window argmax
// (the pooled conv's backward) and is rebuilt at staging time, dY[px][co] = arg[px / 4][co] == px % 4 ?
// dP[px / 4][co] : 0 — the implicit GEMM's UNPOOL gather — so a quarter of the dense bytes is read.  4 waves (one
// per SIMD, 512 registers): wave = column block w & 1 x row blocks 5 (w >> 1) .. +4 on v_mfma_f32_32x32x2_f32 in
// the tile core's k-permuted 8-deep blocks, the next block's fragments read ahead of this block's MFMAs.  k order
// (half, kw, co) — another fp32 summation order than the implicit GEMM's (kw, co) (tests: within 1e-5).
struct Row32DgArgs {
  const float* dy;      // dense [rows][WD][CA], or POOLED [rows][WD / 4][CA]
  const uint8_t* arg;   // POOLED: [rows][WD / 4][CA] window argmax
  const float* wd;      // [(kw, co)][CN] fp32 (the dgrad weight matrix Wd)
  float* dx;            // [rows][WD][CN]
  int rows, groups;
};
template <int KW, int PW, int WD, int CA, int CN, int R, bool POOLED>
__global__ __launch_bounds__(256, 1) void conv_row32_dgrad_kernel(Row32DgArgs a) {
  static_assert(CA == 128 && CN == 64 && WD % 4 == 0 && (R * WD) % 32 == 0 && 2 * PW == KW - 1, "row32 dgrad geometry");
  constexpr int NT = 256, CH = 64;                       // threads; channels of dY per staged half
  constexpr int WP = WD + 2 * PW;
  constexpr int MB = R * WD / 32;                        // row blocks (10)
  constexpr int RB = MB / 2;                             // row blocks per wave (5)
  constexpr int YCH = POOLED ? R * (WD / 4) * (CH / 4) : R * WD * (CH / 4);   // loaded 16-B chunks per half tile
  constexpr int YPT = YCH / NT;                          // per thread (5 pooled / 20 dense)
  constexpr int TCH = CH * CN / 4;                       // 16-B chunks of one (tap, half) slice (1024)
  constexpr int TPT = TCH / NT;                          // per thread (4)
  static_assert(YCH % NT == 0 && TCH % NT == 0 && MB == 10, "row32 dgrad tile split");
  __shared__ __attribute__((aligned(16))) float Yl[R * WP * CH];   // [row][pos][co of the half], ch ^ (pos & 15)
  __shared__ __attribute__((aligned(16))) float Wl[2][CH * CN];    // one slice [co][ci], ci ^ (((co >> 2) & 1) << 5)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cb = wave & 1, rb0 = (wave >> 1) * RB;
  for (int c = tid; c < R * 2 * PW * (CH / 4); c += NT) {   // halo positions, once
    const int rl = c / (2 * PW * (CH / 4)), rem = c % (2 * PW * (CH / 4));
    const int pp = rem / (CH / 4), ch = rem % (CH / 4);
    const int q = pp < PW ? pp : WD + pp;
    *reinterpret_cast<v4f*>(Yl + (rl * WP + q) * CH + ((ch ^ (q & 15)) * 4)) = v4f{0.f, 0.f, 0.f, 0.f};
  }
  v4f yr[YPT], wr[TPT];
  unsigned ar[POOLED ? YPT : 1];
  const auto rsY = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.dy), (short)0, 0x7ffffff0, 0x00020000);
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(POOLED ? a.arg : nullptr), (short)0,
                                                     0x7ffffff0, 0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.wd), (short)0, 0x7ffffff0, 0x00020000);
  constexpr int PXL = POOLED ? WD / 4 : WD;   // loaded positions per row
  auto fetch_y = [&](int g, int h) {   // half h of tile g's dY rows (past the last row: zeros)
    const int last = (a.rows - g * R) * PXL * (CH / 4);
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int c = tid + i * NT, rl = c / (PXL * (CH / 4)), rem = c % (PXL * (CH / 4));
      const int px = rem / (CH / 4), ch = rem % (CH / 4);
      const int e = ((g * R + rl) * PXL + px) * CA + h * CH + ch * 4;   // element index (< 2^31 / 4: host check)
      const bool ok = c < last;
      yr[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rsY, ok ? e * 4 : (int)0x80000000u, 0, 0));
      if constexpr (POOLED) ar[i] = __builtin_amdgcn_raw_buffer_load_b32(rsA, ok ? e : (int)0x80000000u, 0, 0);
    }
  };
  auto stage_y = [&]() {
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int c = tid + i * NT, rl = c / (PXL * (CH / 4)), rem = c % (PXL * (CH / 4));
      const int px = rem / (CH / 4), ch = rem % (CH / 4);
      if constexpr (POOLED) {   // the pooled value goes to the window position its argmax names, zeros elsewhere
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
          const int q = 4 * px + pp + PW;
          v4f v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = ((ar[i] >> (8 * e)) & 0xFFu) == (unsigned)pp ? yr[i][e] : 0.f;
          *reinterpret_cast<v4f*>(Yl + (rl * WP + q) * CH + ((ch ^ (q & 15)) * 4)) = v;
        }
      } else {
        const int q = px + PW;
        *reinterpret_cast<v4f*>(Yl + (rl * WP + q) * CH + ((ch ^ (q & 15)) * 4)) = yr[i];
      }
    }
  };
  auto fetch_w = [&](int kw, int h) {   // slice (kw, h): Wd rows kw * CA + h * CH .. + 63
    const int sbase = __builtin_amdgcn_readfirstlane((kw * CA + h * CH) * CN * 4);
#pragma unroll
    for (int i = 0; i < TPT; ++i)
      wr[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rsW, sbase + (tid + i * NT) * 16, 0, 0));
  };
  auto stage_w = [&](int buf) {
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int c = tid + i * NT, k = c / (CN / 4), col = (c % (CN / 4)) * 4;
      *reinterpret_cast<v4f*>(&Wl[buf][k * CN + (col ^ (((k >> 2) & 1) << 5))]) = wr[i];
    }
  };
  int arow[RB], apos[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    const int p = (rb0 + i) * 32 + (lane & 31);
    arow[i] = (p / WD) * WP;
    apos[i] = p % WD;
  }
  const int lh = lane >> 5, lc = lane & 31;
  const int bcol = (cb * 32 + lc) ^ (lh << 5);
  int g = blockIdx.x;
  if (g < a.groups) fetch_y(g, 0);
  fetch_w(0, 0);
  while (g < a.groups) {
    const int gn = g + (int)gridDim.x;
    f32x16 acc[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      stage_y();
      stage_w(0);
      __syncthreads();
      if (h == 0) fetch_y(g, 1);                  // the second half lands during the first half's MFMAs
      else if (gn < a.groups) fetch_y(gn, 0);     // the next tile's first half during the second's
#pragma unroll 1
      for (int kw = 0; kw < KW; ++kw) {
        if (kw + 1 < KW) fetch_w(kw + 1, h);
        else fetch_w(0, h ^ 1);                   // the next half's (or the next tile's) first slice
        const float* Ws = Wl[kw & 1];
        auto frags = [&](int kb, v4f (&fa)[RB], v4f& fb) {
          const float* q0 = Ws + (kb * 8 + 4 * lh) * CN + bcol;
          fb = v4f{q0[0], q0[CN], q0[2 * CN], q0[3 * CN]};
          const int ch = 2 * kb + lh;
#pragma unroll
          for (int i = 0; i < RB; ++i) {
            const int q = apos[i] + 2 * PW - kw;   // dY position w + PW - kw in the staged (haloed) row
            fa[i] = *reinterpret_cast<const v4f*>(Yl + (arow[i] + q) * CH + ((ch ^ (q & 15)) * 4));
          }
        };
        v4f fa[2][RB], fb[2];
        frags(0, fa[0], fb[0]);
#pragma unroll
        for (int kb = 0; kb < CH / 8; ++kb) {
          const int c = kb & 1;
          if (kb + 1 < CH / 8) frags(kb + 1, fa[c ^ 1], fb[c ^ 1]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
            for (int i = 0; i < RB; ++i)
              acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[c][i][s2], fb[c][s2], acc[i], 0, 0, 0);
        }
        if (kw + 1 < KW) stage_w((kw + 1) & 1);   // that buffer was last read in tap kw - 1 (behind the barrier)
        __syncthreads();
      }
    }
    float* const xbase = a.dx + (size_t)g * R * WD * CN;
    const int nreal = (a.rows - g * R) * WD;   // real pixels of this tile
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = (rb0 + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (p < nreal) xbase[p * CN + cb * 32 + lc] = acc[i][r];
      }
    g = gn;
  }
}

// The fp32 weight gradient of the same conv (option conv_row32): dWt[(kw, ci)][co] = sum over pixels p of
// X[p + kw - PW][ci] dY[p][co], dY = the pooled gradient unpooled through its window argmax (fbanks_cnn's pooled
// backward).  The implicit GEMM (conv_gemm_kernel<wgrad, unpool>) re-gathers every x pixel once per tap from L2
// with per-unit index math and writes 126 split-K slabs; here a persistent workgroup stages R = 8 image rows of x
// ([8][46 padded positions][64 ci] fp32, halo zeros written once, 92 KB) and the same rows' pooled dY + argmax
// ([8][10][128] fp32 + bytes, 50 KB) once per tile.  The GEMM's k is the tile's pixels, so the 7 taps are 7
// shifted reads of the staged rows and one B fragment — unpooled at read time by a select on the argmax byte —
// serves all 7.  8 waves: wave = co block w & 3 x ci half w >> 2, all 7 taps (7 accumulators on
// v_mfma_f32_32x32x2_f32; lane half h supplies pixel 2 s + h of k-step s).  The next tile's rows load into
// registers during this tile's MFMAs.  Each workgroup writes its partial dWt (and the column sums of dY over its
// rows, the bias gradient) to its own slab, reduced in a fixed order afterwards: deterministic.  k order
// (workgroup's tiles, row, pixel pair) — another fp32 summation order than the implicit GEMM's (tests: 1e-5).
struct Row32WgArgs {
  const float* x;       // [rows][WD][CI]
  const float* dy;      // POOLED [rows][WD / 4][CO]
  const uint8_t* arg;   // [rows][WD / 4][CO] window argmax
  float* slab;          // [gridDim.x][KW * CI][CO]
  float* bpart;         // [gridDim.x][CO], or null (no bias gradient)
  int rows, groups;
};
template <int KW, int PW, int WD, int CI, int CO, int R>
__global__ __launch_bounds__(512, 1) void conv_row32_wgrad_kernel(Row32WgArgs a) {
  static_assert(CO == 128 && CI == 64 && WD % 4 == 0 && 2 * PW == KW - 1, "row32 wgrad geometry");
  constexpr int NT = 512;
  constexpr int WP = WD + 2 * PW;             // padded positions per staged row (46)
  constexpr int PQ = WD / 4;                  // pooled positions per row (10)
  constexpr int XCH = R * WD * (CI / 4);      // 16-B chunks of a tile's x rows (5120)
  constexpr int XPT = XCH / NT;               // per thread (10)
  constexpr int YCH = R * PQ * (CO / 4);      // 16-B chunks of the pooled dY rows (2560)
  constexpr int YPT = YCH / NT;               // per thread (5)
  constexpr int ACH = R * PQ * CO / 4;        // 4-B words of the argmax rows (2560)
  constexpr int APT = ACH / NT;               // per thread (5)
  static_assert(XCH % NT == 0 && YCH % NT == 0 && ACH % NT == 0, "row32 wgrad tile split");
  __shared__ __attribute__((aligned(16))) float Xl[R * WP * CI];        // [row][pos][ci]
  __shared__ __attribute__((aligned(16))) float Pl[R * PQ * CO];        // [row][q][co]
  __shared__ __attribute__((aligned(16))) unsigned Al[R * PQ * CO / 4];  // bytes [row][q][co]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cb = wave & 3, hb = wave >> 2, lh = lane >> 5, lc = lane & 31;
  for (int c = tid; c < R * 2 * PW * (CI / 4); c += NT) {   // the halo positions, once
    const int rl = c / (2 * PW * (CI / 4)), rem = c % (2 * PW * (CI / 4));
    const int pp = rem / (CI / 4), ch = rem % (CI / 4);
    const int q = pp < PW ? pp : WD + pp;
    *reinterpret_cast<v4f*>(Xl + (rl * WP + q) * CI + ch * 4) = v4f{0.f, 0.f, 0.f, 0.f};
  }
  v4f xr[XPT], yr[YPT];
  unsigned ar[APT];
  const auto rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), (short)0, 0x7ffffff0, 0x00020000);
  const auto rsY = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.dy), (short)0, 0x7ffffff0, 0x00020000);
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.arg), (short)0, 0x7ffffff0, 0x00020000);
  constexpr int kOOB = (int)0x80000000u;   // past num_records: the load returns zeros
  auto fetch = [&](int g) {   // tile g's rows into registers (past the last row: zeros)
    const int real = a.rows - g * R;
    const int sx = __builtin_amdgcn_readfirstlane(g * R * WD * CI * 4);
    const int sy = __builtin_amdgcn_readfirstlane(g * R * PQ * CO * 4);
    const int sa = __builtin_amdgcn_readfirstlane(g * R * PQ * CO);
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT;
      xr[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rsX, c < real * WD * (CI / 4) ? sx + c * 16 : kOOB,
                                                                             0, 0));
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int c = tid + i * NT;
      yr[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rsY, c < real * PQ * (CO / 4) ? sy + c * 16 : kOOB,
                                                                             0, 0));
    }
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int c = tid + i * NT;
      ar[i] = __builtin_amdgcn_raw_buffer_load_b32(rsA, c < real * PQ * CO / 4 ? sa + c * 4 : kOOB, 0, 0);
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT, rl = c / (WD * (CI / 4)), rem = c % (WD * (CI / 4));
      const int px = rem / (CI / 4), ch = rem % (CI / 4);
      *reinterpret_cast<v4f*>(Xl + (rl * WP + px + PW) * CI + ch * 4) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) *reinterpret_cast<v4f*>(Pl + (tid + i * NT) * 4) = yr[i];
#pragma unroll
    for (int i = 0; i < APT; ++i) Al[tid + i * NT] = ar[i];
  };
  f32x16 acc[KW];
#pragma unroll
  for (int t = 0; t < KW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bsum = 0.f;   // the column sum of dY at co = 32 cb + lc over this workgroup's rows (both lane halves)
  const int col = cb * 32 + lc;
  const float* xlane = Xl + lh * CI + hb * 32 + lc;   // + (row * WP + pixel pair base + tap) * CI
  const uint8_t* abytes = reinterpret_cast<const uint8_t*>(Al);
  int g = blockIdx.x;
  if (g < a.groups) fetch(g);
  while (g < a.groups) {
    stage();
    __syncthreads();
    const int gn = g + (int)gridDim.x;
    if (gn < a.groups) fetch(gn);   // lands during the MFMAs below
#pragma unroll 1
    for (int rl = 0; rl < R; ++rl) {
      const float* xrow = xlane + rl * WP * CI;
      const float* prow = Pl + rl * PQ * CO + col;
      const uint8_t* arow = abytes + rl * PQ * CO + col;
#pragma unroll
      for (int q = 0; q < PQ; ++q) {
        const float pv = prow[q * CO];
        const int am = arow[q * CO];
        bsum += pv;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {   // k-step: pixels 4 q + 2 s2 (lane half 0) and + 1 (half 1)
          const float bv = am == 2 * s2 + lh ? pv : 0.f;
          float av[KW];
#pragma unroll
          for (int t = 0; t < KW; ++t) av[t] = xrow[(4 * q + 2 * s2 + t) * CI];
#pragma unroll
          for (int t = 0; t < KW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[t], bv, acc[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();   // every wave is done reading the tile before the next one is staged
    g = gn;
  }
  float* sl = a.slab + (size_t)blockIdx.x * (KW * CI * CO);
#pragma unroll
  for (int t = 0; t < KW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ci = hb * 32 + 8 * (r >> 2) + 4 * lh + (r & 3);
      sl[(t * CI + ci) * CO + col] = acc[t][r];
    }
  if (a.bpart && hb == 0 && lh == 0) a.bpart[(size_t)blockIdx.x * CO + col] = bsum;
}

// The same weight gradient in 16-bit modes (option conv_row16): x's 16-bit copy (the forward's) and the pooled
// gradient + argmax, unpooled and rounded to 16 bits at staging (the operand values of unpool16 + to16, without
// the dense 16-bit dY in HBM).  v_mfma_f32_32x32x16 with k = 16 pixels per step: the A operand (x^T, m = ci) and
// the B operand (dY, n = co) are both row-contiguous [pixel][channel] images read by ds_read_b64_tr_b16 — a lane
// supplies the address of 4 channels at one pixel, so the 7 taps are 7 base offsets of the same staged rows
// (each lane's pixel + tap, any alignment).  Images: x [8 rows][46 positions][96] (64 channels + 32 pad: the 4
// pixels of a 16-lane read land on 4 distinct 16-bank spans) and dY [320 pixels][128] with 16-B units XOR'd by
// (pixel & 3) << 2 (the ring kernels' TR swizzle).  The bias gradient: fp32 column sums of the pooled gradient
// (before rounding), per thread over its fixed 4 channels, then in a fixed order through LDS.  One slab per
// workgroup, reduced in order (deterministic).
struct Row16WgArgs {
  const unsigned short* x16;   // [rows][WD][CI] 16-bit
  const float* dy;             // POOLED [rows][WD / 4][CO] fp32
  const uint8_t* arg;          // [rows][WD / 4][CO]
  float* slab;                 // [gridDim.x][KW * CI][CO]
  float* bpart;                // [gridDim.x][CO], or null
  int rows, groups;
};
template <int LP, int KW, int PW, int WD, int CI, int CO, int R>
__global__ __launch_bounds__(512, 1) void conv_row16_wgrad_kernel(Row16WgArgs a) {
  static_assert(CO == 128 && CI == 64 && WD % 8 == 0 && 2 * PW == KW - 1 && (R * WD) % 16 == 0, "row16 wgrad geometry");
  constexpr int NT = 512;
  constexpr int WP = WD + 2 * PW;             // padded positions per staged row (46)
  constexpr int XP = CI + 32;                 // x image pitch per position (96 elements)
  constexpr int PQ = WD / 4;                  // pooled positions per row (10)
  constexpr int XCH = R * WD * (CI / 8);      // 16-B chunks of a tile's x16 rows (2560)
  constexpr int XPT = XCH / NT;               // per thread (5)
  constexpr int YCH = R * PQ * (CO / 4);      // 16-B chunks of the pooled dY rows (2560)
  constexpr int YPT = YCH / NT;               // per thread (5)
  constexpr int KS = R * WD / 16;             // k-steps per tile (20)
  static_assert(XCH % NT == 0 && YCH % NT == 0 && NT % (CO / 4) == 0, "row16 wgrad tile split");
  __shared__ __attribute__((aligned(16))) unsigned short Xl[R * WP * XP];   // [row][pos][96]
  __shared__ __attribute__((aligned(16))) unsigned short Yl[R * WD * CO];   // [pixel][128], units swizzled
  __shared__ float Bs[NT / (CO / 4)][CO];                                    // bias partials of the thread rows
  using E4 = typename ConvLp<LP>::e4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cb = wave & 3, hb = wave >> 2, lh = lane >> 5, lc = lane & 31;
  for (int c = tid; c < R * 2 * PW * (CI / 8); c += NT) {   // the halo positions, once
    const int rl = c / (2 * PW * (CI / 8)), rem = c % (2 * PW * (CI / 8));
    const int pp = rem / (CI / 8), ch = rem % (CI / 8);
    const int q = pp < PW ? pp : WD + pp;
    *reinterpret_cast<u32x4_*>(Xl + (rl * WP + q) * XP + ch * 8) = u32x4_{0u, 0u, 0u, 0u};
  }
  u32x4_ xr[XPT];
  v4f yr[YPT];
  unsigned ar[YPT];
  const auto rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(a.x16), (short)0, 0x7ffffff0, 0x00020000);
  const auto rsY = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.dy), (short)0, 0x7ffffff0, 0x00020000);
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.arg), (short)0, 0x7ffffff0, 0x00020000);
  constexpr int kOOB = (int)0x80000000u;
  auto fetch = [&](int g) {   // tile g's rows into registers (past the last row: zeros)
    const int real = a.rows - g * R;
    const int sx = __builtin_amdgcn_readfirstlane(g * R * WD * CI * 2);
    const int sy = __builtin_amdgcn_readfirstlane(g * R * PQ * CO * 4);
    const int sa = __builtin_amdgcn_readfirstlane(g * R * PQ * CO);
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT;
      xr[i] = __builtin_bit_cast(u32x4_, __builtin_amdgcn_raw_buffer_load_b128(
                                              rsX, c < real * WD * (CI / 8) ? sx + c * 16 : kOOB, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int c = tid + i * NT;
      const bool ok = c < real * PQ * (CO / 4);
      yr[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rsY, ok ? sy + c * 16 : kOOB, 0, 0));
      ar[i] = __builtin_amdgcn_raw_buffer_load_b32(rsA, ok ? sa + c * 4 : kOOB, 0, 0);
    }
  };
  // dY unit swizzle: 16-B unit u (8 channels) of pixel p at slot u ^ ((p & 3) << 2)
  auto yoff = [](int p, int n) { return p * CO + ((((n >> 3) ^ ((p & 3) << 2))) << 3) + (n & 7); };
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};   // channels 4 (tid % 32) .. + 3 (every chunk of this thread)
  auto stage = [&]() {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int c = tid + i * NT, rl = c / (WD * (CI / 8)), rem = c % (WD * (CI / 8));
      const int px = rem / (CI / 8), ch = rem % (CI / 8);
      *reinterpret_cast<u32x4_*>(Xl + (rl * WP + px + PW) * XP + ch * 8) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int c = tid + i * NT, rl = c / (PQ * (CO / 4)), rem = c % (PQ * (CO / 4));
      const int q = rem / (CO / 4), n = (rem % (CO / 4)) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) bsum[e] += yr[i][e];
#pragma unroll
      for (int pp = 0; pp < 4; ++pp) {   // the pooled value at the window position its argmax names, zeros elsewhere
        v4f v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = ((ar[i] >> (8 * e)) & 0xFFu) == (unsigned)pp ? yr[i][e] : 0.f;
        *reinterpret_cast<u32x2_*>(Yl + yoff(rl * WD + 4 * q + pp, n)) = __builtin_bit_cast(u32x2_, __builtin_convertvector(v, E4));
      }
    }
  };
  f32x16 acc[KW];
#pragma unroll
  for (int t = 0; t < KW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  // this lane's tr16 addresses: 4 channels (m = 16 ((lane >> 4) & 1) + 4 (lane & 3) of its 32-block) at pixel
  // 16 s + 8 lh + q of k-step s (q = (lane >> 2) & 3) and at + 4 (the fragment's upper half); an 8-pixel run never
  // crosses a row (WD % 8 == 0), so both halves sit in the same staged row
  const int q4 = (lane >> 2) & 3, mo = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  const unsigned short* xl = Xl + hb * 32 + mo;
  const unsigned short* yl = Yl + yoff(8 * lh + q4, cb * 32 + mo);   // pixel 8 lh + q4; + 16 s pixels = 16 s * CO
  int g = blockIdx.x;
  if (g < a.groups) fetch(g);
  while (g < a.groups) {
    stage();
    __syncthreads();
    const int gn = g + (int)gridDim.x;
    if (gn < a.groups) fetch(gn);   // lands during the MFMAs below
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int p0 = 16 * s + 8 * lh + q4;          // this lane's pixel (lower half)
      const int pos = p0 + 2 * PW * (p0 / WD);       // its staged position (tap 0 = pixel - PW + PW)
      const unsigned short* xb = xl + pos * XP;
      const unsigned short* yb = yl + 16 * s * CO;   // (16 s) & 3 == 0: the same swizzle as pixel 8 lh + q4
      const s16x4 blo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)yb);
      const s16x4 bhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(yb + 4 * CO));
      const u32x2_ b2l = __builtin_bit_cast(u32x2_, blo), b2h = __builtin_bit_cast(u32x2_, bhi);
      const u32x4_ bf = u32x4_{b2l.x, b2l.y, b2h.x, b2h.y};
#pragma unroll
      for (int t = 0; t < KW; ++t) {
        const s16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xb + t * XP));
        const s16x4 ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xb + (t + 4) * XP));
        const u32x2_ l2 = __builtin_bit_cast(u32x2_, alo), h2 = __builtin_bit_cast(u32x2_, ahi);
        acc[t] = ConvLp<LP>::mma(u32x4_{l2.x, l2.y, h2.x, h2.y}, bf, acc[t]);
      }
    }
    __syncthreads();   // every wave is done reading the tile before the next one is staged
    g = gn;
  }
  float* sl = a.slab + (size_t)blockIdx.x * (KW * CI * CO);
#pragma unroll
  for (int t = 0; t < KW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ci = hb * 32 + 8 * (r >> 2) + 4 * lh + (r & 3);
      sl[(t * CI + ci) * CO + cb * 32 + lc] = acc[t][r];
    }
  if (a.bpart) {   // the 16 thread rows sharing channels 4 (tid % 32) .. + 3, added in row order
#pragma unroll
    for (int e = 0; e < 4; ++e) Bs[tid / (CO / 4)][(tid % (CO / 4)) * 4 + e] = bsum[e];
    __syncthreads();
    if (tid < CO) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < NT / (CO / 4); ++r) t += Bs[r][tid];
      a.bpart[(size_t)blockIdx.x * CO + tid] = t;
    }
  }
}

// The data gradient of the same conv: dX[w][ci] = sum over (kw, co) of dY[w + PW - kw][co] Wd[(kw,
// co)][ci] — the implicit GEMM's k order, so bitwise its result.  dY (128 channels) has twice the bytes per staged
// position, so the weights cannot stay resident beside 8 staged rows: the workgroup stages 8 rows of the dense 16-bit
// dY once per tile (94 KB) and streams the weight matrix one tap at a time ([128 k][64 ci], 16 KB, double-buffered,
// the next tap's loads in flight during this tap's MFMAs; the whole matrix stays in L2).  4 waves over the 320 x 64
// tile: row blocks 3 / 3 / 2 / 2 per wave x both 32-column blocks (at most 5 fragment reads per 6 MFMAs).
struct RowDgArgs {
  const unsigned short* dy16;   // [rows][W][CA] dense 16-bit dY
  const unsigned short* wd16;   // [(kw, co)][CN] 16-bit (the dgrad weight matrix Wd)
  float* dx;                    // [rows][W][CN]
  int rows, groups;
  const float* dyp;             // POOLED: [rows][W / 4][CA] fp32 pooled gradient (instead of dy16) ...
  const uint8_t* argp;          // ... and its window argmax, unpooled and rounded to 16 bits at staging
};
// BAL (option conv_row16_dgrad = 2): the 20 (row block, column block) units of the tile 5 per wave instead —
// wave w owns units 5w .. 5w + 4 (unit u = row block u / 2, column block u % 2): 3 A + 2 B fragment reads per 5
// MFMAs, every SIMD the same MFMA count (the 3 / 3 / 2 / 2 split leaves two SIMDs idle 1/3 of each k-step).
// POOLED: dY arrives as the pooled gradient + argmax (fbanks_cnn's pooled backward) and is unpooled and rounded at
// staging — the staged values bitwise those of unpool16 + to16 (the same conversion), without the dense 16-bit dY in
// HBM (and without the pass that writes it).
template <int LP, int KW, int PW, int WD, int CA, int CN, int R, bool BAL = false, bool POOLED = false>
__global__ __launch_bounds__(256, 1) void conv_row16_dgrad_kernel(RowDgArgs a) {
  static_assert(CA == 128 && CN == 64 && (R * WD) % 32 == 0 && 2 * PW == KW - 1, "row16 dgrad geometry");
  constexpr int WP = WD + 2 * PW;
  constexpr int MB = R * WD / 32;               // 10 row blocks
  constexpr int XCH = R * WD * (CA / 8);        // 16-B chunks of a tile's dY rows (5120)
  constexpr int XPT = XCH / 256;                // per thread (20)
  constexpr int TCH = CA * CN / 8;              // 16-B chunks of one tap's weights (1024)
  constexpr int TPT = TCH / 256;                // per thread (4)
  static_assert(MB == 10 && XCH % 256 == 0 && TCH % 256 == 0, "row16 dgrad tile split");
  __shared__ __attribute__((aligned(16))) unsigned short Yl[R * WP * CA];    // staged dY rows, chunks swizzled
  // one tap of Wd as a TR image [k][128] (r16_off<false>, the ring kernels' layout; columns 64..127 unused)
  __shared__ __attribute__((aligned(16))) unsigned short Wt[2][CA * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // row blocks of this wave: rs .. rs + rn - 1 (BAL: the 3 row blocks its 5 units touch)
  const int rs = BAL ? (5 * wave) >> 1 : (wave < 2 ? 3 * wave : 6 + 2 * (wave - 2)), rn = BAL || wave < 2 ? 3 : 2;
  for (int c = tid; c < R * 2 * PW * (CA / 8); c += 256) {   // halo positions, once
    const int rl = c / (2 * PW * (CA / 8)), rem = c % (2 * PW * (CA / 8));
    const int pp = rem / (CA / 8), ch = rem % (CA / 8);
    const int q = pp < PW ? pp : WD + pp;
    *reinterpret_cast<u32x4_*>(Yl + (rl * WP + q) * CA + ((ch ^ (q & 15)) * 8)) = u32x4_{0u, 0u, 0u, 0u};
  }
  constexpr int PCH = R * (WD / 4) * (CA / 4);   // POOLED: 16-B chunks of the pooled fp32 rows (2560)
  constexpr int PPT = PCH / 256;                  // per thread (10)
  static_assert(!POOLED || (PCH % 256 == 0 && WD % 4 == 0), "row16 dgrad pooled tile split");
  u32x4_ yr[POOLED ? 1 : XPT], wr[TPT];
  v4f pr[POOLED ? PPT : 1];
  unsigned par[POOLED ? PPT : 1];
  // the loads take 32-bit buffer offsets (past the last row -> 16 zero bytes): 64-bit addresses of the 20 + 4 loads,
  // hoisted out of the loops, spilled; the epilogue stores 32-bit offsets off the tile's base pointer
  const auto rsY = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(a.dy16), (short)0, 0x7ffffff0, 0x00020000);
  const auto rsW = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(a.wd16), (short)0, 0x7ffffff0, 0x00020000);
  const auto rsP = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(POOLED ? a.dyp : nullptr), (short)0, 0x7ffffff0,
                                                     0x00020000);
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(POOLED ? a.argp : nullptr), (short)0,
                                                     0x7ffffff0, 0x00020000);
  auto fetch_y = [&](int g) {
    if constexpr (POOLED) {
      const int lastp = (a.rows - g * R) * (WD / 4) * (CA / 4);
      const int sp = __builtin_amdgcn_readfirstlane(g * R * (WD / 4) * CA * 4);
      const int sa = __builtin_amdgcn_readfirstlane(g * R * (WD / 4) * CA);
#pragma unroll
      for (int i = 0; i < PPT; ++i) {
        const int c = tid + i * 256;
        const bool ok = c < lastp;
        pr[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rsP, ok ? sp + c * 16 : (int)0x80000000u, 0, 0));
        par[i] = __builtin_amdgcn_raw_buffer_load_b32(rsA, ok ? sa + c * 4 : (int)0x80000000u, 0, 0);
      }
    } else {
      const int last = (a.rows - g * R) * WD * (CA / 8);   // chunks of real rows in this tile
      const int sbase = __builtin_amdgcn_readfirstlane(g * R * WD * CA * 2);
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int c = tid + i * 256;
        yr[i] = __builtin_bit_cast(u32x4_, __builtin_amdgcn_raw_buffer_load_b128(
                                                rsY, c < last ? sbase + c * 16 : (int)0x80000000u, 0, 0));
      }
    }
  };
  auto stage_y = [&]() {
    if constexpr (POOLED) {
      using E4 = typename ConvLp<LP>::e4;
#pragma unroll
      for (int i = 0; i < PPT; ++i) {
        const int c = tid + i * 256, rl = c / ((WD / 4) * (CA / 4)), rem = c % ((WD / 4) * (CA / 4));
        const int q4 = rem / (CA / 4), n = (rem % (CA / 4)) * 4, ch = n >> 3;
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {   // the pooled value at the position its argmax names, zeros elsewhere
          const int q = 4 * q4 + pp + PW;
          v4f v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = ((par[i] >> (8 * e)) & 0xFFu) == (unsigned)pp ? pr[i][e] : 0.f;
          *reinterpret_cast<u32x2_*>(Yl + (rl * WP + q) * CA + ((ch ^ (q & 15)) * 8) + (n & 4)) =
              __builtin_bit_cast(u32x2_, __builtin_convertvector(v, E4));
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int c = tid + i * 256, rl = c / (WD * (CA / 8)), rem = c % (WD * (CA / 8));
        const int px = rem / (CA / 8), ch = rem % (CA / 8), q = px + PW;
        *reinterpret_cast<u32x4_*>(Yl + (rl * WP + q) * CA + ((ch ^ (q & 15)) * 8)) = yr[i];
      }
    }
  };
  auto fetch_w = [&](int kw) {
    const int sbase = __builtin_amdgcn_readfirstlane(kw * CA * CN * 2);
#pragma unroll
    for (int i = 0; i < TPT; ++i)
      wr[i] = __builtin_bit_cast(u32x4_, __builtin_amdgcn_raw_buffer_load_b128(rsW, sbase + (tid + i * 256) * 16, 0, 0));
  };
  auto stage_w = [&](int buf) {
#pragma unroll
    for (int i = 0; i < TPT; ++i) {
      const int c = tid + i * 256, k = c / (CN / 8), col = (c % (CN / 8)) * 8;
      *reinterpret_cast<u32x4_*>(&Wt[buf][r16_off<false>(col, k)]) = wr[i];
    }
  };
  int arow[3], apos[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int p = (rs + (i < rn ? i : 0)) * 32 + (lane & 31);
    arow[i] = (p / WD) * WP;
    apos[i] = p % WD;
  }
  const int khalf = lane >> 5, lh = lane >> 5, lc = lane & 31;
  int g = blockIdx.x;
  if (g < a.groups) fetch_y(g);
  fetch_w(0);
  while (g < a.groups) {
    stage_y();
    stage_w(0);
    __syncthreads();
    const int gn = g + (int)gridDim.x;
    float* const xbase = a.dx + (size_t)g * R * WD * CN;
    const int nreal = (a.rows - g * R) * WD;   // real pixels of this tile
    if constexpr (BAL) {
      // unit k of wave parity P: local row block (P + k) / 2, column block (P + k) % 2 (wave-uniform branch)
      auto run = [&](auto par) {
        constexpr int P = decltype(par)::value;
        f32x16 acc[5];
#pragma unroll
        for (int k = 0; k < 5; ++k)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;
#pragma unroll 1
        for (int kw = 0; kw < KW; ++kw) {
          fetch_w(kw + 1 < KW ? kw + 1 : 0);
          if (kw == KW - 1 && gn < a.groups) fetch_y(gn);   // the next tile's rows under the last tap's MFMAs
          const unsigned short* Ws = Wt[kw & 1];
#pragma unroll 1
          for (int c0 = 0; c0 < CA; c0 += 16) {
            const u32x4_ bq[2] = {r16_frag<false>(Ws, 0, c0, lane), r16_frag<false>(Ws, 32, c0, lane)};
            const int ch = (c0 >> 3) + khalf;
            u32x4_ af[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              const int q = apos[i] + 2 * PW - kw;
              af[i] = *reinterpret_cast<const u32x4_*>(Yl + (arow[i] + q) * CA + ((ch ^ (q & 15)) * 8));
            }
#pragma unroll
            for (int k = 0; k < 5; ++k) acc[k] = ConvLp<LP>::mma(af[(P + k) >> 1], bq[(P + k) & 1], acc[k]);
          }
          if (kw + 1 < KW) stage_w((kw + 1) & 1);
          __syncthreads();
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) {
          const int cb = ((P + k) & 1) * 32;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int p = (rs + ((P + k) >> 1)) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (p < nreal) xbase[p * CN + cb + lc] = acc[k][r];
          }
        }
      };
      if (wave & 1) run(std::integral_constant<int, 1>{});
      else run(std::integral_constant<int, 0>{});
    } else {
      f32x16 acc[3][2];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll 1
      for (int kw = 0; kw < KW; ++kw) {
        fetch_w(kw + 1 < KW ? kw + 1 : 0);   // the next tap (tap 0 again for the next tile)
        const unsigned short* Ws = Wt[kw & 1];
#pragma unroll 1
        for (int c0 = 0; c0 < CA; c0 += 16) {
          const u32x4_ b0 = r16_frag<false>(Ws, 0, c0, lane), b1 = r16_frag<false>(Ws, 32, c0, lane);
          const int ch = (c0 >> 3) + khalf;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            if (i < rn) {
              const int q = apos[i] + 2 * PW - kw;   // dY position w + PW - kw, in the staged (haloed) row
              const u32x4_ af = *reinterpret_cast<const u32x4_*>(Yl + (arow[i] + q) * CA + ((ch ^ (q & 15)) * 8));
              acc[i][0] = ConvLp<LP>::mma(af, b0, acc[i][0]);
              acc[i][1] = ConvLp<LP>::mma(af, b1, acc[i][1]);
            }
          }
        }
        if (kw + 1 < KW) stage_w((kw + 1) & 1);   // that buffer was last read in tap kw - 1 (behind the barrier)
        __syncthreads();
      }
      // dX rows of this wave's blocks (fp32, 32 consecutive channels per half-wave store)
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (i >= rn) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int p = (rs + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (p < nreal) {   // global stores off the tile's base (buffer stores here landed wrong on the GPU)
            xbase[p * CN + lc] = acc[i][0][r];
            xbase[p * CN + lc + 32] = acc[i][1][r];
          }
        }
      }
    }
    // the next tile's dY rows after the accumulators are dead (their registers; prefetching them during the MFMAs
    // spilled): the load latency is paid once per tile (BAL: 80 accumulator registers, so under the last tap)
    if (!BAL && gn < a.groups) fetch_y(gn);
    g = gn;
  }
}

// The ring conv when the shape qualifies (fp32 operands, option conv_ring, channel-aligned, stride 1
// for the data gradient, 32-bit byte offsets); returns 1 if it did not run.
// Algorithmic HBM bytes of one implicit-GEMM conv launch (ProfScope::bytes): the two operand tensors read once
// at their element size in HBM (esz: 2 for 16-bit sources, 4 otherwise) and the output written once in fp32
// (a pooled forward: the pooled values + their uint8 argmax).  fwd: x, W -> y; dgrad: dY, W -> dX; wgrad:
// x, dY -> dW.  A pooled backward's gathers read the pooled dY + argmax instead of the dense dY.
inline double conv_bytes(const ConvArgs& c, int mode, int esz) {
  const double x = (double)c.N * c.H * c.W * c.Ci, y = (double)c.N * c.Ho * c.Wo * c.Co,
               w = (double)c.KH * c.KW * c.Ci * c.Co;
  const double dy = c.dy_arg ? y / 4.0 * (esz + 1.0) : y * esz;
  if (mode == kFwd) return (x + w) * esz + (c.pool_w ? y / c.pool_w * 5.0 : y * 4.0);
  if (mode == kDgrad) return dy + w * esz + x * 4.0;
  return x * esz + dy + w * 4.0;
}

template <int MODE>
int try_conv_ring(ConvArgs& c, hipStream_t s, const char* name, float* final_out, float** partial_out, int* splits_out) {
  const int prec = matmul_prec();
  const bool lp = prec != kPrecF32;
  // fp32 operands (option bits 0..2), or the 16-bit operand copies of the S16 path (bits 4..6)
  if (!(g_opt_conv_ring & (1 << (MODE + (lp ? 4 : 0)))) || c.dy_arg || (lp != (c.a16 != nullptr))) return 1;
  // the pooled forward (fbanks_cnn conv2) measured slower on the ring (r04ab: fp32; r04ab3: 16-bit, 2.89
  // vs 2.68 ms per 5 cfg3 steps): only with bit 7
  if (MODE == kFwd && c.pool_w && !(g_opt_conv_ring & 0x80)) return 1;
  // fp32 forward: faster on the deep-K ResNet layers (r04ab6, cfg4: 64000 x 512 x 7680 and 128000 x 256 x
  // 3840 -8 %), slower on fbanks_cnn conv4 (50176 x 512 x 1792: +2 %)
  if (!lp && MODE == kFwd && c.K < 3072 && !(g_opt_conv_ring & 0x80)) return 1;
  const int RBK = lp ? kR16BK : kRBK, unit = lp ? 8 : 4, esz = lp ? 2 : 4;
  const int chans = MODE == kDgrad ? c.Co : c.Ci;
  if (MODE != kWgrad && chans % RBK) return 1;
  if (MODE == kWgrad && c.Ci % unit) return 1;
  if (MODE == kDgrad && (c.sh != 1 || c.sw != 1)) return 1;
  if (c.Nn % unit || c.Nn < 128 || c.M < 256 || c.M >= INT32_MAX || c.K >= INT32_MAX)
    return 1;
  const double xb = (double)esz * c.N * c.H * c.W * c.Ci, yb = (double)esz * c.N * c.Ho * c.Wo * c.Co,
               wb = (double)esz * c.K * c.Nn;
  if (xb >= 2.1e9 || yb >= 2.1e9 || wb >= 2.1e9) return 1;
  const int BN = c.Nn >= 256 ? 256 : 128;
  const int64_t tm = (c.M + 255) / 256, tn = (c.Nn + BN - 1) / BN;
  int splits0 = choose_splits(tm * tn, c.K, RBK, kCUs, MODE == kWgrad ? 256 : 16);
  if (MODE != kWgrad && splits0 > 1) {
    // a split forward / data gradient writes and re-reads its full-size output once per split (the slabs)
    // before the reduction writes it: keep the split only where the MFMA rounds it saves outweigh that traffic
    // (fbanks_cnn conv4's 16-bit forward, 50176 x 512 x 1792: 392 tiles, 181 us on 784 half-K blocks + a 91 us
    // slab reduction vs ~180 us unsplit; the fp32 ResNet layers keep theirs).  Rates: the ring kernels' measured
    // ~0.5 PF (16-bit) / ~0.11 PF (fp32), ~4 TB/s for the slab traffic.
    const double rate = lp ? 0.5e15 : 0.11e15, flops = 2.0 * (double)c.M * (double)c.Nn * (double)c.K;
    auto t_of = [&](int64_t sp) {
      const int64_t w = tm * tn * sp, rounds = (w + kCUs - 1) / kCUs;
      const double eff = (double)w / (double)(rounds * kCUs);
      return flops / (eff * rate) + (sp > 1 ? 2.0 * sp * 4.0 * (double)c.M * (double)c.Nn / 4e12 : 0.0);
    };
    if (t_of(1) <= t_of(splits0)) splits0 = 1;
  }
  c.kchunk = splits0 > 1 ? ((c.K + splits0 - 1) / splits0 + RBK - 1) / RBK * RBK : std::max<int64_t>(c.K, 1);
  const int splits = splits0 > 1 ? (int)((c.K + c.kchunk - 1) / c.kchunk) : 1;
  c.tiles_m = (int)tm;
  c.tiles_n = (int)tn;
  c.tiles = (int)(tm * tn);
  c.nblk = c.tiles * splits;
  c.group_m = std::max(1, (int)std::lround(std::sqrt(32.0 * BN / 256.0)));
  c.partial = nullptr;
  if (splits > 1) {
    if (int rc = conv_scratch((size_t)splits * c.M * c.Nn, &c.partial)) return rc;
  }
  c.colsum_part = nullptr;
  if (MODE == kWgrad && c.db && !lp) {   // the 16-bit path keeps the column-sum kernel (fp32 dY)
    if (int rc = conv_scratch((size_t)splits * c.Nn, &c.colsum_part, g_csb)) return rc;
  }
  c.fd_w = FastDiv((unsigned)(MODE == kDgrad ? c.W : c.Wo));
  c.fd_h = FastDiv((unsigned)(MODE == kDgrad ? c.H : c.Ho));
  c.fd_c = FastDiv((unsigned)chans);
  c.fd_kw = FastDiv((unsigned)c.KW);
  ProfScope prof(lp ? (MODE == kFwd ? "conv_fwd_lp" : MODE == kDgrad ? "conv_dgrad_lp" : "conv_wgrad_lp") : name, s,
                 2.0 * (double)c.M * (double)c.Nn * (double)c.K);
  prof.bytes(conv_bytes(c, MODE, lp ? 2 : 4));
  prof.detail("conv_ring%s_kernel<%s,256x%d%s%s> %lldx%lldx%lld s%d", lp ? "16" : "",
              MODE == kFwd ? "fwd" : MODE == kDgrad ? "dgrad" : "wgrad", BN, (MODE == kFwd && c.pool_w) ? ",pool" : "",
              lp && ((g_opt_conv_ring_qs >> (BN == 128 ? 1 : 2)) & 1) ? ",qs2" : "",
              (long long)c.M, (long long)c.Nn, (long long)c.K, splits);
  const dim3 grid((unsigned)c.nblk), block(512);
  if (!lp) {
    if (BN == 256) hipLaunchKernelGGL((conv_ring_kernel<MODE, 256>), grid, block, 0, s, c);
    else hipLaunchKernelGGL((conv_ring_kernel<MODE, 128>), grid, block, 0, s, c);
  } else {
    // the 16-bit ring: BN x precision x k-steps per section (QS 2 where the option asks for it at this width:
    // bit 1 BN 128, bit 2 BN 256)
    const bool qs2 = (g_opt_conv_ring_qs >> (BN == 128 ? 1 : 2)) & 1;
#define SRK_R16(BN_, LP_)                                                                                   \
  if (qs2) hipLaunchKernelGGL((conv_ring16_kernel<MODE, BN_, LP_, 2>), grid, block, 0, s, c);              \
  else hipLaunchKernelGGL((conv_ring16_kernel<MODE, BN_, LP_, 1>), grid, block, 0, s, c);
    if (prec == kPrecBF16) {
      if (BN == 256) { SRK_R16(256, 1) } else { SRK_R16(128, 1) }
    } else {
      if (BN == 256) { SRK_R16(256, 2) } else { SRK_R16(128, 2) }
    }
#undef SRK_R16
  }
  SRK_CHECK_HIP(hipGetLastError());
  *partial_out = c.partial;
  *splits_out = splits;
  (void)final_out;
  return 0;
}

template <int MODE>
int run_conv_gemm(ConvArgs c, hipStream_t s, const char* name) {
  {
    ConvArgs r = c;
    float* partial = nullptr;
    int splits = 1;
    const int rc = try_conv_ring<MODE>(r, s, name, c.out, &partial, &splits);
    if (rc == 0) {
      if (splits > 1) {   // slab reduction (+ bias), then the pooled output / bias sums as below
        const bool pool = MODE == kFwd && c.pool_w;
        float* dense = c.out;
        if (pool && (rc == 0)) {
          if (int e = conv_scratch((size_t)c.M * c.Nn, &dense, g_csd)) return e;
        }
        const int64_t n = c.M * c.Nn;
        launch_splitk_sum(partial, splits, n, c.Nn, MODE == kFwd ? c.bias : nullptr, dense, s);
        if (pool) {
          const int64_t rows = c.M / c.pool_w;
          hipLaunchKernelGGL(maxpool_arg_kernel, dim3((unsigned)((rows * c.Nn + 255) / 256)), dim3(256), 0, s, dense,
                             rows, (int)c.Nn, c.pool_w, c.out, c.pool_arg);
        }
        SRK_CHECK_HIP(hipGetLastError());
      }
      if (r.colsum_part) {
        hipLaunchKernelGGL(colsum_splits_kernel, dim3((unsigned)((c.Nn + 255) / 256)), dim3(256), 0, s, r.colsum_part,
                           splits, c.Nn, c.db);
        SRK_CHECK_HIP(hipGetLastError());
      }
      return SRK_OK;
    }
    if (rc != 1) return rc;
  }
  const int prec = matmul_prec();
  const int BK = prec == kPrecF32 ? 32 : 64;   // 16-bit: 64-deep k-tiles (4 MFMA k-steps per barrier)
  // tile: 128 x 128 unless the GEMM is narrow (N <= 64: 128 x 64) or small (64 x 64); srk option
  // conv_tile = 256: 256 x BN tiles of 8 waves on tall GEMMs with vector gathers
  int BM = 128, BN = c.Nn <= 64 ? 64 : 128, NW = 4;
  if (((c.M + 127) / 128) * ((c.Nn + BN - 1) / BN) < 64 && c.K < 2048) { BM = 64; BN = 64; }
  {
    const int chans_ = MODE == kDgrad ? c.Co : c.Ci;
    const bool vec_ = chans_ % 4 == 0 && c.Nn % 4 == 0;
    if (g_opt_conv_tile == 256 && prec == kPrecF32 && BM == 128 && vec_ &&
        ((c.M + 255) / 256) * ((c.Nn + BN - 1) / BN) >= kCUs) {
      BM = 256;
      NW = 8;
    }
  }
  const int64_t tm = (c.M + BM - 1) / BM, tn = (c.Nn + BN - 1) / BN;
  SRK_REQUIRE(tm * tn <= (INT32_MAX >> 9), SRK_ERR_INVALID, "conv: grid too large");
  const int lds = prec == kPrecF32 ? 2 * 4 * ((MODE != kWgrad ? BM * (BK + 4) : BK * (BM + 8)) + BK * (BN + 8))
                                   : 2 * 2 * ((MODE != kWgrad ? BM * (BK + 8) : BK * kTrPitch) + BK * kTrPitch);
  const int64_t slots = (int64_t)kCUs * std::min(8, (160 * 1024) / lds);
  // weight-gradient GEMMs reduce over every pixel (K up to millions) onto a few hundred tiles:
  // allow deep splits there (deterministic slab reduction)
  const int splits0 = choose_splits(tm * tn, c.K, BK, slots, MODE == kWgrad ? 256 : 16);
  c.kchunk = splits0 > 1 ? ((c.K + splits0 - 1) / splits0 + BK - 1) / BK * BK : std::max<int64_t>(c.K, 1);
  const int splits = splits0 > 1 ? (int)((c.K + c.kchunk - 1) / c.kchunk) : 1;
  c.tiles_m = (int)tm;
  c.tiles_n = (int)tn;
  c.tiles = (int)(tm * tn);
  c.nblk = c.tiles * splits;
  c.group_m = 8;
  c.partial = nullptr;
  float* final_out = c.out;
  float* pooled_out = nullptr;
  int pool_w = 0;
  if (splits > 1) {
    if (int rc = conv_scratch((size_t)splits * c.M * c.Nn, &c.partial)) return rc;
    if (MODE == kFwd && c.pool_w) {   // no pooled epilogue across split-K slabs: dense, then pool
      pooled_out = c.out;
      if (int rc = conv_scratch((size_t)c.M * c.Nn, &final_out, g_csd)) return rc;
      pool_w = c.pool_w;
      c.pool_w = 0;
    }
  }
  c.colsum_part = nullptr;
  if (MODE == kWgrad && c.db && !c.a16) {
    if (int rc = conv_scratch((size_t)splits * c.Nn, &c.colsum_part, g_csb)) return rc;
  }
  const int chans = MODE == kDgrad ? c.Co : c.Ci;
  SRK_REQUIRE(c.M < INT32_MAX && c.K < INT32_MAX, SRK_ERR_INVALID, "conv: implicit-GEMM extent >= 2^31");
  c.fd_w = FastDiv((unsigned)(MODE == kDgrad ? c.W : c.Wo));
  c.fd_h = FastDiv((unsigned)(MODE == kDgrad ? c.H : c.Ho));
  c.fd_c = FastDiv((unsigned)chans);
  c.fd_kw = FastDiv((unsigned)c.KW);
  c.fd_sh = FastDiv((unsigned)c.sh);
  c.fd_sw = FastDiv((unsigned)c.sw);
  const bool vecb = c.Nn % 4 == 0;
  const bool vec = (chans % 4 == 0) && vecb;
  {
    // fast16 gathers (ConvArgs::fast16): one tap per K-tile, 32-bit buffer offsets
    const double ael = MODE == kDgrad ? (double)c.N * c.Ho * c.Wo * c.Co : (double)c.N * c.H * c.W * c.Ci;
    c.fast16 = g_opt_conv_fast16 && c.a16 && MODE != kWgrad && chans % BK == 0 && c.kchunk % BK == 0 &&
               (MODE != kDgrad || (c.sh == 1 && c.sw == 1)) && ael < 1073741824.0 &&
               (double)c.K * c.Nn < 1073741824.0 && (double)c.M < 2147483647.0;
  }
  SRK_REQUIRE(!c.a16 || (prec != kPrecF32 && c.b16 && chans % 8 == 0 && c.Nn % 8 == 0), SRK_ERR_INTERNAL,
              "conv: 16-bit sources need 8-aligned channels");
  SRK_REQUIRE(!c.dy_arg || (MODE != kFwd && !c.a16 && vec && vecb && c.sh == 1 && c.sw == 1 && c.Wo % 4 == 0),
              SRK_ERR_INTERNAL, "conv: unpooling gathers need fp32 sources, 4-aligned channels and Wo % 4 == 0");
  ProfScope prof(prec == kPrecF32 ? name : (MODE == kFwd ? "conv_fwd_lp" : MODE == kDgrad ? "conv_dgrad_lp" : "conv_wgrad_lp"),
                 s, 2.0 * (double)c.M * (double)c.Nn * (double)c.K);
  prof.bytes(conv_bytes(c, MODE, c.a16 ? 2 : 4));
  prof.detail("conv_gemm_kernel<%s,%dx%d%s%s%s> %lldx%lldx%lld s%d", MODE == kFwd ? "fwd" : MODE == kDgrad ? "dgrad" : "wgrad",
              BM, BN, NW == 8 ? ",8w" : "", c.a16 ? ",s16" : c.dy_arg ? ",unpool" : (MODE == kFwd && c.pool_w) ? ",pool" : "",
              c.fast16 ? ",fast" : "", (long long)c.M, (long long)c.Nn, (long long)c.K, splits);
  const dim3 grid((unsigned)c.nblk);
  if (BM == 64) launch_conv<MODE, 64, 64>(c, grid, s, vec, vecb, prec);
  else if (BM == 256 && BN == 64) launch_conv<MODE, 256, 64, 8>(c, grid, s, vec, vecb, prec);
  else if (BM == 256) launch_conv<MODE, 256, 128, 8>(c, grid, s, vec, vecb, prec);
  else if (BN == 64) launch_conv<MODE, 128, 64>(c, grid, s, vec, vecb, prec);
  else launch_conv<MODE, 128, 128>(c, grid, s, vec, vecb, prec);
  SRK_CHECK_HIP(hipGetLastError());
  if (splits > 1) {
    const int64_t n = c.M * c.Nn;
    launch_splitk_sum(c.partial, splits, n, c.Nn, MODE == kFwd ? c.bias : nullptr, final_out, s);
    SRK_CHECK_HIP(hipGetLastError());
    if (pooled_out) {
      const int64_t rows = c.M / pool_w;
      hipLaunchKernelGGL(maxpool_arg_kernel, dim3((unsigned)((rows * c.Nn + 255) / 256)), dim3(256), 0, s, final_out,
                         rows, (int)c.Nn, pool_w, pooled_out, c.pool_arg);
      SRK_CHECK_HIP(hipGetLastError());
    }
  }
  if (c.colsum_part) {
    hipLaunchKernelGGL(colsum_splits_kernel, dim3((unsigned)((c.Nn + 255) / 256)), dim3(256), 0, s, c.colsum_part,
                       splits, c.Nn, c.db);
    SRK_CHECK_HIP(hipGetLastError());
  }
  return SRK_OK;
}

// fbanks_cnn conv2's pooled backward in 16-bit modes (options conv_row16 and conv_row16_dgrad on): both gradients on
// the row-staged kernels straight from the pooled gradient + argmax — the data gradient (conv_row16_dgrad_kernel
// <POOLED>) and the weight gradient (conv_row16_wgrad_kernel, one slab per workgroup reduced in order, the bias sums
// in the same pass) unpool and round dY at staging, so the dense 16-bit dY (and the pass that writes it with the
// bias sums, colsum8 / unpool16) is never made.  x's 16-bit copy is the forward's when it kept one.
int conv2_bwd16_pooled(const float* x, int64_t N, int64_t H, const float* w, const float* dyp, const uint8_t* arg,
                       float* dx, float* dw, float* db, float* ws, const void* x16, hipStream_t s) {
  constexpr int64_t W = 40, Ci = 64, Co = 128, KH = 1, KW = 7;
  const int prec = matmul_prec();
  const int64_t nw = Co * Ci * KH * KW, rows = N * H, groups = (rows + 7) / 8;
  int rc;
  if (dx)
    hipLaunchKernelGGL(weight_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, w, (int)Co, (int)Ci,
                       (int)KH, (int)KW, 1, ws);
  unsigned short* d16[2] = {static_cast<unsigned short*>(const_cast<void*>(x16)), nullptr};   // x, Wd
  {
    const float* src[2] = {x, ws};
    const int64_t n[2] = {rows * W * Ci, nw};
    const bool ready[2] = {x16 != nullptr, false};
    if ((rc = to16_all(prec, src, n, dx ? 2 : 1, d16, s, ready))) return rc;
  }
  if (dx) {
    RowDgArgs ra{};
    ra.wd16 = d16[1];
    ra.dx = dx;
    ra.rows = (int)rows;
    ra.groups = (int)groups;
    ra.dyp = dyp;
    ra.argp = arg;
    ProfScope prof("conv_dgrad_lp", s, 2.0 * (double)(rows * W) * (double)Ci * (double)(KW * Co));
    prof.detail("conv_row16_dgrad_kernel<unpool> %lldx%lldx%lld", (long long)(rows * W), (long long)Ci, (long long)(KW * Co));
    prof.bytes(5.0 / 4.0 * (double)(rows * W) * Co + 2.0 * (double)(KW * Co) * Ci + 4.0 * (double)(rows * W) * Ci);
    const dim3 grid((unsigned)std::min<int64_t>(groups, kCUs)), block(256);
    const bool bal = g_opt_conv_row16_dgrad == 2;
    if (prec == kPrecBF16 && bal)
      hipLaunchKernelGGL((conv_row16_dgrad_kernel<1, 7, 3, 40, 128, 64, 8, true, true>), grid, block, 0, s, ra);
    else if (prec == kPrecBF16)
      hipLaunchKernelGGL((conv_row16_dgrad_kernel<1, 7, 3, 40, 128, 64, 8, false, true>), grid, block, 0, s, ra);
    else if (bal)
      hipLaunchKernelGGL((conv_row16_dgrad_kernel<2, 7, 3, 40, 128, 64, 8, true, true>), grid, block, 0, s, ra);
    else
      hipLaunchKernelGGL((conv_row16_dgrad_kernel<2, 7, 3, 40, 128, 64, 8, false, true>), grid, block, 0, s, ra);
    SRK_CHECK_HIP(hipGetLastError());
  }
  const int64_t G = std::min<int64_t>(groups, kCUs), nslab = KW * Ci * Co;
  float* slab = nullptr;
  float* bpart = nullptr;
  if ((rc = conv_scratch((size_t)(G * nslab), &slab))) return rc;
  if (db && (rc = conv_scratch((size_t)(G * Co), &bpart, g_csb))) return rc;
  Row16WgArgs wa{};
  wa.x16 = d16[0];
  wa.dy = dyp;
  wa.arg = arg;
  wa.slab = slab;
  wa.bpart = bpart;
  wa.rows = (int)rows;
  wa.groups = (int)groups;
  {
    ProfScope prof("conv_wgrad_lp", s, 2.0 * (double)(rows * W) * (double)(KW * Ci) * (double)Co);
    prof.detail("conv_row16_wgrad_kernel<unpool> %lldx%lldx%lld", (long long)(KW * Ci), (long long)Co, (long long)(rows * W));
    prof.bytes(2.0 * (double)(rows * W) * Ci + 5.0 / 4.0 * (double)(rows * W) * Co + 4.0 * (double)(G * nslab));
    if (prec == kPrecBF16)
      hipLaunchKernelGGL((conv_row16_wgrad_kernel<1, 7, 3, 40, 64, 128, 8>), dim3((unsigned)G), dim3(512), 0, s, wa);
    else
      hipLaunchKernelGGL((conv_row16_wgrad_kernel<2, 7, 3, 40, 64, 128, 8>), dim3((unsigned)G), dim3(512), 0, s, wa);
  }
  launch_splitk_sum(slab, (int)G, nslab, Co, nullptr, ws, s);
  if (bpart)
    hipLaunchKernelGGL(colsum_blocks_kernel, dim3((unsigned)((Co + 63) / 64)), dim3(64 * kCsWaves), 0, s, bpart, (int)G,
                       (int)Co, db);
  hipLaunchKernelGGL(weight_grad_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, ws, (int)Co,
                     (int)Ci, (int)KH, (int)KW, dw, 0);
  SRK_CHECK_HIP(hipGetLastError());
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
  return srk_conv2d_nhwc_fwd16(x, N, H, W, Ci, w, bias, Co, KH, KW, ph, pw, sh, sw, y, ws, nullptr, nullptr, stream);
}

int srk_conv2d_nhwc_fwd16(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                          const float* bias, int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh,
                          int64_t sw, float* y, float* ws, void* x16, int* x16_written, void* stream) {
  SRK_API_BEGIN
  const bool x16_ready = x16 && x16_written && *x16_written == 2;   // the producer's copy (srk_batchnorm_fwd16)
  if (x16_written) *x16_written = 0;
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
  // A full-width "valid" conv (model_fbanks_cnn.py:74, conv3 (1, 10) on width 10) is the plain GEMM
  //   Y[(n,h)][co] = X[(n,h)][(kw,ci)] . Wt[(kw,ci)][co] + bias
  // (x rows are already the GEMM rows: no gather, no split-K slabs of the implicit GEMM's tall 2-tile-wide grid)
  const bool full_width = KH == 1 && ph == 0 && pw == 0 && sh == 1 && KW == W && Wo == 1 && srk::g_opt_conv_fw_gemm;
  auto fw_gemm = [&](const unsigned short* a16, const unsigned short* b16, const char* cat) -> int {
    srk::GemmDesc g;
    g.M = N * H; g.N = Co; g.K = KW * Ci;
    g.A = x; g.lda = KW * Ci;
    g.B = ws; g.ldb = Co;
    g.C = y; g.ldc = Co;
    g.bias = bias; g.bias_mode = bias ? 1 : 0;
    g.A16 = a16; g.B16 = b16;
    srk::ProfScope prof(cat, s, 2.0 * (double)g.M * (double)g.N * (double)g.K);
    prof.detail("conv_fwd_as_gemm %lldx%lldx%lld", (long long)g.M, (long long)g.N, (long long)g.K);
    prof.bytes((a16 ? 2.0 : 4.0) * ((double)g.M * g.K + (double)g.K * g.N) + 4.0 * (double)g.M * g.N);
    return srk::gemm_f32(g, s);
  };
  if (srk::g_opt_conv_fwd_fp32 && srk::matmul_prec() != srk::kPrecF32) {
    // the faithful 16-bit mode: this forward on fp32 operands; a producer's 16-bit copy of x stays the
    // backward's (its weight gradient runs 16-bit)
    if (x16_ready && x16_written) *x16_written = 1;
    srk::PrecScope fp32(srk::kPrecF32);
    if (full_width) return fw_gemm(nullptr, nullptr, "conv_fwd");
    return srk::run_conv_gemm<srk::kFwd>(c, s, "conv_fwd");
  }
  const int prec = srk::matmul_prec();
  if (srk::s16_ok(prec, Ci, Co, {x, ws, x16})) {
    const float* src[2] = {x, ws};
    const int64_t n[2] = {N * H * W * Ci, nw};
    unsigned short* d16[2] = {static_cast<unsigned short*>(x16), nullptr};   // x16: the caller keeps x's copy
    const bool ready[2] = {x16_ready, false};
    if (int rc = srk::to16_all(prec, src, n, 2, d16, s, ready)) return rc;
    c.a16 = d16[0];
    c.b16 = d16[1];
    if (x16 && x16_written) *x16_written = 1;
  }
  if (full_width) return fw_gemm(c.a16, c.b16, prec == srk::kPrecF32 ? "conv_fwd" : "conv_fwd_lp");
  return srk::run_conv_gemm<srk::kFwd>(c, s, "conv_fwd");
  SRK_API_END
}

int srk_conv2d_nhwc_bwd(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w, int64_t Co,
                        int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw, const float* dy,
                        float* dx, float* dw, float* db, float* ws, void* stream) {
  return srk_conv2d_nhwc_bwd16(x, N, H, W, Ci, w, Co, KH, KW, ph, pw, sh, sw, dy, dx, dw, db, ws, nullptr, stream);
}

}  // extern "C"

namespace srk {
// the conv backward; dy_arg != null: dy is the (1, 4)-pooled gradient and the gathers unpool it
// (the caller guarantees fp32 sources, the fused bias sums and no full-width data gradient)
int conv_bwd(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w, int64_t Co, int64_t KH,
             int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw, const float* dy, const uint8_t* dy_arg,
             float* dx, float* dw, float* db, float* ws, const void* x16, void* stream,
             const unsigned short* dy16 = nullptr, int dw_accumulate = 0) {
  int64_t Ho, Wo;
  if (int rc = srk::check(N, H, W, Ci, Co, KH, KW, ph, pw, sh, sw, &Ho, &Wo)) return rc;
  SRK_REQUIRE(x && w && (dy || dy16) && dw && ws, SRK_ERR_INVALID, "conv bwd: null pointer");
  hipStream_t s = srk::as_stream(stream);
  const int64_t nw = Co * Ci * KH * KW;
  srk::ConvArgs c{};
  c.N = (int)N; c.H = (int)H; c.W = (int)W; c.Ci = (int)Ci; c.Ho = (int)Ho; c.Wo = (int)Wo; c.Co = (int)Co;
  c.KH = (int)KH; c.KW = (int)KW; c.ph = (int)ph; c.pw = (int)pw; c.sh = (int)sh; c.sw = (int)sw;
  c.x = x; c.dy = dy;
  c.dy_arg = dy_arg;
  int rc;
  const bool full_width = KH == 1 && ph == 0 && sh == 1 && pw == 0 && KW == W && Wo == 1;
  SRK_REQUIRE(!dy_arg || (!full_width && (!db || srk::g_opt_conv_fused_db)), SRK_ERR_INTERNAL,
              "conv bwd: pooled dY needs the implicit data gradient and the fused bias sums");
  // dy16 without dy: the caller's 16-bit dY only (the pooled backward): the implicit 16-bit-source GEMMs, no
  // bias sums here; dy16 beside dy: a ready copy, used where the 16-bit path would round dy
  SRK_REQUIRE(!dy16 || dy || (!dy_arg && !full_width && !db && srk::s16_ok(srk::matmul_prec(), Ci, Co, {x, ws, x16, dy16})),
              SRK_ERR_INTERNAL, "conv bwd: a 16-bit dY needs the 16-bit-source implicit GEMMs");
  const bool dgrad_implicit = dx && !full_width;
  if (dgrad_implicit)
    hipLaunchKernelGGL(srk::weight_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, w, (int)Co,
                       (int)Ci, (int)KH, (int)KW, 1, ws);
  // 16-bit sources: x and dY serve both GEMMs, Wd the data gradient (one scratch allocation)
  unsigned short* d16[3] = {nullptr, nullptr, nullptr};   // x, dY, Wd
  const int prec = srk::matmul_prec();
  bool db_done = false;
  if (!dy_arg && srk::s16_ok(prec, Ci, Co, {x, dy, ws, x16, dy16})) {
    const float* src[3] = {x, dy, ws};
    const int64_t n[3] = {N * H * W * Ci, N * Ho * Wo * Co, nw};
    // the bias gradient with dY's conversion (or alone when the producer's copy is ready): one read of dY
    const bool cs = db && dy && srk::colsum8_ok(Co);
    bool ready[3] = {x16 != nullptr, dy16 != nullptr || cs, false};   // x16: the forward's copy of x
    d16[0] = const_cast<unsigned short*>(static_cast<const unsigned short*>(x16));
    d16[1] = const_cast<unsigned short*>(dy16);
    if (cs && !dy16) {
      float* d = nullptr;
      if ((rc = srk::conv_scratch((size_t)(n[1] + 1) / 2, &d, srk::g_csy))) return rc;
      d16[1] = reinterpret_cast<unsigned short*>(d);
    }
    if ((rc = srk::to16_all(prec, src, n, dgrad_implicit ? 3 : 2, d16, s, ready))) return rc;
    if (cs) {
      if ((rc = srk::colsum8(dy16 ? 0 : 1, prec, dy, nullptr, N * Ho * Wo, (int)Co, 1, d16[1], db, s))) return rc;
      db_done = true;
    }
  }
  if (dx && full_width) {
    // A full-width "valid" conv (model_fbanks_cnn.py:74, conv3 1x10 on width 10): every input
    // column meets exactly one tap, so the data gradient is the plain GEMM
    //   dX[(n,h)][(kw,ci)] = dY[(n,h)][co] * Wt[(kw,ci)][co]^T
    // instead of an implicit GEMM whose k range is 90 % structurally-zero taps.
    hipLaunchKernelGGL(srk::weight_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, w, (int)Co,
                       (int)Ci, (int)KH, (int)KW, 0, ws);
    srk::GemmDesc g;
    g.M = N * H; g.N = KW * Ci; g.K = Co;
    g.A = dy; g.lda = Co;
    g.B = ws; g.ldb = Co; g.tb = true;
    g.C = dx; g.ldc = KW * Ci;
    srk::ProfScope prof(srk::matmul_prec() == srk::kPrecF32 ? "conv_dgrad" : "conv_dgrad_lp", s,
                        2.0 * (double)g.M * (double)g.N * (double)g.K);
    prof.detail("conv_dgrad_as_gemm %lldx%lldx%lld", (long long)g.M, (long long)g.N, (long long)g.K);
    prof.bytes(4.0 * ((double)g.M * g.K + (double)g.K * g.N + (double)g.M * g.N));
    if ((rc = srk::gemm_f32(g, s))) return rc;
  } else if (dgrad_implicit && d16[0] && srk::g_opt_conv_row16_dgrad && KH == 1 && KW == 7 && ph == 0 && pw == 3 &&
             sh == 1 && sw == 1 && W == 40 && Ci == 64 && Co == 128 && (N * H) < (1LL << 30) / (W * Co)) {
    // fbanks_cnn conv2's data gradient: the row-staged kernel (conv_row16_dgrad_kernel)
    srk::RowDgArgs ra{};
    ra.dy16 = d16[1];
    ra.wd16 = d16[2];
    ra.dx = dx;
    ra.rows = (int)(N * H);
    ra.groups = (int)((N * H + 7) / 8);
    srk::ProfScope prof("conv_dgrad_lp", s, 2.0 * (double)(N * H * W) * (double)Ci * (double)(KW * Co));
    prof.detail("conv_row16_dgrad_kernel %lldx%lldx%lld", (long long)(N * H * W), (long long)Ci, (long long)(KW * Co));
    prof.bytes(2.0 * (double)(N * H * W) * Co + 2.0 * (double)(KW * Co) * Ci + 4.0 * (double)(N * H * W) * Ci);
    const dim3 grid((unsigned)std::min<int64_t>(ra.groups, srk::kCUs)), block(256);
    const bool bal = srk::g_opt_conv_row16_dgrad == 2;
    if (prec == srk::kPrecBF16 && bal)
      hipLaunchKernelGGL((srk::conv_row16_dgrad_kernel<1, 7, 3, 40, 128, 64, 8, true>), grid, block, 0, s, ra);
    else if (prec == srk::kPrecBF16)
      hipLaunchKernelGGL((srk::conv_row16_dgrad_kernel<1, 7, 3, 40, 128, 64, 8>), grid, block, 0, s, ra);
    else if (bal)
      hipLaunchKernelGGL((srk::conv_row16_dgrad_kernel<2, 7, 3, 40, 128, 64, 8, true>), grid, block, 0, s, ra);
    else
      hipLaunchKernelGGL((srk::conv_row16_dgrad_kernel<2, 7, 3, 40, 128, 64, 8>), grid, block, 0, s, ra);
  } else if (dgrad_implicit && !d16[0] && prec == srk::kPrecF32 && srk::g_opt_conv_row32 && KH == 1 && KW == 7 &&
             ph == 0 && pw == 3 && sh == 1 && sw == 1 && W == 40 && Ci == 64 && Co == 128 && dy && dy_arg &&
             (N * H) < (1LL << 29) / (W * Co)) {
    // fbanks_cnn conv2's data gradient on fp32 operands (the pooled backward: the pooled gradient + argmax): the
    // row-staged kernel (conv_row32_dgrad_kernel; its dense-dY form spills at one wave per SIMD, not used)
    srk::Row32DgArgs ra{};
    ra.dy = dy;
    ra.arg = dy_arg;
    ra.wd = ws;
    ra.dx = dx;
    ra.rows = (int)(N * H);
    ra.groups = (int)((N * H + 7) / 8);
    srk::ProfScope prof("conv_dgrad", s, 2.0 * (double)(N * H * W) * (double)Ci * (double)(KW * Co));
    prof.detail("conv_row32_dgrad_kernel<unpool> %lldx%lldx%lld", (long long)(N * H * W), (long long)Ci,
                (long long)(KW * Co));
    prof.bytes(5.0 / 4.0 * (double)(N * H * W) * Co + 4.0 * (double)(KW * Co) * Ci + 4.0 * (double)(N * H * W) * Ci);
    const dim3 grid((unsigned)std::min<int64_t>(ra.groups, srk::kCUs)), block(256);
    hipLaunchKernelGGL((srk::conv_row32_dgrad_kernel<7, 3, 40, 128, 64, 8, true>), grid, block, 0, s, ra);
  } else if (dgrad_implicit) {
    srk::ConvArgs d = c;
    d.wmat = ws; d.out = dx;
    d.M = N * H * W; d.Nn = Ci; d.K = KH * KW * Co;
    if (d16[0]) {
      d.a16 = d16[1];
      d.b16 = d16[2];
    }
    if ((rc = srk::run_conv_gemm<srk::kDgrad>(d, s, "conv_dgrad"))) return rc;
  }
  if (!d16[0] && prec == srk::kPrecF32 && srk::g_opt_conv_row32 && KH == 1 && KW == 7 && ph == 0 && pw == 3 &&
      sh == 1 && sw == 1 && W == 40 && Ci == 64 && Co == 128 && dy && dy_arg && (N * H) < (1LL << 31) / (W * Ci * 4)) {
    // fbanks_cnn conv2's weight gradient on fp32 operands from the pooled gradient + argmax: the row-staged kernel
    // (conv_row32_wgrad_kernel), one slab per workgroup, reduced in order; the bias gradient from the same pass
    const int64_t rows = N * H, groups = (rows + 7) / 8, G = std::min<int64_t>(groups, srk::kCUs);
    const int64_t nslab = KW * Ci * Co;
    float* slab = nullptr;
    float* bpart = nullptr;
    if ((rc = srk::conv_scratch((size_t)(G * nslab), &slab))) return rc;
    if (db && (rc = srk::conv_scratch((size_t)(G * Co), &bpart, srk::g_csb))) return rc;
    srk::Row32WgArgs ra{};
    ra.x = x;
    ra.dy = dy;
    ra.arg = dy_arg;
    ra.slab = slab;
    ra.bpart = bpart;
    ra.rows = (int)rows;
    ra.groups = (int)groups;
    {
      srk::ProfScope prof("conv_wgrad", s, 2.0 * (double)(N * H * W) * (double)(KW * Ci) * (double)Co);
      prof.detail("conv_row32_wgrad_kernel<unpool> %lldx%lldx%lld", (long long)(KW * Ci), (long long)Co,
                  (long long)(N * H * W));
      prof.bytes(4.0 * (double)(N * H * W) * Ci + 5.0 / 4.0 * (double)(N * H * W) * Co + 4.0 * (double)(G * nslab));
      hipLaunchKernelGGL((srk::conv_row32_wgrad_kernel<7, 3, 40, 64, 128, 8>), dim3((unsigned)G), dim3(512), 0, s, ra);
    }
    srk::launch_splitk_sum(slab, (int)G, nslab, Co, nullptr, ws, s);
    if (db)
      hipLaunchKernelGGL(srk::colsum_blocks_kernel, dim3((unsigned)((Co + 63) / 64)), dim3(64 * srk::kCsWaves), 0, s,
                         bpart, (int)G, (int)Co, db);
    hipLaunchKernelGGL(srk::weight_grad_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, ws,
                       (int)Co, (int)Ci, (int)KH, (int)KW, dw, dw_accumulate);
  } else {
    srk::ConvArgs g = c;
    g.out = ws;   // dWt [(kh,kw,ci)][co], then re-laid out into dw
    g.M = KH * KW * Ci; g.Nn = Co; g.K = N * Ho * Wo;
    if (d16[0]) {
      g.a16 = d16[0];
      g.b16 = d16[1];
    }
    // the bias gradient = column sums of dY, fused into the weight-gradient kernel (fp32-source
    // paths: the sums of the unrounded values); the 16-bit-source path keeps the column-sum kernel
    g.db = srk::g_opt_conv_fused_db ? db : nullptr;
    if ((rc = srk::run_conv_gemm<srk::kWgrad>(g, s, "conv_wgrad"))) return rc;
    hipLaunchKernelGGL(srk::weight_grad_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, ws,
                       (int)Co, (int)Ci, (int)KH, (int)KW, dw, dw_accumulate);
    if (db && !db_done && (!g.db || g.a16) && (rc = srk::colsum_f32(dy, N * Ho * Wo, Co, Co, db, 0.f, s))) return rc;
  }
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}
}  // namespace srk

extern "C" {

int srk_conv2d_nhwc_bwd16(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w, int64_t Co,
                          int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw, const float* dy,
                          float* dx, float* dw, float* db, float* ws, const void* x16, void* stream) {
  SRK_API_BEGIN
  return srk::conv_bwd(x, N, H, W, Ci, w, Co, KH, KW, ph, pw, sh, sw, dy, nullptr, dx, dw, db, ws, x16, stream);
  SRK_API_END
}

int srk_conv2d_nhwc_bwd16_dy16(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                               int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw,
                               const float* dy, const void* dy16, float* dx, float* dw, float* db, float* ws,
                               const void* x16, void* stream) {
  return srk_conv2d_nhwc_bwd16_acc(x, N, H, W, Ci, w, Co, KH, KW, ph, pw, sh, sw, dy, dy16, dx, dw, db, ws, x16, 0,
                                   stream);
}

int srk_conv2d_nhwc_bwd16_acc(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                              int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t sh, int64_t sw,
                              const float* dy, const void* dy16, float* dx, float* dw, float* db, float* ws,
                              const void* x16, int dw_accumulate, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(dy, SRK_ERR_INVALID, "conv bwd: null pointer");
  return srk::conv_bwd(x, N, H, W, Ci, w, Co, KH, KW, ph, pw, sh, sw, dy, nullptr, dx, dw, db, ws, x16, stream,
                       static_cast<const unsigned short*>(dy16), dw_accumulate ? 1 : 0);
  SRK_API_END
}

int srk_conv2d_nhwc_fwd_pool(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w,
                             const float* bias, int64_t Co, int64_t KH, int64_t KW, int64_t ph, int64_t pw,
                             int64_t pool_w, float* y, uint8_t* argmax, float* ws, void* x16, int* x16_written,
                             void* stream) {
  SRK_API_BEGIN
  const bool x16_ready = x16 && x16_written && *x16_written == 2;   // the producer's copy (srk_conv1_pool_fwd16)
  if (x16_written) *x16_written = 0;
  // the faithful 16-bit mode ("conv_fwd_fp32"): this forward on fp32 operands, a producer's copy kept for the
  // backward
  const bool fwd32 = srk::g_opt_conv_fwd_fp32 && srk::matmul_prec() != srk::kPrecF32;
  if (fwd32 && x16_ready) *x16_written = 1;
  srk::PrecScope fp32(fwd32 ? srk::kPrecF32 : -1);
  if (fwd32) x16 = nullptr;
  int64_t Ho, Wo;
  if (int rc = srk::check(N, H, W, Ci, Co, KH, KW, ph, pw, 1, 1, &Ho, &Wo)) return rc;
  SRK_REQUIRE(x && w && y && argmax && ws, SRK_ERR_INVALID, "conv fwd_pool: null pointer");
  SRK_REQUIRE(pool_w == 4 && Wo % pool_w == 0, SRK_ERR_INVALID,
              "conv fwd_pool: the fused pooling needs a (1, 4) window that divides the output width");
  hipStream_t s = srk::as_stream(stream);
  const int64_t nw = Co * Ci * KH * KW;
  hipLaunchKernelGGL(srk::weight_layout_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, w, (int)Co,
                     (int)Ci, (int)KH, (int)KW, 0, ws);
  srk::ConvArgs c{};
  c.N = (int)N; c.H = (int)H; c.W = (int)W; c.Ci = (int)Ci; c.Ho = (int)Ho; c.Wo = (int)Wo; c.Co = (int)Co;
  c.KH = (int)KH; c.KW = (int)KW; c.ph = (int)ph; c.pw = (int)pw; c.sh = 1; c.sw = 1;
  c.x = x; c.wmat = ws; c.out = y; c.bias = bias;
  c.M = N * Ho * Wo; c.Nn = Co; c.K = KH * KW * Ci;
  c.pool_w = (int)pool_w;
  c.pool_arg = argmax;
  const int prec = srk::matmul_prec();
  if (srk::s16_ok(prec, Ci, Co, {x, ws, x16})) {
    const float* src[2] = {x, ws};
    const int64_t n[2] = {N * H * W * Ci, nw};
    unsigned short* d16[2] = {static_cast<unsigned short*>(x16), nullptr};
    const bool ready[2] = {x16_ready, false};
    if (int rc = srk::to16_all(prec, src, n, 2, d16, s, ready)) return rc;
    c.a16 = d16[0];
    c.b16 = d16[1];
    if (x16 && x16_written) *x16_written = 1;
    // fbanks_cnn conv2 + maxpool2: the row-staged kernel (weights resident in LDS, 8 image rows per tile)
    if (srk::g_opt_conv_row16 && KH == 1 && KW == 7 && ph == 0 && pw == 3 && W == 40 && Ci == 64 && Co == 128 &&
        pool_w == 4 && (N * H) < (1LL << 30) / (W * Ci)) {
      srk::RowArgs ra{};
      ra.x16 = c.a16;
      ra.w16 = c.b16;
      ra.bias = bias;
      ra.y = y;
      ra.arg = argmax;
      ra.rows = (int)(N * H);
      ra.groups = (int)((N * H + 7) / 8);
      srk::ProfScope prof("conv_fwd_lp", s, 2.0 * (double)c.M * (double)c.Nn * (double)c.K);
      prof.detail("conv_row16_pool_kernel %lldx%lldx%lld", (long long)c.M, (long long)c.Nn, (long long)c.K);
      prof.bytes(srk::conv_bytes(c, srk::kFwd, 2));
      const bool w4 = srk::g_opt_conv_row16 == 2;
      const dim3 grid((unsigned)std::min<int64_t>(ra.groups, srk::kCUs)), block(w4 ? 256 : 512);
      if (prec == srk::kPrecBF16) {
        if (w4) hipLaunchKernelGGL((srk::conv_row16_pool_kernel<1, 7, 3, 40, 64, 128, 8, 4>), grid, block, 0, s, ra);
        else hipLaunchKernelGGL((srk::conv_row16_pool_kernel<1, 7, 3, 40, 64, 128, 8, 8>), grid, block, 0, s, ra);
      } else {
        if (w4) hipLaunchKernelGGL((srk::conv_row16_pool_kernel<2, 7, 3, 40, 64, 128, 8, 4>), grid, block, 0, s, ra);
        else hipLaunchKernelGGL((srk::conv_row16_pool_kernel<2, 7, 3, 40, 64, 128, 8, 8>), grid, block, 0, s, ra);
      }
      SRK_CHECK_HIP(hipGetLastError());
      return SRK_OK;
    }
  }
  // fbanks_cnn conv2 + maxpool2 on fp32 operands: the row-staged kernel (weights streamed per tap), unless the
  // ring pooled forward is asked for (conv_ring bit 7)
  if (!c.a16 && srk::matmul_prec() == srk::kPrecF32 && srk::g_opt_conv_row32 && !(srk::g_opt_conv_ring & 0x80) &&
      KH == 1 && KW == 7 && ph == 0 &&
      pw == 3 && W == 40 && Ci == 64 && Co == 128 && pool_w == 4 && (N * H) < (1LL << 31) / (W * Ci * 4)) {
    srk::Row32Args ra{};
    ra.x = x;
    ra.wt = ws;
    ra.bias = bias;
    ra.y = y;
    ra.arg = argmax;
    ra.rows = (int)(N * H);
    ra.groups = (int)((N * H + 7) / 8);
    srk::ProfScope prof("conv_fwd", s, 2.0 * (double)c.M * (double)c.Nn * (double)c.K);
    prof.detail("conv_row32_pool_kernel %lldx%lldx%lld", (long long)c.M, (long long)c.Nn, (long long)c.K);
    prof.bytes(srk::conv_bytes(c, srk::kFwd, 4));
    hipLaunchKernelGGL((srk::conv_row32_pool_kernel<7, 3, 40, 64, 128, 8>),
                       dim3((unsigned)std::min<int64_t>(ra.groups, srk::kCUs)), dim3(512), 0, s, ra);
    SRK_CHECK_HIP(hipGetLastError());
    return SRK_OK;
  }
  return srk::run_conv_gemm<srk::kFwd>(c, s, "conv_fwd");
  SRK_API_END
}

int srk_conv2d_nhwc_bwd_pool(const float* x, int64_t N, int64_t H, int64_t W, int64_t Ci, const float* w, int64_t Co,
                             int64_t KH, int64_t KW, int64_t ph, int64_t pw, int64_t pool_w, const float* dy_pooled,
                             const uint8_t* argmax, float* dx, float* dw, float* db, float* ws, const void* x16,
                             void* stream) {
  SRK_API_BEGIN
  int64_t Ho, Wo;
  if (int rc = srk::check(N, H, W, Ci, Co, KH, KW, ph, pw, 1, 1, &Ho, &Wo)) return rc;
  SRK_REQUIRE(dy_pooled && argmax, SRK_ERR_INVALID, "conv bwd_pool: null pointer");
  SRK_REQUIRE(pool_w == 4 && Wo % pool_w == 0 && Co % 4 == 0 && (uintptr_t)dy_pooled % 16 == 0 &&
                  (uintptr_t)argmax % 4 == 0,
              SRK_ERR_INVALID, "conv bwd_pool: (1, 4) window dividing the output width, Co % 4, aligned buffers");
  hipStream_t s = srk::as_stream(stream);
  // fp32 sources (fp32, or a 16-bit mode whose channel counts rule out the 16-bit copies): the
  // data- and weight-gradient gathers read the pooled gradient through the argmax themselves
  const bool full_width = KH == 1 && ph == 0 && pw == 0 && KW == W && Wo == 1;
  if (srk::g_opt_conv_unpool_gather && !full_width && (!db || srk::g_opt_conv_fused_db) &&
      !srk::s16_ok(srk::matmul_prec(), Ci, Co, {x, w, x16}))
    return srk::conv_bwd(x, N, H, W, Ci, w, Co, KH, KW, ph, pw, 1, 1, dy_pooled, argmax, dx, dw, db, ws, x16, stream);
  const int64_t rows = N * Ho * Wo / pool_w;
  const int prec = srk::matmul_prec();
  if (srk::g_opt_conv_unpool16 && !full_width && Co % 8 == 0 && srk::s16_ok(prec, Ci, Co, {x, w, x16, ws})) {
    // fbanks_cnn conv2 (Conv2d(64, 128, (1, 7), padding (0, 3)) over W = 40 + MaxPool2d((1, 4))): both gradients from
    // the pooled gradient on the row-staged kernels, no dense dY
    if (srk::g_opt_conv_row16 && srk::g_opt_conv_row16_dgrad && KH == 1 && KW == 7 && ph == 0 && pw == 3 && W == 40 &&
        Ci == 64 && Co == 128 && dw && (N * H) < (1LL << 30) / (W * Co))
      return srk::conv2_bwd16_pooled(x, N, H, w, dy_pooled, argmax, dx, dw, db, ws, x16, s);
    // 16-bit-source modes: the dense dY straight as its 16-bit copy, the bias gradient from the pooled
    // gradient (each pooled value sits once in the dense dY, the rest are zeros), then the backward
    float* d = nullptr;
    if (int rc = srk::conv_scratch((size_t)(N * Ho * Wo * Co + 1) / 2, &d, srk::g_csd)) return rc;
    unsigned short* dy16 = reinterpret_cast<unsigned short*>(d);
    if (db && srk::colsum8_ok(Co)) {   // the dense 16-bit dY and the bias gradient in one pass over the pooled dY
      if (int rc = srk::colsum8(2, prec, dy_pooled, argmax, rows, (int)Co, (int)pool_w, dy16, db, s)) return rc;
    } else {
      srk::ProfScope prof("conv_unpool16", s, (double)rows * Co * (4.0 + 1.0 + 2.0 * pool_w));
      const dim3 grid((unsigned)((rows * (Co / 8) + 255) / 256));
      if (prec == srk::kPrecBF16)
        hipLaunchKernelGGL(srk::unpool16_kernel<1>, grid, dim3(256), 0, s, dy_pooled, argmax, rows, (int)Co, (int)pool_w, dy16);
      else
        hipLaunchKernelGGL(srk::unpool16_kernel<2>, grid, dim3(256), 0, s, dy_pooled, argmax, rows, (int)Co, (int)pool_w, dy16);
      SRK_CHECK_HIP(hipGetLastError());
      if (db)
        if (int rc = srk::colsum_f32(dy_pooled, rows, Co, Co, db, 0.f, s)) return rc;
    }
    return srk::conv_bwd(x, N, H, W, Ci, w, Co, KH, KW, ph, pw, 1, 1, nullptr, nullptr, dx, dw, nullptr, ws, x16, stream,
                         dy16);
  }
  float* dy = nullptr;   // else: the dense gradient in library scratch, then the plain backward
  if (int rc = srk::conv_scratch((size_t)(N * Ho * Wo * Co), &dy, srk::g_csd)) return rc;
  hipLaunchKernelGGL(srk::unpool_kernel, dim3((unsigned)((rows * (Co / 4) + 255) / 256)), dim3(256), 0, s, dy_pooled,
                     argmax, rows, (int)Co, (int)pool_w, dy);
  SRK_CHECK_HIP(hipGetLastError());
  return srk::conv_bwd(x, N, H, W, Ci, w, Co, KH, KW, ph, pw, 1, 1, dy, nullptr, dx, dw, db, ws, x16, stream);
  SRK_API_END
}

int srk_maxpool_nhwc_fwd(const float* x, int64_t N, int64_t H, int64_t W, int64_t C, int64_t kh, int64_t kw,
                         float* y, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(x && y && N > 0 && C > 0 && kh > 0 && kw > 0 && H >= kh && W >= kw, SRK_ERR_INVALID, "maxpool: bad args");
  SRK_REQUIRE(C % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)y % 16 == 0, SRK_ERR_INVALID,
              "maxpool: channels must be a multiple of 4 and tensors 16-B aligned");
  const int64_t n = N * (H / kh) * (W / kw) * C;
  srk::ProfScope prof("maxpool_fwd", srk::as_stream(stream), 4.0 * (N * H * W * C + n));
  hipLaunchKernelGGL(srk::maxpool_fwd_kernel, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, srk::as_stream(stream), x,
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
  SRK_REQUIRE(C % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)dy % 16 == 0 && (uintptr_t)dx % 16 == 0,
              SRK_ERR_INVALID, "maxpool bwd: channels must be a multiple of 4 and tensors 16-B aligned");
  hipStream_t s = srk::as_stream(stream);
  const int64_t Ho = H / kh, Wo = W / kw;
  const int64_t n = N * Ho * Wo * C;
  if (Ho * kh != H || Wo * kw != W) {   // rows/cols dropped by floor mode get zero gradient
    const int64_t all = N * H * W * C;
    hipLaunchKernelGGL(srk::zero_kernel, dim3((unsigned)((all + 255) / 256)), dim3(256), 0, s, dx, all);
  }
  srk::ProfScope prof("maxpool_bwd", s, 4.0 * (2 * N * H * W * C + n));
  hipLaunchKernelGGL(srk::maxpool_bwd_kernel, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, s, x, dy, (int)N, (int)H,
                     (int)W, (int)C, (int)kh, (int)kw, dx);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"

namespace srk {
int release_conv_scratch() {
  std::lock_guard<std::mutex> lk(g_cs_mu);
  SRK_CHECK_HIP(hipDeviceSynchronize());
  for (ConvScratch* pool : {g_cs, g_cs16, g_csb, g_csd, g_csy})
    for (int d = 0; d < 64; ++d) {
      if (pool[d].p) SRK_CHECK_HIP(hipFree(pool[d].p));
      pool[d].p = nullptr;
      pool[d].floats = 0;
    }
  g_scratch_gen.fetch_add(1);
  return SRK_OK;
}
}  // namespace srk
