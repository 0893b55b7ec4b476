// fp32 GEMM on the gfx950 matrix cores: v_mfma_f32_32x32x2_f32 (exact fp32 fma chain — the same
// numerics class as the reference's fp32 cuBLAS/CPU GEMMs; SURVEY.md Appendix A "logits 1e-4").
//
// Tile: BM x BN x BK per 256-thread workgroup (2 x 2 waves), each wave owns (BM/2) x (BN/2) as
// 32x32 MFMA tiles (64 FLOP/clk/SIMD, one f32 operand per lane per 2-deep k step).  Operands are
// staged k-major in LDS ([k][m], [k][n]) through registers, double-buffered: tile k+1 is fetched
// while tile k is multiplied.  Rows written by scalar transposing stores get a +1 float pad
// (conflict-free ds_write_b32), rows written by float4 stores stay unpadded.
//
// Tall-K shapes that would leave the chip under-filled (the weight-gradient GEMMs, K = B*T) are
// split over K: each split writes an fp32 partial slab, a second kernel sums the slabs in a fixed
// order (deterministic) and applies alpha / beta / bias.  Optionally the kernel also produces
// rowsum[m] = sum_k op(A)[m, k] from the A tiles it already stages (the bias gradient of a
// dW = dY^T X GEMM, fused: no separate pass over dY).
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "gemm.h"
#include "mfma_tile.h"

namespace srk {
namespace {

using namespace tile;

struct KernelArgs {
  GemmDesc d;
  int tiles_m, tiles_n;
  int tiles;             // tiles_m * tiles_n (one split's output grid)
  int nblk;              // tiles * splits = gridDim.x
  int group_m;           // tile rows per swizzle group (L2 reuse of B panels)
  int remap;             // XCD-aware block remap on/off (A/B measurement only)
  int64_t kchunk;        // K range per split (a multiple of BK)
  float* partial;        // [splits][M][N] when split
  float* rs_partial;     // [splits][M] when split and rowsum requested
  // stream-K (gemm_p32_kernel, option gemm_streamk): sk_wgs workgroups split the tiles x sk_ki K-tiles
  // into equal contiguous runs; a tile covered by several runs is written as partial sums into
  // sk_slab[order of the run within the tile][M][N] and summed by sk_fixup_kernel
  int sk_wgs;
  int sk_ki;
  float* sk_slab;
};

// tile index t (one split's grid, grouped order) -> (tile row, tile column); see map_tile
__device__ __forceinline__ void tile_of(int t, int tiles_m, int tiles_n, int group_m, int& tm, int& tn) {
  const int gsz_full = group_m * tiles_n;
  const int grp = t / gsz_full, first_m = grp * group_m;
  const int gm = tiles_m - first_m < group_m ? tiles_m - first_m : group_m;
  const int tin = t - grp * gsz_full;
  tm = first_m + tin % gm;
  tn = tin / gm;
}
// stream-K: run w covers K-tile iterations [w total / W, (w + 1) total / W); the run holding iteration it
__device__ __forceinline__ int64_t sk_begin(int64_t w, int64_t total, int64_t W) { return w * total / W; }
__device__ __forceinline__ int sk_owner(int64_t it, int64_t total, int64_t W) { return (int)(((it + 1) * W - 1) / total); }

// Epilogue shared by the tile kernels.  32x32 accumulator: col = lane & 31,
// row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5).  Split-K launches write the raw fp32 slab.
template <int TM, int TN>
__device__ __forceinline__ void store_acc(const KernelArgs& ka, const f32x16 (&acc)[TM][TN], int split, int64_t m0,
                                          int64_t n0, int wm0, int wn0, int lane, int64_t z) {
  const GemmDesc& d = ka.d;
  const int lh = lane >> 5, lc = lane & 31;
  const bool split_mode = ka.partial != nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t col = n0 + wn0 + j * 32 + lc;
      if (col >= d.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row >= d.M) continue;
        if (split_mode) {
          ka.partial[((int64_t)split * d.M + row) * d.N + col] = acc[i][j][r];
          continue;
        }
        float* C = d.C + z * d.sC;
        float v = d.alpha * acc[i][j][r];
        if (d.bias_mode == 1) v += d.bias[col];
        else if (d.bias_mode == 2) v += d.bias[row];
        float* c = C + row * d.ldc + col;
        if (d.beta != 0.f) v += d.beta * *c;
        *c = v;
      }
    }
  }
}

// NW = waves per workgroup: 4 (2 x 2, each wave (BM/2) x (BN/2)) or 8 (2 x 4, each (BM/2) x (BN/4):
// twice the waves per SIMD to cover the k-tile barrier / staging phases).
#ifndef SRK_GEMM_PREFETCH
#define SRK_GEMM_PREFETCH 1
#endif
constexpr int kGemmPrefetch = SRK_GEMM_PREFETCH;   // k-tiles staged ahead in registers (1 or 2)
static_assert(kGemmPrefetch == 1 || kGemmPrefetch == 2, "SRK_GEMM_PREFETCH must be 1 or 2");

// 16 zero bytes: the LDS-DMA source of k >= ke quads (the k tail must multiply as exact zeros)
__device__ __attribute__((aligned(16))) float g_zero4[4];

// GL: operands staged by global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip, lane-linear
// ImgL images) instead of global_load -> registers -> ds_write (needs the VEC conditions).
template <bool TA, bool TB, int BM, int BN, int BK, bool VEC, int NW, bool GL = false>
__global__ __launch_bounds__(NW * 64) void gemm_f32_kernel(KernelArgs ka) {
  constexpr int NT = NW * 64;
  // wave grid: 2 x NW/2, except the 256-row tile (8 waves as 4 x 2: every wave 64 x 64)
  constexpr int WM = (BM == 256) ? 4 : 2, WN = NW / WM;
  constexpr bool AKC = !TA, BKC = TB;         // k-contiguous in HBM?
  static_assert(!GL || VEC, "LDS-DMA staging needs the 16-B vector conditions");
  using IA = std::conditional_t<GL, ImgL<AKC, BM, BK>, Img<AKC, BM, BK>>;
  using IB = std::conditional_t<GL, ImgL<BKC, BN, BK>, Img<BKC, BN, BK>>;
  constexpr int VA = BM * BK / 4 / NT, VB = BN * BK / 4 / NT;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;   // 32x32 tiles per wave per dim
  static_assert(VA >= 1 && VB >= 1 && TM >= 1 && TN >= 1 && BK % 8 == 0, "bad tile");
  __shared__ __attribute__((aligned(16))) float smem[2 * (IA::FLOATS + IB::FLOATS)];
  const GemmDesc& d = ka.d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  int split, tm, tn;
  map_tile(ka.nblk, ka.tiles, ka.tiles_m, ka.tiles_n, ka.group_m, ka.remap != 0, split, tm, tn);

  const int64_t z = blockIdx.z;
  const float* __restrict__ A = d.A + z * d.sA;
  const float* __restrict__ B = d.B + z * d.sB;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kb0 = split * ka.kchunk;
  const int64_t ke = (kb0 + ka.kchunk < d.K) ? kb0 + ka.kchunk : d.K;
  const int wm0 = (wave / WN) * (BM / WM), wn0 = (wave % WN) * (BN / WN);
  const bool do_rs = d.rowsum != nullptr && tn == 0;

  // Global -> register staging.  Every index is CLAMPED into range instead of predicated, so no
  // load is exec-masked and nothing waits on a load before this tile's MFMAs: rows >= M (A) or
  // >= N (B) only feed output rows / columns that are never stored, and k >= ke (the k tail of the
  // last tile of a split) is zeroed in the A image at LDS-store time (after the MFMAs), which
  // makes those products exactly 0 (clamped B values are copies of finite inputs).
  // PF register sets: tile t is staged in set t % PF, so with PF = 2 the loads of tile k + 2 are in
  // flight while tile k is multiplied and tile k + 1 waits in registers for its LDS store.
  constexpr int PF = kGemmPrefetch;
  v4f ra[PF][VA], rb[PF][VB];
  // KC: 4 consecutive k of row r (stored [row][ld]);  !KC: rows r..r+3 at k (stored [k][ld])
  auto ld_op = [&](const float* __restrict__ P, int64_t ld, bool kc, int64_t rows, int64_t r, int64_t k) -> v4f {
    if (kc) {
      const float* q = P + (r < rows ? r : rows - 1) * ld;
      if (VEC) return ld4(q + (k < ke - 3 ? k : ke - 4));   // VEC: ke % 4 == 0 (see gemm_f32)
      v4f v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = q[k + e < ke ? k + e : ke - 1];
      return v;
    }
    const float* q = P + (k < ke ? k : ke - 1) * ld;
    if (VEC) return ld4(q + (r < rows ? r : rows - 4));     // VEC: rows % 4 == 0
    v4f v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = q[r + e < rows ? r + e : rows - 1];
    return v;
  };
  auto load_tile = [&](int st, int64_t k0) {
#pragma unroll
    for (int i = 0; i < VA; ++i) {
      const int vi = tid + i * NT;
      if (AKC) ra[st][i] = ld_op(A, d.lda, true, d.M, m0 + vi / (BK / 4), k0 + (vi % (BK / 4)) * 4);
      else     ra[st][i] = ld_op(A, d.lda, false, d.M, m0 + (vi % (BM / 4)) * 4, k0 + vi / (BM / 4));
    }
#pragma unroll
    for (int i = 0; i < VB; ++i) {
      const int vi = tid + i * NT;
      if (BKC) rb[st][i] = ld_op(B, d.ldb, true, d.N, n0 + vi / (BK / 4), k0 + (vi % (BK / 4)) * 4);
      else     rb[st][i] = ld_op(B, d.ldb, false, d.N, n0 + (vi % (BN / 4)) * 4, k0 + vi / (BN / 4));
    }
  };
  auto store_tile = [&](int st, int buf, int64_t k0) {
    float* As = smem + buf * (IA::FLOATS + IB::FLOATS);
    float* Bs = As + IA::FLOATS;
    const bool tail = k0 + BK > ke;
#pragma unroll
    for (int i = 0; i < VA; ++i) {
      const int vi = tid + i * NT;
      v4f v = ra[st][i];
      if (AKC) {
        const int kq = (vi % (BK / 4)) * 4;
        if (tail) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = k0 + kq + e < ke ? v[e] : 0.f;
        }
        st4(As + (vi / (BK / 4)) * IA::P + kq, v);
      } else {
        const int kr = vi / (BM / 4);
        if (tail && k0 + kr >= ke) v = v4f{0.f, 0.f, 0.f, 0.f};
        st4(As + kr * IA::P + (vi % (BM / 4)) * 4, v);
      }
    }
#pragma unroll
    for (int i = 0; i < VB; ++i) {
      const int vi = tid + i * NT;
      if (BKC) st4(Bs + (vi / (BK / 4)) * IB::P + (vi % (BK / 4)) * 4, rb[st][i]);
      else     st4(Bs + (vi / (BN / 4)) * IB::P + (vi % (BN / 4)) * 4, rb[st][i]);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // fused rowsum: thread owns row (tid % BM) and k phase (tid / BM)
  constexpr int RSP = NT / BM;
  float rs = 0.f;

  const int64_t nk = ke > kb0 ? (ke - kb0 + BK - 1) / BK : 0;
  const int lh = lane >> 5, lc = lane & 31;
  if constexpr (GL) {
    // LDS-DMA staging: wave w fills 1 KB chunks w, w + NW, ... of each image.  Rows >= M / N are
    // clamped (finite values feeding discarded outputs), k >= ke quads read zeros.
    typedef __attribute__((address_space(3))) void* lds_ptr;
    constexpr int CA = IA::FLOATS / 256, CB = IB::FLOATS / 256;
    static_assert(CA % NW == 0 && CB % NW == 0, "image chunks must split evenly over the waves");
    auto chunk = [&](auto KC_, auto ROWS_, const float* __restrict__ P, int64_t ld, int64_t rows, int64_t r0,
                     int64_t k0, float* dst, int c) {
      constexpr bool KC = decltype(KC_)::value;
      constexpr int ROWS = decltype(ROWS_)::value;
      const float* src;
      if constexpr (KC) {
        const int row = c * (256 / BK) + lane / (BK / 4);
        const int lq = (lane % (BK / 4)) ^ ImgL<true, ROWS, BK>::swz(row);
        const int64_t k = k0 + lq * 4, r = r0 + row < rows ? r0 + row : rows - 1;
        src = k < ke ? P + r * ld + k : g_zero4;
      } else {
        const int64_t k = k0 + c * (256 / ROWS) + lane / (ROWS / 4);
        const int64_t col = r0 + (lane % (ROWS / 4)) * 4;
        src = k < ke ? P + k * ld + (col < rows ? col : rows - 4) : g_zero4;
      }
      __builtin_amdgcn_global_load_lds(src, (lds_ptr)(dst + c * 256), 16, 0, 0);
    };
    auto dma_tile = [&](int buf, int64_t k0) {
      float* As = smem + buf * (IA::FLOATS + IB::FLOATS);
      float* Bs = As + IA::FLOATS;
#pragma unroll
      for (int i = 0; i < CA / NW; ++i)
        chunk(std::integral_constant<bool, AKC>{}, std::integral_constant<int, BM>{}, A, d.lda, d.M, m0, k0, As,
              wave + i * NW);
#pragma unroll
      for (int i = 0; i < CB / NW; ++i)
        chunk(std::integral_constant<bool, BKC>{}, std::integral_constant<int, BN>{}, B, d.ldb, d.N, n0, k0, Bs,
              wave + i * NW);
    };
    if (nk > 0) dma_tile(0, kb0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int64_t kt = 0; kt < nk; ++kt) {
      const int cur = (int)(kt & 1);
      if (kt + 1 < nk) dma_tile(cur ^ 1, kb0 + (kt + 1) * BK);   // buffer cur^1 was last read before the barrier
      const float* As = smem + cur * (IA::FLOATS + IB::FLOATS);
      const float* Bs = As + IA::FLOATS;
      mma_stage<IA, IB, TM, TN, BK>(As, Bs, acc, wm0, wn0, lane);
      if (do_rs) {
#pragma unroll
        for (int k = tid / BM; k < BK; k += RSP) rs += IA::elem(As, tid % BM, k);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of tile kt+1 has landed
      __syncthreads();                                     // ... and every other wave's
    }
  } else {
  if (nk > 0) load_tile(0, kb0);
  if (PF == 2 && nk > 1) load_tile(1 % PF, kb0 + BK);
  if (nk > 0) store_tile(0, 0, kb0);
  __syncthreads();
  // one k-tile: buffer (and register set) parity P = kt & 1 (static, the loop is unrolled by 2)
  auto step = [&](auto P_, int64_t kt) {
    constexpr int P = decltype(P_)::value;
#if !(defined(SRK_GEMM_EXP) && SRK_GEMM_EXP >= 1)   // experiment builds only: no global loads in the loop
    if (PF == 2) {
      if (kt + 2 < nk) load_tile(P % PF, kb0 + (kt + 2) * BK);
    } else {
      if (kt + 1 < nk) load_tile(0, kb0 + (kt + 1) * BK);
    }
#endif
    const float* As = smem + P * (IA::FLOATS + IB::FLOATS);
    const float* Bs = As + IA::FLOATS;
    mma_stage<IA, IB, TM, TN, BK>(As, Bs, acc, wm0, wn0, lane);
    if (do_rs) {
#pragma unroll
      for (int k = tid / BM; k < BK; k += RSP)
        rs += IA::elem(As, tid % BM, k);
    }
    asm volatile("" ::: "memory");      // keep the stage-k+1 LDS store (and its vmcnt wait)
    __builtin_amdgcn_sched_barrier(0);   // after this stage's MFMAs
#if defined(SRK_GEMM_EXP) && SRK_GEMM_EXP >= 2   // experiment builds only: no LDS stores either
    if (false)
#endif
    if (kt + 1 < nk) store_tile((P ^ 1) % PF, P ^ 1, kb0 + (kt + 1) * BK);
    __syncthreads();
  };
  for (int64_t kt = 0; kt < nk; kt += 2) {
    step(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < nk) step(std::integral_constant<int, 1>{}, kt + 1);
  }
  }   // register staging

  store_acc<TM, TN>(ka, acc, split, m0, n0, wm0, wn0, lane, z);
  if (do_rs) {
    float* red = smem;
    __syncthreads();
    red[tid] = rs;
    __syncthreads();
    if (tid < BM) {
      float t = 0.f;
#pragma unroll
      for (int p = 0; p < RSP; ++p) t += red[p * BM + tid];
      const int64_t row = m0 + tid;
      if (row < d.M) {
        if (ka.partial) ka.rs_partial[(int64_t)split * d.M + row] = t;
        else d.rowsum[row] = d.rowsum_beta != 0.f ? d.rowsum_beta * d.rowsum[row] + t : t;
      }
    }
  }
}

// ------------------------------------------------------------------ bf16 / fp16 operands
// Reduced-precision matrix-core GEMM (srk_set_option "matmul_precision" 1 / 2): the same fp32
// tensors in HBM, rounded to bf16 / fp16 (nearest-even, v_cvt_pk_*_f32) when a k-tile is staged into
// LDS, multiplied by v_mfma_f32_32x32x16_{bf16,f16} (1024 FLOP/clk/SIMD = 16x the fp32 MFMA) into
// fp32 accumulators; the epilogue, split-K slabs and fused row sums stay fp32 (row sums are taken
// from the fp32 staging registers, before rounding).
//
// Tile 128 x 128 x 64, 4 waves (2 x 2, each 64 x 64 = 2 x 2 MFMA tiles).  LDS images are
// k-contiguous for BOTH operands: [row][64 + 8] 16-bit elements (a 144-B pitch: a fragment
// ds_read_b128 of 32 rows hits 16 distinct bank quads per lane group).  A lane's MFMA operand is 8
// consecutive k of one row (k = 16 s + 8 (lane >> 5) + j), one ds_read_b128.  Staging unit per
// thread: k-contiguous operand -> 8 consecutive k of one row (2 float4 loads, 1 pack); row-contiguous
// operand -> 8 k x 4 rows (8 float4 loads, transposed in registers into 4 packs).
template <bool F16>
struct LpOps;
template <>
struct LpOps<false> {
  typedef __bf16 e8 __attribute__((ext_vector_type(8)));
  __device__ static __forceinline__ f32x16 mma(e8 a, e8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct LpOps<true> {
  typedef _Float16 e8 __attribute__((ext_vector_type(8)));
  __device__ static __forceinline__ f32x16 mma(e8 a, e8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};
typedef float v8f __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kLpBK = 64;
constexpr int kLpPitchQ = kLpBK / 8 + 1;            // image row pitch in 16-B quads (72 elements)

// Staging of one operand tile (ROWS x 64 k, fp32 in HBM) by NT threads.  Unit = KW consecutive k
// (KW = 8 -> one 16-B pack, KW = 4 -> one 8-B half pack) of 1 row (k-contiguous operand, 2 or 1
// float4 loads) or of 4 rows (row-contiguous operand: KW float4 loads transposed in registers into
// 4 packs).  Consecutive lanes walk k (LDS stores of 8 / 16 lanes fill one 128-B row chunk).
template <bool KC, int ROWS, int NT>
struct LpStage {
  static constexpr int UNITS8 = KC ? ROWS * (kLpBK / 8) : (ROWS / 4) * (kLpBK / 8);
  static constexpr int KW = UNITS8 >= NT ? 8 : 4;
  static constexpr int KCH = kLpBK / KW;                      // k chunks per row
  static constexpr int UNITS = KC ? ROWS * KCH : (ROWS / 4) * KCH;
  static constexpr int U = UNITS / NT;                        // units per thread
  static constexpr int V = KC ? U * KW / 4 : U * KW;          // float4 registers per thread
  static constexpr int RS = KC ? U : 4 * U;                   // rows per thread (fused row sums)
  static_assert(UNITS % NT == 0 && U >= 1, "staging must divide evenly");
};

template <int BM, int BN>
constexpr int lp_per_cu() { return 2 * (BM + BN) * kLpPitchQ * 16 <= 80 * 1024 ? 2 : 1; }

template <bool TA, bool TB, int BM, int BN, int NW, bool VEC, bool F16, int PF>
__global__ __launch_bounds__(NW * 64, (lp_per_cu<BM, BN>())) void gemm_lp_kernel(KernelArgs ka) {
  using Ops = LpOps<F16>;
  using e8 = typename Ops::e8;
  typedef typename LpOps<F16>::e8 e8_t;
  typedef __attribute__((ext_vector_type(4))) typename std::conditional<F16, _Float16, __bf16>::type e4;
  constexpr int NT = NW * 64, BK = kLpBK;
  constexpr int WM = (NW == 4) ? 2 : (BM >= 256 ? 4 : 2), WN = NW / WM;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1, "bad wave grid");
  constexpr bool AKC = !TA, BKC = TB;
  using SA = LpStage<AKC, BM, NT>;
  using SB = LpStage<BKC, BN, NT>;
  constexpr int IMGA = BM * kLpPitchQ, IMGB = BN * kLpPitchQ;   // quads
  __shared__ __attribute__((aligned(16))) u32x4 smem[2 * (IMGA + IMGB)];   // [stage][A | B] images
  const GemmDesc& d = ka.d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int split, tm, tn;
  map_tile(ka.nblk, ka.tiles, ka.tiles_m, ka.tiles_n, ka.group_m, ka.remap != 0, split, tm, tn);
  const int64_t z = blockIdx.z;
  const float* __restrict__ A = d.A + z * d.sA;
  const float* __restrict__ B = d.B + z * d.sB;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kb0 = split * ka.kchunk;
  const int64_t ke = (kb0 + ka.kchunk < d.K) ? kb0 + ka.kchunk : d.K;
  const int wm0 = (wave / WN) * (BM / WM), wn0 = (wave % WN) * (BN / WN);
  const bool do_rs = d.rowsum != nullptr && tn == 0;

  v4f ra[PF][SA::V], rb[PF][SB::V];
  // Loads are CLAMPED (rows >= rows -> last row / row group, k >= ke -> last k) and never
  // predicated; the k tail is zeroed at LDS-store time in BOTH images (a clamped duplicate may
  // overflow fp16).
  // Full k-tiles of VEC shapes load through buffer instructions: a per-thread 32-bit VGPR byte
  // offset fixed for the whole k loop (rows clamped once) + the k-tile's uniform byte offset in an
  // SGPR, so no per-load address arithmetic lands on the VALU (which the on-chip bf16 conversion
  // already keeps busy).  The host guarantees both operands' byte extents are < 2^31 for VEC.
  auto rsrc_of = [](const float* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7fffffff, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rsA = rsrc_of(A), rsB = rsrc_of(B);
  unsigned voA[SA::U], voB[SB::U];
  auto init_voff = [&](auto S_, unsigned* vo, int64_t ld, int64_t rows, int64_t r0) {
    using S = decltype(S_);
    constexpr bool KC = std::is_same<S, SA>::value ? AKC : BKC;
    const int kc = tid % S::KCH;
#pragma unroll
    for (int u = 0; u < S::U; ++u) {
      const int un = tid / S::KCH + u * (NT / S::KCH);
      if (KC) {
        const int64_t row = r0 + un < rows ? r0 + un : rows - 1;
        vo[u] = (unsigned)((row * ld + kc * S::KW) * 4);
      } else {
        const int64_t col = r0 + un * 4 < rows ? r0 + un * 4 : rows - 4;
        vo[u] = (unsigned)((kc * S::KW * ld + col) * 4);
      }
    }
  };
  if (VEC) {
    init_voff(SA{}, voA, d.lda, d.M, m0);
    init_voff(SB{}, voB, d.ldb, d.N, n0);
  }
  auto load_fast = [&](auto S_, v4f* r, __amdgpu_buffer_rsrc_t rs, const unsigned* vo, int64_t ld, int64_t k0) {
    using S = decltype(S_);
    constexpr bool KC = std::is_same<S, SA>::value ? AKC : BKC;
    constexpr int KW = S::KW;
#pragma unroll
    for (int u = 0; u < S::U; ++u) {
      if (KC) {
#pragma unroll
        for (int h = 0; h < KW / 4; ++h)
          r[u * (KW / 4) + h] = __builtin_bit_cast(
              v4f, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(vo[u] + 16 * h), (int)(k0 * 4), 0));
      } else {
#pragma unroll
        for (int e = 0; e < KW; ++e)
          r[u * KW + e] = __builtin_bit_cast(
              v4f, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo[u], (int)((k0 + e) * ld * 4), 0));
      }
    }
  };
  // Generic (tail tiles, unaligned shapes): CLAMPED addresses (rows >= rows -> last row / row group,
  // k >= ke -> last k), never predicated; the k tail is zeroed at LDS-store time in BOTH images (a
  // clamped duplicate may overflow fp16).
  auto load_op = [&](auto S_, v4f* r, const float* __restrict__ P, int64_t ld, int64_t rows, int64_t r0, int64_t k0) {
    using S = decltype(S_);
    constexpr bool KC = std::is_same<S, SA>::value ? AKC : BKC;
    constexpr int KW = S::KW, KCH = S::KCH;
    const int kc = tid % KCH;
#pragma unroll
    for (int u = 0; u < S::U; ++u) {
      const int un = tid / KCH + u * (NT / KCH);   // row (KC) or row group (!KC) of unit u
      if (KC) {
        const int64_t row = r0 + un;
        const float* q = P + (row < rows ? row : rows - 1) * ld;
#pragma unroll
        for (int h = 0; h < KW / 4; ++h) {
          const int64_t k = k0 + kc * KW + 4 * h;
          if (VEC) {
            r[u * (KW / 4) + h] = ld4(q + (k < ke - 3 ? k : ke - 4));
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) r[u * (KW / 4) + h][e] = q[k + e < ke ? k + e : ke - 1];
          }
        }
      } else {
        const int64_t col = r0 + un * 4;
#pragma unroll
        for (int e = 0; e < KW; ++e) {
          const int64_t k = k0 + kc * KW + e;
          const float* q = P + (k < ke ? k : ke - 1) * ld;
          if (VEC) {
            r[u * KW + e] = ld4(q + (col < rows ? col : rows - 4));
          } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) r[u * KW + e][c] = q[col + c < rows ? col + c : rows - 1];
          }
        }
      }
    }
  };
  float rs[SA::RS];
#pragma unroll
  for (int i = 0; i < SA::RS; ++i) rs[i] = 0.f;
  auto store_op = [&](auto S_, auto MASK_, const v4f* r, u32x4* img, int64_t k0, bool rowsum) {
    using S = decltype(S_);
    constexpr bool KC = std::is_same<S, SA>::value ? AKC : BKC;
    constexpr bool MASK = decltype(MASK_)::value;   // tail k-tile: zero k >= ke
    constexpr int KW = S::KW, KCH = S::KCH;
    const int kc = tid % KCH;
    const int64_t kbase = k0 + kc * KW;
    char* base = reinterpret_cast<char*>(img);
#pragma unroll
    for (int u = 0; u < S::U; ++u) {
      const int un = tid / KCH + u * (NT / KCH);
#pragma unroll
      for (int c = 0; c < (KC ? 1 : 4); ++c) {
        float v[KW];
#pragma unroll
        for (int e = 0; e < KW; ++e) {
          const float x = KC ? r[u * (KW / 4) + (e >> 2)][e & 3] : r[u * KW + e][c];
          v[e] = (MASK && kbase + e >= ke) ? 0.f : x;
        }
        if (rowsum) {
          float t = 0.f;
#pragma unroll
          for (int e = 0; e < KW; ++e) t += v[e];
          rs[KC ? u : 4 * u + c] += t;
        }
        const int row = KC ? un : 4 * un + c;
        char* dst = base + (size_t)row * kLpPitchQ * 16 + kc * KW * 2;
        if constexpr (KW == 8) {
          const v8f w{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
          *reinterpret_cast<u32x4*>(dst) = __builtin_bit_cast(u32x4, __builtin_convertvector(w, e8_t));
        } else {
          const v4f w{v[0], v[1], v[2], v[3]};
          typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
          *reinterpret_cast<u32x2*>(dst) = __builtin_bit_cast(u32x2, __builtin_convertvector(w, e4));
        }
      }
    }
  };
  auto load_tile = [&](int st, int64_t k0) {
    if (VEC && k0 + BK <= ke) {   // uniform branch
      load_fast(SA{}, ra[st], rsA, voA, d.lda, k0);
      load_fast(SB{}, rb[st], rsB, voB, d.ldb, k0);
    } else {
      load_op(SA{}, ra[st], A, d.lda, d.M, m0, k0);
      load_op(SB{}, rb[st], B, d.ldb, d.N, n0, k0);
    }
  };
  auto store_tile = [&](int st, int buf, int64_t k0) {
    u32x4* As = smem + buf * (IMGA + IMGB);
    if (k0 + BK <= ke) {   // uniform branch: only a split's last k-tile needs the k-tail mask
      store_op(SA{}, std::false_type{}, ra[st], As, k0, do_rs);
      store_op(SB{}, std::false_type{}, rb[st], As + IMGA, k0, false);
    } else {
      store_op(SA{}, std::true_type{}, ra[st], As, k0, do_rs);
      store_op(SB{}, std::true_type{}, rb[st], As + IMGA, k0, false);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lh = lane >> 5, lc = lane & 31;
  const int64_t nk = ke > kb0 ? (ke - kb0 + BK - 1) / BK : 0;
  auto mma_tile = [&](int buf) {
    const u32x4* As = smem + buf * (IMGA + IMGB);
    const u32x4* Bs = As + IMGA;
    u32x4 fa[2][TM], fb[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[0][i] = As[(wm0 + i * 32 + lc) * kLpPitchQ + lh];
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[0][j] = Bs[(wn0 + j * 32 + lc) * kLpPitchQ + lh];
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int c = ks & 1;
      if (ks + 1 < BK / 16) {
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[c ^ 1][i] = As[(wm0 + i * 32 + lc) * kLpPitchQ + 2 * (ks + 1) + lh];
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[c ^ 1][j] = Bs[(wn0 + j * 32 + lc) * kLpPitchQ + 2 * (ks + 1) + lh];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = Ops::mma(__builtin_bit_cast(e8, fa[c][i]), __builtin_bit_cast(e8, fb[c][j]), acc[i][j]);
    }
  };

  if (nk > 0) load_tile(0, kb0);
  if (PF == 2 && nk > 1) load_tile(1 % PF, kb0 + BK);
  if (nk > 0) store_tile(0, 0, kb0);
  __syncthreads();
  // k-tile kt: LDS buffer kt & 1, register set kt % PF (static: the loop is unrolled by 2)
  auto step = [&](auto P_, int64_t kt) {
    constexpr int P = decltype(P_)::value;
    if (PF == 2) {
      if (kt + 2 < nk) load_tile(P % PF, kb0 + (kt + 2) * BK);   // set P was stored last step
    } else {
      if (kt + 1 < nk) load_tile(0, kb0 + (kt + 1) * BK);
    }
    mma_tile(P);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);   // the next tile's LDS store after this tile's MFMAs
    if (kt + 1 < nk) store_tile((P ^ 1) % PF, P ^ 1, kb0 + (kt + 1) * BK);
    __syncthreads();
  };
  for (int64_t kt = 0; kt < nk; kt += 2) {
    step(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < nk) step(std::integral_constant<int, 1>{}, kt + 1);
  }
  store_acc<TM, TN>(ka, acc, split, m0, n0, wm0, wn0, lane, z);
  if (do_rs) {   // deterministic: partials [k chunk][row] in LDS, summed in chunk order
    constexpr int KCH = SA::KCH;
    float* red = reinterpret_cast<float*>(smem);
    static_assert(KCH * BM * 4 <= (int)sizeof(smem), "row-sum scratch");
    __syncthreads();
    const int kc = tid % KCH;
#pragma unroll
    for (int u = 0; u < SA::U; ++u) {
      const int un = tid / KCH + u * (NT / KCH);
      if (AKC) {
        red[kc * BM + un] = rs[u];
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) red[kc * BM + 4 * un + c] = rs[4 * u + c];
      }
    }
    __syncthreads();
    for (int t = tid; t < BM; t += NT) {
      float sum = 0.f;
#pragma unroll
      for (int p = 0; p < KCH; ++p) sum += red[p * BM + t];
      const int64_t row = m0 + t;
      if (row < d.M) {
        if (ka.partial) ka.rs_partial[(int64_t)split * d.M + row] = sum;
        else d.rowsum[row] = d.rowsum_beta != 0.f ? d.rowsum_beta * d.rowsum[row] + sum : sum;
      }
    }
  }
}

// ------------------------------------------------------------------ 16-bit operands in memory
// Both operands already bf16 / fp16 in HBM (GemmDesc::A16 / B16, written by their producers): every
// staged 16-B unit is 8 elements that go to LDS unchanged, so the tile moves HALF the bytes of the
// on-chip-rounding kernel above and spends no VALU on conversion.
//   k-contiguous operand:   unit = 8 consecutive k of one row  -> image [row][64 + 8], fragment =
//                           one ds_read_b128;
//   row-contiguous operand: unit = 8 consecutive rows at one k -> image [k][ROWS + 32] (pitch = 32
//                           mod 128 elements), fragment = 2 x ds_read_b64_tr_b16 (hardware transpose).
// VEC only (host-checked): 16-B aligned bases, leading dimensions % 8 == 0, K % 8 (k-contiguous) and
// rows % 8 (row-contiguous) == 0, so a unit is wholly valid or wholly invalid; invalid units are
// clamped loads zeroed at LDS-store time (k tail), or feed discarded outputs (rows).
typedef short s16x4_ __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));

template <bool KC, int ROWS>
struct H16Img {
  static constexpr int P = KC ? kLpBK + 8 : ROWS + 32;      // elements
  static constexpr int ELEMS = KC ? ROWS * P : kLpBK * P;
  static_assert(KC || P % 128 == 32, "transposed image pitch");
  __device__ static __forceinline__ u32x4 frag(const unsigned short* img, int c0, int kk, int lane) {
    if (KC) return *reinterpret_cast<const u32x4*>(img + (c0 + (lane & 31)) * P + kk + 8 * (lane >> 5));
    const int q = (lane >> 2) & 3, p = lane & 3;
    const unsigned short* a = img + (kk + 8 * (lane >> 5) + q) * P + c0 + 16 * ((lane >> 4) & 1) + 4 * p;
    typedef __attribute__((address_space(3))) s16x4_ lds_s16x4;
    const s16x4_ lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a));
    const s16x4_ hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 4 * P));
    const u32x2_ l2 = __builtin_bit_cast(u32x2_, lo), h2 = __builtin_bit_cast(u32x2_, hi);
    return u32x4{l2.x, l2.y, h2.x, h2.y};
  }
};

template <bool TA, bool TB, int BM, int BN>
constexpr int h16_per_cu() { return 2 * 2 * (H16Img<!TA, BM>::ELEMS + H16Img<TB, BN>::ELEMS) <= 80 * 1024 ? 2 : 1; }

template <bool TA, bool TB, int BM, int BN, int NW, bool F16>
__global__ __launch_bounds__(NW * 64, (h16_per_cu<TA, TB, BM, BN>())) void gemm_h16_kernel(KernelArgs ka) {
  using Ops = LpOps<F16>;
  using e8 = typename Ops::e8;
  constexpr int NT = NW * 64, BK = kLpBK;
  constexpr int WM = (NW == 4) ? 2 : (BM >= 256 ? 4 : 2), WN = NW / WM;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr bool AKC = !TA, BKC = TB;
  using IA = H16Img<AKC, BM>;
  using IB = H16Img<BKC, BN>;
  constexpr int UA = BM * 8 / NT, UB = BN * 8 / NT;   // 16-B units per thread per operand
  static_assert(UA >= 1 && UB >= 1 && BM * 8 % NT == 0 && BN * 8 % NT == 0, "staging");
  constexpr int STAGE = IA::ELEMS + IB::ELEMS;         // 16-bit elements per stage
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * STAGE];
  const GemmDesc& d = ka.d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int split, tm, tn;
  map_tile(ka.nblk, ka.tiles, ka.tiles_m, ka.tiles_n, ka.group_m, ka.remap != 0, split, tm, tn);
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t kb0 = split * ka.kchunk;
  const int64_t ke = (kb0 + ka.kchunk < d.K) ? kb0 + ka.kchunk : d.K;
  const int wm0 = (wave / WN) * (BM / WM), wn0 = (wave % WN) * (BN / WN);
  auto rsrc_of = [](const uint16_t* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(p), (short)0, 0x7fffffff, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rsA = rsrc_of(d.A16), rsB = rsrc_of(d.B16);

  // per-unit fixed byte offset (rows clamped once), LDS element offset and k offset within the tile
  unsigned voA[UA], voB[UB];
  int ldsA[UA], ldsB[UB], kuA[UA], kuB[UB];
  auto init = [&](auto KC_, auto ROWS_, unsigned* vo, int* lo, int* ku, int64_t ld, int64_t rows, int64_t r0) {
    constexpr bool KC = decltype(KC_)::value;
    constexpr int ROWS = decltype(ROWS_)::value;
    constexpr int U = ROWS * 8 / NT;
    using I = H16Img<KC, ROWS>;
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int u = tid + i * NT;
      if (KC) {   // row u / 8, k chunk u % 8
        const int row = u >> 3, kc = u & 7;
        const int64_t r = r0 + row < rows ? r0 + row : rows - 1;
        vo[i] = (unsigned)((r * ld + kc * 8) * 2);
        lo[i] = row * I::P + kc * 8;
        ku[i] = kc * 8;
      } else {    // k u / (ROWS / 8), row chunk u % (ROWS / 8)
        const int k = u / (ROWS / 8), rc = u % (ROWS / 8);
        const int64_t c = r0 + rc * 8 < rows ? r0 + rc * 8 : rows - 8;
        vo[i] = (unsigned)((k * ld + c) * 2);
        lo[i] = k * I::P + rc * 8;
        ku[i] = k;
      }
    }
  };
  init(std::integral_constant<bool, AKC>{}, std::integral_constant<int, BM>{}, voA, ldsA, kuA, d.lda, d.M, m0);
  init(std::integral_constant<bool, BKC>{}, std::integral_constant<int, BN>{}, voB, ldsB, kuB, d.ldb, d.N, n0);

  u32x4 ra[UA], rb[UB];
  // k-contiguous: k advances along the row (+2 B per k); row-contiguous: a k row is ld elements.
  // Full k-tiles (a uniform test) carry the k offset in the scalar soffset; only the k tail uses
  // per-lane offsets, where an invalid unit re-reads a valid one (k 0 of its row / k row ke - 1) and
  // is zeroed at LDS-store time.  (A per-lane soffset would make the compiler waterfall every load.)
  auto load_op = [&](auto KC_, auto U_, __amdgpu_buffer_rsrc_t rs, const unsigned* vo, const int* ku, int64_t ld,
                     u32x4* r, int64_t k0) {
    constexpr bool KC = decltype(KC_)::value;
    constexpr int U = decltype(U_)::value;
    const int64_t step = KC ? 2 : ld * 2;   // bytes per k
    if (k0 + BK <= ke) {
      const int soff = (int)(k0 * step);
#pragma unroll
      for (int i = 0; i < U; ++i)
        r[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vo[i], soff, 0));
    } else {
#pragma unroll
      for (int i = 0; i < U; ++i) {
        const int64_t off = k0 + ku[i] < ke ? (int64_t)vo[i] + k0 * step
                                            : (KC ? (int64_t)vo[i] - ku[i] * 2 : (int64_t)vo[i] + ((ke - 1) - ku[i]) * step);
        r[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
      }
    }
  };
  auto load_tile = [&](int64_t k0) {
    load_op(std::integral_constant<bool, AKC>{}, std::integral_constant<int, UA>{}, rsA, voA, kuA, d.lda, ra, k0);
    load_op(std::integral_constant<bool, BKC>{}, std::integral_constant<int, UB>{}, rsB, voB, kuB, d.ldb, rb, k0);
  };
  auto store_tile = [&](int buf, int64_t k0) {
    unsigned short* As = smem + buf * STAGE;
    unsigned short* Bs = As + IA::ELEMS;
    const bool tail = k0 + BK > ke;   // uniform
#pragma unroll
    for (int i = 0; i < UA; ++i) {
      const u32x4 v = (tail && k0 + kuA[i] >= ke) ? u32x4{0u, 0u, 0u, 0u} : ra[i];
      *reinterpret_cast<u32x4*>(As + ldsA[i]) = v;
    }
#pragma unroll
    for (int i = 0; i < UB; ++i) {
      const u32x4 v = (tail && k0 + kuB[i] >= ke) ? u32x4{0u, 0u, 0u, 0u} : rb[i];
      *reinterpret_cast<u32x4*>(Bs + ldsB[i]) = v;
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int64_t nk = ke > kb0 ? (ke - kb0 + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tile(kb0);
    store_tile(0, kb0);
  }
  __syncthreads();
  for (int64_t kt = 0; kt < nk; ++kt) {
    const int cur = (int)(kt & 1);
    if (kt + 1 < nk) load_tile(kb0 + (kt + 1) * BK);
    const unsigned short* As = smem + cur * STAGE;
    const unsigned short* Bs = As + IA::ELEMS;
    u32x4 fa[2][TM], fb[2][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[0][i] = IA::frag(As, wm0 + i * 32, 0, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[0][j] = IB::frag(Bs, wn0 + j * 32, 0, lane);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int c = ks & 1;
      if (ks + 1 < BK / 16) {
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[c ^ 1][i] = IA::frag(As, wm0 + i * 32, 16 * (ks + 1), lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[c ^ 1][j] = IB::frag(Bs, wn0 + j * 32, 16 * (ks + 1), lane);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = Ops::mma(__builtin_bit_cast(e8, fa[c][i]), __builtin_bit_cast(e8, fb[c][j]), acc[i][j]);
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) store_tile(cur ^ 1, kb0 + (kt + 1) * BK);
    __syncthreads();
  }
  store_acc<TM, TN>(ka, acc, split, m0, n0, wm0, wn0, lane, 0);
}

// map_tile for a virtual block index v (persistent kernels: v = blockIdx.x + r gridDim.x), same order
__device__ __forceinline__ void map_tile_v(int v, int nblk, int tiles, int tiles_m, int tiles_n, int group_m,
                                           bool remap, int& split, int& tm, int& tn) {
  int lin = v;
  if (remap) {
    const int xcd = v & 7, q = nblk >> 3, r = nblk & 7;
    lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (v >> 3);
  }
  split = lin / tiles;
  tile_of(lin - split * tiles, tiles_m, tiles_n, group_m, tm, tn);
}

// Epilogue of the ping-pong kernels (gemm_g16_kernel, gemm_p32_kernel): each wave stages 64 x 64
// fp32 of its 128 x 64 accumulator block per pass through LDS (16 KB per wave, 128 KB for the 8
// waves; the K ring is idle by then), then writes rows as 16-B vectors (4 rows x 256 B per
// instruction) instead of the 32x32 accumulator layout's 4-B scalar stores.  Split-K launches write
// the raw slab; otherwise alpha, bias and beta are applied.
__device__ __forceinline__ void pp_epilogue(const KernelArgs& ka, const f32x16 (&acc)[4][2], float* lds, int split,
                                            int64_t m0, int64_t n0, int grp, int wc, int wave, int lane,
                                            int64_t z = 0, float* slab = nullptr) {
  const GemmDesc& d = ka.d;
  float* st = lds + wave * 4096;
  const bool split_mode = ka.partial != nullptr || slab != nullptr;   // raw partial sums, [M][N]
  // batched launches: batch z's slabs follow batch z - 1's ([batch][splits][M][N])
  float* C = slab ? slab : split_mode ? ka.partial + (z * (ka.nblk / ka.tiles) + split) * d.M * d.N : d.C + z * d.sC;
  const int64_t ldc = split_mode ? d.N : d.ldc;
  const bool vec = (ldc % 4 == 0) && ((uintptr_t)C % 16 == 0);
  const int lh = lane >> 5, lc = lane & 31;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          st[(i2 * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * 64 + j * 32 + lc] = acc[2 * h + i2][j][r];
#pragma unroll 4
    for (int v = 0; v < 16; ++v) {
      const int rl = v * 4 + (lane >> 4), c4 = (lane & 15) * 4;
      const int64_t row = m0 + grp * 128 + h * 64 + rl, col = n0 + wc * 64 + c4;
      if (row >= d.M || col >= d.N) continue;
      v4f x = *reinterpret_cast<const v4f*>(st + rl * 64 + c4);
      float* c = C + row * ldc + col;
      if (!split_mode) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          x[e] *= d.alpha;
          if (d.bias_mode == 1) x[e] += col + e < d.N ? d.bias[col + e] : 0.f;
          else if (d.bias_mode == 2) x[e] += d.bias[row];
        }
      }
      if (vec && col + 3 < d.N) {
        if (!split_mode && d.beta != 0.f) x += d.beta * *reinterpret_cast<const v4f*>(c);
        *reinterpret_cast<v4f*>(c) = x;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (col + e >= d.N) break;
          float y = x[e];
          if (!split_mode && d.beta != 0.f) y += d.beta * c[e];
          c[e] = y;
        }
      }
    }
  }
}

// ------------------------------------------------------------------ 16-bit operands: LDS-DMA ping-pong
// gemm_g16_kernel: the same contract as gemm_h16_kernel (16-bit A16 / B16 in HBM, fp32 accumulation,
// split-K slabs), restructured so the matrix pipe never waits on staging:
//
//  * 256 x 256 output tile, 8 waves = two GROUPS of 4 (group g = wave >> 2 owns A rows 128 g .. +128;
//    wave w & 3 owns columns 64 (w & 3) .. +64), 128 x 64 outputs per wave as 4 x 2 32x32x16 MFMA tiles;
//  * the k loop is a sequence of PHASES, one per 16-deep k-step (8 MFMAs = 256 cycles per wave, all 8
//    accumulators once); a phase is a LOAD section (the k-step's 6 fragments — 4 A row blocks, 2 B
//    column blocks — plus part of a later K-tile's LDS-DMA issue) and an MFMA section, each closed
//    by a raw s_barrier.  The two groups run one section apart (group 1 takes one extra barrier up
//    front, group 0 one at the end): while one group's waves multiply, the other group's waves — one
//    per SIMD in each group — read LDS, so each SIMD's matrix pipe alternates between its two waves;
//  * operands reach LDS by buffer_load_dwordx4 ... lds (LDS-DMA, no VGPR round trip) into lane-linear
//    half-tile images (8 KB: 128 rows x 32 k, or 32 k x 128 rows) swizzled on the SOURCE address; a
//    k-tail or out-of-range unit is read past the descriptor's num_records, i.e. as 16 zero bytes, so
//    the products are exact zeros; per lane one fixed offset, the K-tile's k in the scalar soffset;
//  * a ring of NST K-tile stages of 32 k (32 KB each; NST = 4 measured faster than 5): K-tile t + NST - 1
//    is issued into the stage of K-tile t - 1 in K-tile t's two phases (A halves, then B halves) —
//    that stage's last reads retired before the previous barrier (every load section waits
//    lgkmcnt(0) before its barrier) — and K-tile t + 1 is retired by a counted vmcnt in K-tile t's
//    last load section, NST - 2 K-tiles after its issue (~2 x 256 MFMA cycles x 2 (NST - 1) of
//    latency cover).  MI355X_MICROARCH.md / cdna_hip_programming.md rules: raw s_barrier, never
//    __syncthreads() while a DMA is in flight; one __shared__ array; the DMA is inline asm, so the
//    compiler knows of no pending LDS write and inserts no vmcnt(0) before the fragment reads (with
//    the builtin it did, before every ds_read_b64_tr_b16, draining the ring every K-tile);
//  * the epilogue stages each wave's accumulators through the (then idle) LDS and writes 16-B rows.
//
// KC image (operand k-contiguous in HBM): [128 rows][4 units of 8 k] (64-B rows), unit slot
//   kc ^ ((row >> 2) & 3); a 32x32x16 fragment (lane: row l & 31, 8 k at 8 (l >> 5)) is one
//   conflict-free ds_read_b128 (the 4 rows sharing a bank row per 16-lane group get 4 slots).
// TR image (row-contiguous): [32 k][16 units of 8 rows] (256-B rows), unit slot u ^ ((k & 3) << 2);
//   a fragment is 2 x ds_read_b64_tr_b16 whose 4 k-rows per half-wave land on 4 distinct 64-B groups.
constexpr int kG16BK = 32;
template <bool KC>
struct G16Half {
  static constexpr int ELEMS = 128 * kG16BK;   // 8 KB
  static constexpr int PIECES = ELEMS / 512;   // 1-KB DMA pieces (one wave-instruction each)
  // element offset of logical (row, k); the 16-B unit holding it is whole, so fragments stay contiguous
  __device__ static __forceinline__ int off(int row, int k) {
    if (KC) return row * kG16BK + ((((k >> 3) ^ ((row >> 2) & 3))) << 3) + (k & 7);
    return k * 128 + ((((row >> 3) ^ ((k & 3) << 2))) << 3) + (row & 7);
  }
  // 32x32x16 operand fragment for rows r0 .. r0 + 31 (within the half), k = kk .. kk + 15
  __device__ static __forceinline__ u32x4 frag(const unsigned short* img, int r0, int kk, int lane) {
    if (KC) return *reinterpret_cast<const u32x4*>(img + off(r0 + (lane & 31), kk + 8 * (lane >> 5)));
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int k = kk + 8 * (lane >> 5) + q, row = r0 + 16 * ((lane >> 4) & 1) + 4 * p;
    typedef __attribute__((address_space(3))) s16x4_ lds_s16x4;
    const s16x4_ lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off(row, k)));
    const s16x4_ hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + off(row, k + 4)));
    const u32x2_ l2 = __builtin_bit_cast(u32x2_, lo), h2 = __builtin_bit_cast(u32x2_, hi);
    return u32x4{l2.x, l2.y, h2.x, h2.y};
  }
  // The unit lane `lane` of DMA piece `piece` brings into this half image, for the K-tile at k0 = 0:
  // its byte offset from the operand base, the k offset kk of that unit within the K-tile, and
  // whether its rows are in range.  A K-tile at k0 adds k0 * KSTEP bytes (the buffer load's soffset).
  __device__ static __forceinline__ void src(int piece, int lane, int64_t r0, int64_t rows, int64_t ld, unsigned& voff,
                                             int& kk, bool& row_ok) {
    const int p = piece * 64 + lane;
    if (KC) {   // p = row * 4 + slot
      const int row = p >> 2, kc = (p & 3) ^ ((row >> 2) & 3);
      voff = (unsigned)(((r0 + row) * ld + kc * 8) * 2);
      kk = kc * 8;
      row_ok = r0 + row < rows;
    } else {    // p = k * 16 + slot
      const int k = p >> 4, u = (p & 15) ^ ((k & 3) << 2);
      voff = (unsigned)((k * ld + r0 + u * 8) * 2);
      kk = k;
      row_ok = r0 + u * 8 < rows;
    }
  }
  __device__ static __forceinline__ int64_t kstep_bytes(int64_t ld) { return KC ? 2 : 2 * ld; }
};

#ifndef SRK_G16_STAGES
#define SRK_G16_STAGES 4
#endif
constexpr int kG16Stages = SRK_G16_STAGES;
static_assert(kG16Stages >= 4 && kG16Stages <= 5, "g16 ring: 4..5 stages of 32 KB (the epilogue needs 128 KB)");

// Measured and dropped (rounds 4-5, git history keeps them): a persistent tile loop with a direct
// epilogue, 32-deep sections (16 MFMAs between barriers), static priority for the second group,
// non-temporal C stores.
template <bool TA, bool TB, bool F16>
__global__ __launch_bounds__(512, 1) void gemm_g16_kernel(KernelArgs ka) {
  using Ops = LpOps<F16>;
  using e8 = typename Ops::e8;
  constexpr int BK = kG16BK, NST = kG16Stages;
  constexpr bool AKC = !TA, BKC = TB;
  using HA = G16Half<AKC>;
  using HB = G16Half<BKC>;
  constexpr int HALF = HA::ELEMS;                 // 16-bit elements per half image
  constexpr int STAGE = 4 * HALF;                 // A0 A1 B0 B1 = 32 KB
  static_assert(NST * STAGE * 2 >= 8 * 4096 * 4, "the epilogue stages 128 KB of fp32 through the ring");
  __shared__ __attribute__((aligned(1024))) unsigned short smem[NST * STAGE];   // the only LDS object
  typedef __attribute__((address_space(3))) void* lds_ptr;
  // raw workgroup barrier (no vmcnt drain: DMAs stay in flight across it); the empty asm statements
  // keep the compiler from moving LDS reads across it
  auto bar = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const GemmDesc& d = ka.d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, grp = wave >> 2, wc = wave & 3;
  const int vblk = blockIdx.x;
  int split, tm, tn;
  map_tile_v(vblk, ka.nblk, ka.tiles, ka.tiles_m, ka.tiles_n, ka.group_m, ka.remap != 0, split, tm, tn);
  const int64_t m0 = (int64_t)tm * 256, n0 = (int64_t)tn * 256;
  const int64_t kb0 = split * ka.kchunk;
  const int64_t ke = (kb0 + ka.kchunk < d.K) ? kb0 + ka.kchunk : d.K;
  const int nk = ke > kb0 ? (int)((ke - kb0 + BK - 1) / BK) : 0;

  // LDS-DMA by buffer_load_dwordx4 ... lds (inline asm: the compiler knows of no pending LDS write, so
  // it inserts no vmcnt(0) before the fragment reads — with the global_load_lds builtin it did, before
  // every ds_read_b64_tr_b16, draining the ring every K-tile).  Per lane a fixed 32-bit byte offset
  // (rows clamped once); the K-tile's k0 goes in the scalar soffset; a unit outside the rows or past
  // the split's k end gets an offset beyond num_records, which the buffer range check turns into 16
  // zero bytes.  M0 = the piece's LDS base (saved and restored around the DMA).
  typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
  auto rsrc16 = [](const uint16_t* p) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    return u32x4s{(unsigned)__builtin_amdgcn_readfirstlane((unsigned)a),
                  (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)), 0x7ffffff0u, 0x00020000u};
  };
  const int64_t z = blockIdx.y;   // batch index (grid.y = batch; strides sA / sB in elements)
  const u32x4s rsA = rsrc16(d.A16 + z * d.sA), rsB = rsrc16(d.B16 + z * d.sB);
  constexpr unsigned kOOB = 0x80000000u;
  unsigned vo[4];
  int kk[4];
  bool rok[4];
  G16Half<AKC>::src(wave, lane, m0, d.M, d.lda, vo[0], kk[0], rok[0]);
  G16Half<AKC>::src(wave, lane, m0 + 128, d.M, d.lda, vo[1], kk[1], rok[1]);
  G16Half<BKC>::src(wave, lane, n0, d.N, d.ldb, vo[2], kk[2], rok[2]);
  G16Half<BKC>::src(wave, lane, n0 + 128, d.N, d.ldb, vo[3], kk[3], rok[3]);
  const int64_t ksA = G16Half<AKC>::kstep_bytes(d.lda), ksB = G16Half<BKC>::kstep_bytes(d.ldb);
  const unsigned lds0 =
      (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ptr)smem + (unsigned)wave * 1024u);
  auto dma = [&](int t, int h) {   // K-tile t, half image h (0, 1: A rows; 2, 3: B columns)
    const int64_t k0 = kb0 + (int64_t)t * BK;
    const bool full = k0 + BK <= ke;   // uniform: only a split's last K-tile has a k tail
    const unsigned v = (rok[h] && (full || k0 + kk[h] < ke)) ? vo[h] : kOOB;
    const unsigned soff = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(k0 * (h < 2 ? ksA : ksB)));
    const unsigned ldsa = lds0 + (unsigned)(((t % NST) * STAGE + h * HALF) * 2);
    unsigned keep;
    if (h < 2)
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(v), "s"(rsA), "s"(ldsa), "s"(soff)
                   : "memory");
    else
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(v), "s"(rsB), "s"(ldsa), "s"(soff)
                   : "memory");
  };
  auto dma_a = [&](int t) { dma(t, 0); dma(t, 1); };   // K-tile t's A halves (2 DMA instructions per wave)
  auto dma_b = [&](int t) { dma(t, 2); dma(t, 3); };   // K-tile t's B halves

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // prologue: K-tiles 0 .. NST - 2 in flight (4 DMA instructions per wave each), tile 0 retired
  for (int t = 0; t < NST - 1; ++t)
    if (t < nk) {
      dma_a(t);
      dma_b(t);
    }
  // vmcnt wants an immediate: retire tile 0, leaving min(nk - 1, NST - 2) tiles in flight
  auto retire_keep = [](int tiles_in_flight) {
    if (tiles_in_flight >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (tiles_in_flight == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (tiles_in_flight == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  retire_keep(min(nk - 1, NST - 2));
  bar();
  if (grp == 1) bar();   // the groups run one section apart

  const int bh = wc >> 1, bc0 = (wc & 1) * 64;   // this wave's B half image and its column base there
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned short* S = smem + (kt % NST) * STAGE;
    const unsigned short* As = S + grp * HALF;
    const unsigned short* Bs = S + (2 + bh) * HALF;
    const int tn_ = kt + NST - 1;   // the K-tile issued during this one (into K-tile kt - 1's stage)
#pragma unroll
    for (int q = 0; q < BK / 16; ++q) {
      // ---- load section: k-step q's fragments (4 A row blocks, 2 B column blocks)
      u32x4 fa[4], fb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = HA::frag(As, i * 32, 16 * q, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = HB::frag(Bs, bc0 + j * 32, 16 * q, lane);
#if !(defined(SRK_G16_EXP) && SRK_G16_EXP == 1)   // experiment builds only: no DMA after the prologue
      if (tn_ < nk) {
        if (q == 0) dma_a(tn_);
        else dma_b(tn_);
      }
#endif
#if !(defined(SRK_G16_EXP) && SRK_G16_EXP == 2)   // experiment builds only: DMA never waited for in the loop
      if (q + 1 == BK / 16) retire_keep(min(nk - 1 - (kt + 1), NST - 2));   // K-tile kt + 1 landed (this wave's part)
#endif
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this section's fragments are in registers
      bar();
      // ---- MFMA section: 8 independent accumulators
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = Ops::mma(__builtin_bit_cast(e8, fa[i]), __builtin_bit_cast(e8, fb[j]), acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
  }
  if (grp == 0) bar();   // equal barrier counts; every wave is past its last LDS read and DMA wait

  // ---- epilogue (the ring is idle now): pp_epilogue
#if defined(SRK_G16_EXP) && SRK_G16_EXP == 3   // experiment builds only: no C stores (kept live)
  if (d.alpha != 12345.f) return;
#endif
  pp_epilogue(ka, acc, reinterpret_cast<float*>(smem), split, m0, n0, grp, wc, wave, lane, z);
}

// ------------------------------------------------------------------ skinny GEMMs (VALU)
// GEMMs with one dimension <= 16 — the 12-class output layer of every model (models/model_*.py
// `fc`: forward x W^T, dx = dY W, dW = dY^T x with db) — are a few MFLOP: on the 128 x 128 matrix-core
// tiles they are 15-30 us of launch, staging and split-K reduction each (tools/step_kernels.py, r03s3:
// 59 us of the 1.45 ms cfg2 bf16 step).  These kernels stream the long operand once, coalesced, and
// keep the <= 16 short-side accumulators in registers: fp32 FMAs on the operands rounded exactly as
// the matrix cores would (RND 1 bf16, 2 fp16, nearest-even: the products of two 16-bit values are
// exact in fp32, so only the fp32 summation order differs from the MFMA kernels); row sums of op(A)
// from the unrounded values, as in the tile kernels.
template <int RND>
__device__ __forceinline__ float rnd16(float x) {
  if constexpr (RND == 1) return (float)(__bf16)x;
  else if constexpr (RND == 2) return (float)(_Float16)x;
  else return x;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ void skinny_store(const GemmDesc& d, int64_t m, int64_t n, float acc) {
  float v = d.alpha * acc;
  if (d.bias_mode == 1) v += d.bias[n];
  else if (d.bias_mode == 2) v += d.bias[m];
  float* c = d.C + m * d.ldc + n;
  if (d.beta != 0.f) v += d.beta * *c;
  *c = v;
}

// N <= 16, A k-contiguous (!ta): a 256-thread block per row m of C; the 4 waves interleave over k
// (lane + 64 w + 256 i: A's row read once, coalesced), 4 k per lane per iteration with every load
// issued before the FMAs (K = 1024: one iteration), N accumulators per lane, a wave reduction per
// column, then the 4 waves' sums added through LDS in wave order (deterministic).
template <int RND, bool TB>
__global__ __launch_bounds__(256) void skinny_n_kernel(GemmDesc d) {
  __shared__ float part[4][17];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t m = blockIdx.x;
  float acc[16], rs = 0.f;
#pragma unroll
  for (int n = 0; n < 16; ++n) acc[n] = 0.f;
  const float* __restrict__ a = d.A + m * d.lda;
  for (int64_t k0 = lane + 64 * w; k0 < d.K; k0 += 1024) {
    float av[4], bv[4][16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t k = k0 + 256 * u;
      const bool ok = k < d.K;
      const int64_t kc = ok ? k : 0;   // clamped: loads stay unconditional
      av[u] = ok ? a[kc] : 0.f;
#pragma unroll
      for (int n = 0; n < 16; ++n) {
        const int nn = n < d.N ? n : (int)d.N - 1;   // clamped column, never stored
        bv[u][n] = TB ? d.B[nn * d.ldb + kc] : d.B[kc * d.ldb + nn];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      rs += av[u];
      const float ar = rnd16<RND>(av[u]);
#pragma unroll
      for (int n = 0; n < 16; ++n) acc[n] = fmaf(ar, rnd16<RND>(bv[u][n]), acc[n]);   // av = 0 past K
    }
  }
#pragma unroll
  for (int n = 0; n < 16; ++n) {   // predicated, no early exit: the accumulators stay in registers
    const float t = wave_sum(acc[n]);
    if (lane == n) part[w][n] = t;
  }
  const float r = wave_sum(rs);
  if (lane == 0) part[w][16] = r;
  __syncthreads();
  if (w == 0 && lane < d.N) skinny_store(d, m, lane, ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane]);
  if (w == 0 && lane == 16 && d.rowsum) {
    const float t = ((part[0][16] + part[1][16]) + part[2][16]) + part[3][16];
    d.rowsum[m] = d.rowsum_beta != 0.f ? d.rowsum_beta * d.rowsum[m] + t : t;
  }
}

// M <= 16, B row-contiguous (!tb), K <= 1024: a 1024-thread block owns 64 columns of C (lane =
// column).  op(A) (<= 16 x 1024) is first staged into LDS as [k][16]; the 16 waves split K into 16
// ranges and walk them 16 k at a time — 16 coalesced B loads in flight per lane, op(A)[., k] read as
// four broadcast ds_read_b128 — and the 16 partial sums per element are added through LDS in wave
// order (deterministic).  Block 0 also reduces the row sums (of the unrounded op(A)).
template <int RND, bool TA>
__global__ __launch_bounds__(1024) void skinny_m_kernel(GemmDesc d) {
  __shared__ __attribute__((aligned(16))) float As[1024 * 16];
  __shared__ float red[16][16][64];
  __shared__ float rsred[16][16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < d.K * 16; i += 1024) {
    const int k = i >> 4, m = i & 15;
    As[i] = m < d.M ? (TA ? d.A[(int64_t)k * d.lda + m] : d.A[(int64_t)m * d.lda + k]) : 0.f;
  }
  __syncthreads();
  const int64_t n = (int64_t)blockIdx.x * 64 + lane;
  const int64_t nc = n < d.N ? n : d.N - 1;   // clamped: every lane takes part in the loads
  const int kper = (int)((d.K + 15) / 16), kb = w * kper, ke = kb + kper < d.K ? kb + kper : (int)d.K;
  float acc[16], rs[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) acc[m] = rs[m] = 0.f;
  for (int k0 = kb; k0 < ke; k0 += 16) {
    float bv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const bool ok = k0 + u < ke;
      bv[u] = ok ? d.B[(int64_t)(k0 + u) * d.ldb + nc] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (k0 + u >= ke) break;   // uniform
      const float b = rnd16<RND>(bv[u]);
      const v4f* arow = reinterpret_cast<const v4f*>(As + (k0 + u) * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const v4f a4 = arow[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          rs[4 * q + e] += a4[e];
          acc[4 * q + e] = fmaf(rnd16<RND>(a4[e]), b, acc[4 * q + e]);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    red[w][m][lane] = acc[m];
    if (lane == 0) rsred[w][m] = rs[m];
  }
  __syncthreads();
  const int m = w;   // wave m finalizes row m of this block's 64 columns
  if (m < d.M) {
    float t = 0.f;
    for (int q = 0; q < 16; ++q) t += red[q][m][lane];
    if (n < d.N) skinny_store(d, m, n, t);
    if (d.rowsum && blockIdx.x == 0 && lane == 0) {
      float r = 0.f;
      for (int q = 0; q < 16; ++q) r += rsred[q][m];
      d.rowsum[m] = d.rowsum_beta != 0.f ? d.rowsum_beta * d.rowsum[m] + r : r;
    }
  }
}

// K <= 16, B row-contiguous (!tb): one thread per C element, block = 256 columns of one row m; the
// k loop is unrolled so every load is in flight at once (op(A)[m, k] is block-uniform).
template <int RND, bool TA>
__global__ __launch_bounds__(256) void skinny_k_kernel(GemmDesc d) {
  const int64_t m = blockIdx.y, n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nc = n < d.N ? n : d.N - 1;
  float av[16], bv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const bool ok = k < d.K;
    av[k] = ok ? (TA ? d.A[k * d.lda + m] : d.A[m * d.lda + k]) : 0.f;
    bv[k] = ok ? d.B[k * d.ldb + nc] : 0.f;
  }
  float acc = 0.f, rs = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    rs += av[k];
    acc = fmaf(rnd16<RND>(av[k]), rnd16<RND>(bv[k]), acc);
  }
  if (n < d.N) skinny_store(d, m, n, acc);
  if (d.rowsum && blockIdx.x == 0 && threadIdx.x == 0)
    d.rowsum[m] = d.rowsum_beta != 0.f ? d.rowsum_beta * d.rowsum[m] + rs : rs;
}

// Algorithmic HBM bytes of one GEMM launch (ProfScope::bytes): op(A) and op(B) read once at their element
// size in HBM, C written once (and read once when beta != 0), per batch entry.
inline double gemm_bytes(const GemmDesc& d, int esz) {
  const double c = (double)d.M * (double)d.N * 4.0 * (d.beta != 0.f ? 2.0 : 1.0);
  return ((double)d.M * (double)d.K * esz + (double)d.K * (double)d.N * esz + c) * (double)d.batch;
}

template <int RND>
int launch_skinny_rnd(const GemmDesc& d, int kind, hipStream_t s) {
  ProfScope prof(RND == 0 ? "gemm_f32" : RND == 1 ? "gemm_bf16" : "gemm_f16", s,
                 2.0 * (double)d.M * (double)d.N * (double)d.K);
  prof.bytes(gemm_bytes(d, 4));
  const char* kn = kind == 0 ? "skinny_n" : kind == 1 ? "skinny_m" : "skinny_k";
  prof.detail("%s_kernel<%c%c> %lldx%lldx%lld", kn, d.ta ? 'T' : 'N', d.tb ? 'T' : 'N', (long long)d.M,
              (long long)d.N, (long long)d.K);
  if (kind == 0) {
    const dim3 grid((unsigned)d.M);
    if (d.tb) hipLaunchKernelGGL((skinny_n_kernel<RND, true>), grid, dim3(256), 0, s, d);
    else hipLaunchKernelGGL((skinny_n_kernel<RND, false>), grid, dim3(256), 0, s, d);
  } else if (kind == 1) {
    const dim3 grid((unsigned)((d.N + 63) / 64));
    if (d.ta) hipLaunchKernelGGL((skinny_m_kernel<RND, true>), grid, dim3(1024), 0, s, d);
    else hipLaunchKernelGGL((skinny_m_kernel<RND, false>), grid, dim3(1024), 0, s, d);
  } else {
    const dim3 grid((unsigned)((d.N + 255) / 256), (unsigned)d.M);
    if (d.ta) hipLaunchKernelGGL((skinny_k_kernel<RND, true>), grid, dim3(256), 0, s, d);
    else hipLaunchKernelGGL((skinny_k_kernel<RND, false>), grid, dim3(256), 0, s, d);
  }
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

// Which skinny kernel takes this GEMM (-1: none; the matrix-core tiles run it).  Sizes keep each
// kernel's per-thread loop short and its streamed operand a few MB at most.
int skinny_kind(const GemmDesc& d) {
  if (!g_opt_gemm_skinny || d.batch != 1 || d.A16 || d.B16 || d.K <= 0) return -1;
  if (d.N <= 16 && !d.ta && d.M <= 65535 * 16 && d.M * d.K <= (int64_t)1 << 24) return 0;
  if (d.M <= 16 && !d.tb && d.K <= 1024 && d.N * d.K <= (int64_t)1 << 24) return 1;
  if (d.K <= 16 && !d.tb && d.M <= 65535 && d.M * d.N <= (int64_t)1 << 24) return 2;
  return -1;
}

// ------------------------------------------------------------------ fp32: LDS-DMA ping-pong
// gemm_p32_kernel: the exact-fp32 GEMM (v_mfma_f32_32x32x2_f32) on the structure of gemm_g16_kernel —
// 256 x 256 tiles, two 4-wave groups running one section apart behind raw barriers, a ring of four
// 16-deep K-tiles (32 KB each) filled by inline-asm buffer_load ... lds with zero-filled edges, and
// the LDS-staged epilogue.  A phase is one 8-deep k block: its load section reads 6 fragments (4 A
// row blocks, 2 B column blocks, 4 k per lane each: the k order inside a block is permuted so lanes of
// half h take k = 8 kb + 4 h + s at sub-step s, as in the register-staged kernel) and issues 2 DMA
// pieces; its MFMA section is 32 MFMAs = 2,048 cycles per wave.  The register-staged gemm_f32_kernel
// keeps the matrix pipe 64-76 % busy at the clock it holds (PMC, profiles/r02c_gemm_f32_pmc.txt; its
// waves park ~28 % of their cycles at the per-K-tile drain and barrier); this structure gains 6-7 %
// on the dx / dW_ih shapes and loses on the x W^T projection, so it is used for the former only —
// the fp32 matrix pipe, not the staging, is what binds both.  Row sums of op(A) (the dW GEMMs' fused bias gradient) come from the A
// fragments of the column-0 waves.
//
// KC image (k-contiguous operand): [128 rows][4 units of 4 k] (64-B rows), unit slot u ^ ((row >> 2) & 3):
//   a fragment (row l & 31, 4 k at unit 2 kb + (l >> 5)) is one conflict-free ds_read_b128.
// TR image (row-contiguous operand): [16 k][128 rows] (512-B rows), unswizzled: a fragment is 4
//   ds_read_b32 of 32 consecutive rows per half-wave (the halves on k rows 4 apart).
constexpr int kP32BK = 16;
template <bool KC>
struct P32Half {
  static constexpr int FLOATS = 128 * kP32BK;   // 8 KB
  __device__ static __forceinline__ v4f frag(const float* img, int r0, int kb, int lane) {
    const int row = r0 + (lane & 31), h = lane >> 5;
    if (KC) return *reinterpret_cast<const v4f*>(img + row * kP32BK + (((2 * kb + h) ^ ((row >> 2) & 3)) << 2));
    const float* q = img + (8 * kb + 4 * h) * 128 + row;
    return v4f{q[0], q[128], q[256], q[384]};
  }
  // lane's unit of DMA piece `piece` (1 KB = 64 units of 16 B) for the K-tile at k0 = 0: byte offset,
  // k offset within the K-tile, rows in range
  __device__ static __forceinline__ void src(int piece, int lane, int64_t r0, int64_t rows, int64_t ld, unsigned& voff,
                                             int& kk, bool& row_ok) {
    const int p = piece * 64 + lane;
    if (KC) {   // p = row * 4 + slot
      const int row = p >> 2, kc = (p & 3) ^ ((row >> 2) & 3);
      voff = (unsigned)(((r0 + row) * ld + kc * 4) * 4);
      kk = kc * 4;
      row_ok = r0 + row < rows;
    } else {    // p = k * 32 + unit (4 rows)
      const int k = p >> 5, u = p & 31;
      voff = (unsigned)((k * ld + r0 + u * 4) * 4);
      kk = k;
      row_ok = r0 + u * 4 < rows;
    }
  }
  __device__ static __forceinline__ int64_t kstep_bytes(int64_t ld) { return KC ? 4 : 4 * ld; }
};

template <bool TA, bool TB>
__global__ __launch_bounds__(512, 1) void gemm_p32_kernel(KernelArgs ka) {
  constexpr int BK = kP32BK, NST = 4;
  constexpr bool AKC = !TA, BKC = TB;
  using HA = P32Half<AKC>;
  using HB = P32Half<BKC>;
  constexpr int HALF = HA::FLOATS;
  constexpr int STAGE = 4 * HALF;   // A0 A1 B0 B1 = 32 KB
  __shared__ __attribute__((aligned(1024))) float smem[NST * STAGE];   // 128 KB, the only LDS object
  typedef __attribute__((address_space(3))) void* lds_ptr;
  auto bar = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const GemmDesc& d = ka.d;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, grp = wave >> 2, wc = wave & 3;
  // stream-K: this workgroup's run of K-tile iterations, walked tile by tile (segments)
  const bool sk = ka.sk_wgs > 0;
  int64_t sk_it = 0, sk_end = 0;
  const int64_t sk_total = (int64_t)ka.tiles * ka.sk_ki;
  if (sk) {
    int lin = blockIdx.x;
    if (ka.remap) {   // the XCD remap of map_tile: neighbouring runs (tiles) on one XCD
      const int b = blockIdx.x, xcd = b & 7, q = ka.nblk >> 3, r = ka.nblk & 7;
      lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    }
    sk_it = sk_begin(lin, sk_total, ka.sk_wgs);
    sk_end = sk_begin(lin + 1, sk_total, ka.sk_wgs);
  }
  for (bool first_seg = true;; first_seg = false) {
  int split = 0, tm, tn;
  int64_t kb0, ke;
  float* seg_slab = nullptr;
  if (sk) {
    if (sk_it >= sk_end) break;
    const int t = (int)(sk_it / ka.sk_ki);
    const int64_t t0 = (int64_t)t * ka.sk_ki, kt_end = min((int64_t)ka.sk_ki, sk_end - t0);
    kb0 = (sk_it - t0) * BK;
    ke = min(d.K, kt_end * BK);
    tile_of(t, ka.tiles_m, ka.tiles_n, ka.group_m, tm, tn);
    const int w0 = sk_owner(t0, sk_total, ka.sk_wgs), w1 = sk_owner(t0 + ka.sk_ki - 1, sk_total, ka.sk_wgs);
    const int wme = sk_owner(sk_it, sk_total, ka.sk_wgs);
    if (w1 > w0) seg_slab = ka.sk_slab + (int64_t)(wme - w0) * d.M * d.N;   // a partial tile
    sk_it = t0 + ka.sk_ki;
    if (!first_seg) __syncthreads();   // the previous segment's epilogue is done with the LDS ring
  } else {
    if (!first_seg) break;
    map_tile(ka.nblk, ka.tiles, ka.tiles_m, ka.tiles_n, ka.group_m, ka.remap != 0, split, tm, tn);
    kb0 = split * ka.kchunk;
    ke = (kb0 + ka.kchunk < d.K) ? kb0 + ka.kchunk : d.K;
  }
  const int64_t m0 = (int64_t)tm * 256, n0 = (int64_t)tn * 256;
  const int nk = ke > kb0 ? (int)((ke - kb0 + BK - 1) / BK) : 0;

  typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
  auto rsrc32 = [](const float* p) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    return u32x4s{(unsigned)__builtin_amdgcn_readfirstlane((unsigned)a),
                  (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)), 0x7ffffff0u, 0x00020000u};
  };
  const int64_t z = blockIdx.y;   // batch index (grid.y = batch)
  const u32x4s rsA = rsrc32(d.A + z * d.sA), rsB = rsrc32(d.B + z * d.sB);
  constexpr unsigned kOOB = 0x80000000u;
  unsigned vo[4];
  int kk[4];
  bool rok[4];
  P32Half<AKC>::src(wave, lane, m0, d.M, d.lda, vo[0], kk[0], rok[0]);
  P32Half<AKC>::src(wave, lane, m0 + 128, d.M, d.lda, vo[1], kk[1], rok[1]);
  P32Half<BKC>::src(wave, lane, n0, d.N, d.ldb, vo[2], kk[2], rok[2]);
  P32Half<BKC>::src(wave, lane, n0 + 128, d.N, d.ldb, vo[3], kk[3], rok[3]);
  const int64_t ksA = P32Half<AKC>::kstep_bytes(d.lda), ksB = P32Half<BKC>::kstep_bytes(d.ldb);
  const unsigned lds0 =
      (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ptr)smem + (unsigned)wave * 1024u);
  auto dma = [&](int t, int h) {   // K-tile t, half image h (0, 1: A rows; 2, 3: B columns)
    const int64_t k0 = kb0 + (int64_t)t * BK;
    const bool full = k0 + BK <= ke;
    const unsigned v = (rok[h] && (full || k0 + kk[h] < ke)) ? vo[h] : kOOB;
    const unsigned soff = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(k0 * (h < 2 ? ksA : ksB)));
    const unsigned ldsa = lds0 + (unsigned)(((t % NST) * STAGE + h * HALF) * 4);
    unsigned keep;
    if (h < 2)
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(v), "s"(rsA), "s"(ldsa), "s"(soff)
                   : "memory");
    else
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(v), "s"(rsB), "s"(ldsa), "s"(soff)
                   : "memory");
  };
  auto dma_a = [&](int t) { dma(t, 0); dma(t, 1); };
  auto dma_b = [&](int t) { dma(t, 2); dma(t, 3); };
  auto retire_keep = [](int tiles_in_flight) {   // retire all but the youngest tiles (4 DMAs each)
    if (tiles_in_flight >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (tiles_in_flight == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const bool do_rs = d.rowsum != nullptr && tn == 0 && wc == 0;   // one wave per 128 rows
  float rs[4] = {0.f, 0.f, 0.f, 0.f};

  for (int t = 0; t < NST - 1; ++t)
    if (t < nk) {
      dma_a(t);
      dma_b(t);
    }
  retire_keep(min(nk - 1, NST - 2));
  bar();
  if (grp == 1) bar();

  const int bh = wc >> 1, bc0 = (wc & 1) * 64;
  for (int kt = 0; kt < nk; ++kt) {
    const float* S = smem + (kt % NST) * STAGE;
    const float* As = S + grp * HALF;
    const float* Bs = S + (2 + bh) * HALF;
    const int tn_ = kt + NST - 1;
#pragma unroll
    for (int q = 0; q < BK / 8; ++q) {
      v4f fa[4], fb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = HA::frag(As, i * 32, q, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = HB::frag(Bs, bc0 + j * 32, q, lane);
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
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][ss], fb[j][ss], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (do_rs) {
#pragma unroll
        for (int i = 0; i < 4; ++i) rs[i] += (fa[i][0] + fa[i][1]) + (fa[i][2] + fa[i][3]);
      }
      bar();
    }
  }
  if (grp == 0) bar();

  pp_epilogue(ka, acc, smem, split, m0, n0, grp, wc, wave, lane, z, seg_slab);
  if (do_rs) {   // lanes l and l + 32 hold the two k halves of row (l & 31) of each row block
    const int splits = ka.nblk / ka.tiles;
    float* rsum = d.rowsum + z * d.sRS;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float t = rs[i] + __shfl_xor(rs[i], 32);
      const int64_t row = m0 + grp * 128 + i * 32 + (lane & 31);
      if (lane < 32 && row < d.M) {
        if (ka.partial) ka.rs_partial[(z * splits + split) * d.M + row] = t;
        else rsum[row] = d.rowsum_beta != 0.f ? d.rowsum_beta * rsum[row] + t : t;
      }
    }
  }
  }   // segments
}

// Stream-K fixup: a tile covered by several runs = the sum of its partial slabs in run order, then
// alpha / bias / beta (the splitk_reduce epilogue).  kSkFixupSlices workgroups per tile, each 256 / that
// rows, every thread's (row, column quad) items loaded together (all slab loads in flight before the
// in-order adds: one workgroup per tile read at ~1.8 TB/s, r06); whole tiles return.
constexpr int kSkFixupSlices = 8;
__global__ __launch_bounds__(256) void sk_fixup_kernel(KernelArgs ka) {
  const GemmDesc& d = ka.d;
  const int t = blockIdx.x / kSkFixupSlices, slice = blockIdx.x - t * kSkFixupSlices;
  const int64_t total = (int64_t)ka.tiles * ka.sk_ki, t0 = (int64_t)t * ka.sk_ki;
  const int w0 = sk_owner(t0, total, ka.sk_wgs), w1 = sk_owner(t0 + ka.sk_ki - 1, total, ka.sk_wgs);
  if (w1 == w0) return;
  int tm, tn;
  tile_of(t, ka.tiles_m, ka.tiles_n, ka.group_m, tm, tn);
  const int nseg = w1 - w0 + 1;   // <= 3 (launch_p32: tiles >= W / 2)
  const int64_t MN = d.M * d.N;
  const bool vec = d.N % 4 == 0 && d.ldc % 4 == 0 && (uintptr_t)d.C % 16 == 0 && (uintptr_t)ka.sk_slab % 16 == 0 &&
                   (d.bias_mode != 1 || (uintptr_t)d.bias % 16 == 0);
  constexpr int ROWS = 256 / kSkFixupSlices, ITEMS = ROWS * 64 / 256;   // per thread
  const int64_t r0 = (int64_t)tm * 256 + slice * ROWS;
  if (vec) {
    v4f v[ITEMS];
    int64_t off[ITEMS];
    bool ok[ITEMS];
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {   // (row, column quad) of the slice
      const int i = threadIdx.x + 256 * u;
      const int64_t row = r0 + (i >> 6), col = (int64_t)tn * 256 + (i & 63) * 4;
      ok[u] = row < d.M && col < d.N;   // col + 3 < N (N % 4 == 0)
      off[u] = ok[u] ? row * d.N + col : 0;
      v[u] = *reinterpret_cast<const v4f*>(ka.sk_slab + off[u]);
    }
    v4f v1[ITEMS], v2[ITEMS];
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) v1[u] = *reinterpret_cast<const v4f*>(ka.sk_slab + MN + off[u]);
    if (nseg > 2) {
#pragma unroll
      for (int u = 0; u < ITEMS; ++u) v2[u] = *reinterpret_cast<const v4f*>(ka.sk_slab + 2 * MN + off[u]);
    }
#pragma unroll
    for (int u = 0; u < ITEMS; ++u) {
      if (!ok[u]) continue;
      v4f x = v[u] + v1[u];
      if (nseg > 2) x += v2[u];
      const int i = threadIdx.x + 256 * u;
      const int64_t row = r0 + (i >> 6), col = (int64_t)tn * 256 + (i & 63) * 4;
      x *= d.alpha;
      if (d.bias_mode == 1) x += *reinterpret_cast<const v4f*>(d.bias + col);
      else if (d.bias_mode == 2) x += d.bias[row];
      float* c = d.C + row * d.ldc + col;
      if (d.beta != 0.f) x += d.beta * *reinterpret_cast<const v4f*>(c);
      *reinterpret_cast<v4f*>(c) = x;
    }
    return;
  }
  for (int i = threadIdx.x; i < ROWS * 64; i += 256) {
    const int64_t row = r0 + (i >> 6), col = (int64_t)tn * 256 + (i & 63) * 4;
    if (row >= d.M || col >= d.N) continue;
    const int64_t o = row * d.N + col;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (col + e >= d.N) break;
      float v = 0.f;
      for (int g = 0; g < nseg; ++g) v += ka.sk_slab[g * MN + o + e];
      v *= d.alpha;
      if (d.bias_mode == 1) v += d.bias[col + e];
      else if (d.bias_mode == 2) v += d.bias[row];
      float* c = d.C + row * d.ldc + col + e;
      if (d.beta != 0.f) v += d.beta * *c;
      *c = v;
    }
  }
}

// Sums the split-K slabs in split order and applies the GEMM epilogue.
// Batched launches (grid.y = batch): batch z reads its own [splits][M][N] slabs and writes C + z sC.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmDesc d, const float* __restrict__ partial, int splits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.M * d.N) return;
  partial += (int64_t)blockIdx.y * splits * d.M * d.N;
  d.C += (int64_t)blockIdx.y * d.sC;
  const int64_t row = i / d.N, col = i % d.N;
  float s = 0.f;
#pragma unroll 8   // loads ahead of the in-order adds
  for (int k = 0; k < splits; ++k) s += partial[(int64_t)k * d.M * d.N + i];
  float v = d.alpha * s;
  if (d.bias_mode == 1) v += d.bias[col];
  else if (d.bias_mode == 2) v += d.bias[row];
  float* c = d.C + row * d.ldc + col;
  if (d.beta != 0.f) v += d.beta * *c;
  *c = v;
}

// The same with 4 consecutive columns per thread (N % 4 == 0, ldc % 4 == 0, 16-B aligned C): 16-B
// slab loads and one 16-B store per thread.
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(GemmDesc d, const float* __restrict__ partial, int splits) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n4 = d.N >> 2;
  if (q >= d.M * n4) return;
  const int64_t row = q / n4, col = (q - row * n4) * 4, i = row * d.N + col;
  const int64_t slab = d.M * d.N;
  partial += (int64_t)blockIdx.y * splits * slab;
  d.C += (int64_t)blockIdx.y * d.sC;
  v4f s = *reinterpret_cast<const v4f*>(partial + i);
#pragma unroll 8   // loads ahead of the in-order adds
  for (int k = 1; k < splits; ++k) s += *reinterpret_cast<const v4f*>(partial + (int64_t)k * slab + i);
  v4f v = d.alpha * s;
  if (d.bias_mode == 1) v += *reinterpret_cast<const v4f*>(d.bias + col);
  else if (d.bias_mode == 2) v += d.bias[row];
  v4f* c = reinterpret_cast<v4f*>(d.C + row * d.ldc + col);
  if (d.beta != 0.f) v += d.beta * *c;
  *c = v;
}

// grid.y = batch: batch z reads rp + z splits M and writes out + z out_stride
__global__ void rowsum_reduce_kernel(float* __restrict__ out, float beta, const float* __restrict__ rp, int64_t M,
                                     int splits, int64_t out_stride = 0) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  rp += (int64_t)blockIdx.y * splits * M;
  out += (int64_t)blockIdx.y * out_stride;
  float t = 0.f;
#pragma unroll 8   // loads ahead of the in-order adds (not one dependent load latency per split)
  for (int k = 0; k < splits; ++k) t += rp[(int64_t)k * M + m];
  out[m] = beta != 0.f ? beta * out[m] + t : t;
}

// ------------------------------------------------------------------ column sums (rows split)
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, int64_t M, int64_t N, int64_t ldx,
                                                     float* __restrict__ out, float beta, int64_t rows_per,
                                                     float* __restrict__ part_out) {
  __shared__ float part[4][64];
  const int c = threadIdx.x & 63, rp = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 64 + c;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = r0 + rows_per < M ? r0 + rows_per : M;
  float s = 0.f;
  if (col < N)
    for (int64_t m = r0 + rp; m < r1; m += 4) s += X[m * ldx + col];
  part[rp][c] = s;
  __syncthreads();
  if (rp == 0 && col < N) {
    const float t = (part[0][c] + part[1][c]) + (part[2][c] + part[3][c]);
    if (part_out) part_out[(int64_t)blockIdx.y * N + col] = t;
    else out[col] = beta != 0.f ? beta * out[col] + t : t;
  }
}

// ------------------------------------------------------------------ scratch (split-K slabs)
struct Scratch {
  float* p = nullptr;
  size_t floats = 0;
};
Scratch g_scratch[64];
std::mutex g_scratch_mu;

int get_scratch(size_t floats, float** out) {
  int dev = 0;
  SRK_CHECK_HIP(hipGetDevice(&dev));
  SRK_REQUIRE(dev >= 0 && dev < 64, SRK_ERR_INVALID, "device out of range");
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  Scratch& s = g_scratch[dev];
  if (s.floats < floats) {   // grow-only: steady state never allocates
    if (s.p) {
      SRK_CHECK_HIP(hipDeviceSynchronize());
      SRK_CHECK_HIP(hipFree(s.p));
      s.p = nullptr;
    }
    const size_t want = floats + floats / 4;
    SRK_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&s.p), want * sizeof(float)));
    g_scratch_gen.fetch_add(1);
    s.floats = want;
  }
  *out = s.p;
  return SRK_OK;
}

// Resident workgroups per CU for the 256-thread, 2 x (BK x BM + BK x BN) fp32 LDS tile kernels.
int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

// Grid, split-K and scratch for one launch of a BM x BN x BK tile kernel with `per_cu` resident
// workgroups per CU; fills ka and returns the split count (tile::choose_splits).
// split_batched: the kernel handles split-K slabs of batched launches ([batch][splits][M][N]; the
// ping-pong kernels); the others split only batch-1 launches.
int plan_launch(const GemmDesc& d, int BM, int BN, int BK, int per_cu, KernelArgs& ka, int* splits_out,
                bool allow_split = true, bool split_batched = false) {
  const int64_t tm = (d.M + BM - 1) / BM, tn = (d.N + BN - 1) / BN;
  SRK_REQUIRE(tm * tn <= (INT32_MAX >> 5) && d.batch <= 65535, SRK_ERR_INVALID, "gemm: grid too large");
  static const int remap = env_int("SRK_GEMM_REMAP", 1);
  const int64_t slots = (int64_t)kCUs * per_cu;
  ka = KernelArgs{};
  ka.d = d;
  ka.tiles_m = (int)tm;
  ka.tiles_n = (int)tn;
  ka.tiles = (int)(tm * tn);
  // tile rows per swizzle group: an XCD runs ~32 x per_cu tiles at once out of a contiguous run of
  // the grouped order (XCD remap), i.e. g rows x (32 per_cu / g) columns of tiles, whose distinct
  // operand panels (g BM + 32 per_cu BN / g rows of K) its 4 MB L2 must hold; g = sqrt(32 per_cu
  // BN / BM) minimises them (256 x 128 tiles: 4, was 8 — 8 A panels of 1 MB re-read per round)
  static const int group_env = env_int("SRK_GROUP_M", 0);   // A/B measurements
  ka.group_m = group_env > 0 ? group_env
                             : std::max(1, (int)std::lround(std::sqrt(32.0 * per_cu * BN / (double)BM)));
  ka.remap = remap;
  // Split K when the output grid leaves resident slots idle and K is long (tile::choose_splits).
  const bool can_split = allow_split && (d.batch == 1 || split_batched);
  int splits = can_split ? choose_splits(tm * tn * d.batch, d.K, BK, slots, 16) : 1;
  static const int splits_env = env_int("SRK_GEMM_SPLITS", 0);   // A/B measurements only
  if (splits_env > 0 && d.batch == 1 && d.K >= (int64_t)splits_env * 4 * BK) splits = splits_env;
  ka.kchunk = splits > 1 ? ((d.K + splits - 1) / splits + BK - 1) / BK * BK : std::max<int64_t>(d.K, 1);
  if (splits > 1) splits = (int)((d.K + ka.kchunk - 1) / ka.kchunk);
  ka.nblk = ka.tiles * splits;
  if (splits > 1) {
    float* scratch = nullptr;
    const size_t need = (size_t)d.batch * splits * (d.M * d.N + (d.rowsum ? d.M : 0));
    if (int rc = get_scratch(need, &scratch)) return rc;
    ka.partial = scratch;
    ka.rs_partial = d.rowsum ? scratch + (size_t)d.batch * splits * d.M * d.N : nullptr;
  }
  *splits_out = splits;
  return SRK_OK;
}

// After a split launch: the deterministic slab reduction (+ epilogue) and the row-sum reduction.
int finish_splits(const GemmDesc& d, const KernelArgs& ka, int splits, hipStream_t s) {
  SRK_CHECK_HIP(hipGetLastError());
  if (splits > 1) {
    const int64_t n = d.M * d.N;
    const bool vec4 = d.N % 4 == 0 && d.ldc % 4 == 0 && (uintptr_t)d.C % 16 == 0 && d.sC % 4 == 0 &&
                      (d.bias_mode != 1 || (uintptr_t)d.bias % 16 == 0);
    if (vec4)
      hipLaunchKernelGGL(splitk_reduce4_kernel, dim3((unsigned)((n / 4 + 255) / 256), (unsigned)d.batch), dim3(256), 0,
                         s, d, ka.partial, splits);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)d.batch), dim3(256), 0, s, d,
                         ka.partial, splits);
    if (d.rowsum)
      hipLaunchKernelGGL(rowsum_reduce_kernel, dim3((unsigned)((d.M + 255) / 256), (unsigned)d.batch), dim3(256), 0, s,
                         d.rowsum, d.rowsum_beta, ka.rs_partial, d.M, splits, d.sRS);
    SRK_CHECK_HIP(hipGetLastError());
  }
  return SRK_OK;
}

template <bool TA, bool TB, int BM, int BN, int BK>
int launch(const GemmDesc& d, hipStream_t s, bool vec) {
  constexpr int lds = 2 * 4 * (Img<!TA, BM, BK>::FLOATS + Img<TB, BN, BK>::FLOATS);
  constexpr int per_cu0 = (160 * 1024) / lds < 8 ? (160 * 1024) / lds : 8;
  constexpr int per_cu = per_cu0 > 0 ? per_cu0 : 1;
  KernelArgs ka;
  int splits = 1;
  if (int rc = plan_launch(d, BM, BN, BK, per_cu, ka, &splits)) return rc;
  ProfScope prof("gemm_f32", s, 2.0 * (double)d.M * (double)d.N * (double)d.K * d.batch);
  prof.bytes(gemm_bytes(d, 4));
  // 8 waves (4 per SIMD at 2 workgroups / CU) cover the k-tile staging + barrier phases better
  // (measured: weight-gradient GEMMs +4..17 %); the x W^T projection shape keeps 4.
  static const int waves_env = env_int("SRK_GEMM_WAVES", 0);
  const int waves = BM == 256 ? 8 : (waves_env ? waves_env : ((!TA && TB) ? 4 : 8));
  prof.detail("gemm_f32_kernel<%c%c,%dx%d,%dw> %lldx%lldx%lld b%lld s%d", TA ? 'T' : 'N', TB ? 'T' : 'N', BM, BN, waves,
              (long long)d.M, (long long)d.N, (long long)d.K, (long long)d.batch, splits);
  const dim3 grid((unsigned)ka.nblk, 1, (unsigned)d.batch);
  // LDS-DMA staging (global_load_lds_dwordx4) whenever the 16-B vector conditions hold
  static const int glds_env = env_int("SRK_GEMM_GLDS", 1);
  const bool gl = vec && glds_env != 0;
  bool done = false;
  if constexpr (BN >= 128) {
    if (waves == 8) {
      if (gl) hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, BM, BN, BK, true, 8, true>), grid, dim3(512), 0, s, ka);
      else if (vec) hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, BM, BN, BK, true, 8>), grid, dim3(512), 0, s, ka);
      else hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, BM, BN, BK, false, 8>), grid, dim3(512), 0, s, ka);
      done = true;
    }
  }
  if constexpr (BM != 256) {
    if (!done) {
      if (gl) hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, BM, BN, BK, true, 4, true>), grid, dim3(256), 0, s, ka);
      else if (vec) hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, BM, BN, BK, true, 4>), grid, dim3(256), 0, s, ka);
      else hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, BM, BN, BK, false, 4>), grid, dim3(256), 0, s, ka);
    }
  }
  return finish_splits(d, ka, splits, s);
}

template <bool TA, bool TB, int BM, int BN, int NW, int PF>
int launch_lp_cfg(const GemmDesc& d, hipStream_t s, bool vec, bool f16) {
  constexpr int per_cu = lp_per_cu<BM, BN>();
  // buffer-instruction byte offsets are 32-bit: VEC also needs both operands' extents < 2^31 B
  const double ext_a = (double)(d.ta ? d.K : d.M) * d.lda * 4, ext_b = (double)(d.tb ? d.N : d.K) * d.ldb * 4;
  if (ext_a >= 2147483648.0 || ext_b >= 2147483648.0 || d.batch != 1) vec = false;
  KernelArgs ka;
  int splits = 1;
  if (int rc = plan_launch(d, BM, BN, kLpBK, per_cu, ka, &splits)) return rc;
  ProfScope prof(f16 ? "gemm_f16" : "gemm_bf16", s, 2.0 * (double)d.M * (double)d.N * (double)d.K * d.batch);
  prof.bytes(gemm_bytes(d, 4));   // fp32 operands in HBM, rounded on chip
  prof.detail("gemm_lp_kernel<%c%c,%dx%d> %lldx%lldx%lld s%d", TA ? 'T' : 'N', TB ? 'T' : 'N', BM, BN, (long long)d.M,
              (long long)d.N, (long long)d.K, splits);
  const dim3 grid((unsigned)ka.nblk, 1, (unsigned)d.batch), block(NW * 64);
  if (f16) {
    if (vec) hipLaunchKernelGGL((gemm_lp_kernel<TA, TB, BM, BN, NW, true, true, PF>), grid, block, 0, s, ka);
    else hipLaunchKernelGGL((gemm_lp_kernel<TA, TB, BM, BN, NW, false, true, PF>), grid, block, 0, s, ka);
  } else {
    if (vec) hipLaunchKernelGGL((gemm_lp_kernel<TA, TB, BM, BN, NW, true, false, PF>), grid, block, 0, s, ka);
    else hipLaunchKernelGGL((gemm_lp_kernel<TA, TB, BM, BN, NW, false, false, PF>), grid, block, 0, s, ka);
  }
  return finish_splits(d, ka, splits, s);
}

// Tile configuration of the bf16 / fp16 GEMM (SRK_LP_CFG overrides the choice for A/B measurements):
//   1: 128 x 128, 4 waves, 1 k-tile of register prefetch (2 workgroups / CU)
//   2: 128 x 128, 4 waves, 2 k-tiles in flight
//   3: 256 x 128, 8 waves (4 x 2, 64 x 64 each), 1 k-tile (1 workgroup / CU)
//   4: 256 x 128, 8 waves, 2 k-tiles in flight
//   5: 128 x 128, 8 waves (2 x 4, 64 x 32 each), 2 k-tiles in flight
template <bool TA, bool TB>
int launch_lp(const GemmDesc& d, hipStream_t s, bool vec, bool f16) {
  static const int cfg_env = env_int("SRK_LP_CFG", 0);
  int cfg = cfg_env;
  // measured (profiles/r01zf_gemm_bench_bf16_cfg*.txt): 256 x 128 tiles win whenever an operand is
  // row-contiguous (dx, dW: 12-25 %), the 128 x 128 tile on the x W^T projection (both k-contiguous)
  if (!cfg) cfg = (d.M >= 1024 && !(!TA && TB)) ? 3 : 1;
  switch (cfg) {
    case 2: return launch_lp_cfg<TA, TB, 128, 128, 4, 2>(d, s, vec, f16);
    case 3: return launch_lp_cfg<TA, TB, 256, 128, 8, 1>(d, s, vec, f16);
    case 4: return launch_lp_cfg<TA, TB, 256, 128, 8, 2>(d, s, vec, f16);
    case 5: return launch_lp_cfg<TA, TB, 128, 128, 8, 2>(d, s, vec, f16);
    default: return launch_lp_cfg<TA, TB, 128, 128, 4, 1>(d, s, vec, f16);
  }
}

template <bool TA, bool TB, int BM, int BN, int NW>
int launch_h16_cfg(const GemmDesc& d, hipStream_t s, bool f16) {
  constexpr int per_cu = h16_per_cu<TA, TB, BM, BN>();
  KernelArgs ka;
  int splits = 1;
  if (int rc = plan_launch(d, BM, BN, kLpBK, per_cu, ka, &splits)) return rc;
  ProfScope prof(f16 ? "gemm_f16" : "gemm_bf16", s, 2.0 * (double)d.M * (double)d.N * (double)d.K);
  prof.bytes(gemm_bytes(d, 2));
  prof.detail("gemm_h16_kernel<%c%c,%dx%d> %lldx%lldx%lld s%d", TA ? 'T' : 'N', TB ? 'T' : 'N', BM, BN, (long long)d.M,
              (long long)d.N, (long long)d.K, splits);
  const dim3 grid((unsigned)ka.nblk), block(NW * 64);
  if (f16) hipLaunchKernelGGL((gemm_h16_kernel<TA, TB, BM, BN, NW, true>), grid, block, 0, s, ka);
  else hipLaunchKernelGGL((gemm_h16_kernel<TA, TB, BM, BN, NW, false>), grid, block, 0, s, ka);
  return finish_splits(d, ka, splits, s);
}

template <bool TA, bool TB>
int launch_g16(const GemmDesc& d, hipStream_t s, bool f16) {
  KernelArgs ka;
  int splits = 1;
  // split K only when the 256 x 256 output grid leaves more than half of the CUs idle: the slabs
  // (M x N fp32 per split, written and re-read) cost more than a partly filled round otherwise
  const int64_t tiles = ((d.M + 255) / 256) * ((d.N + 255) / 256) * d.batch;
  if (int rc = plan_launch(d, 256, 256, kG16BK, 1, ka, &splits, tiles * 2 < kCUs, true)) return rc;
  ProfScope prof(f16 ? "gemm_f16" : "gemm_bf16", s, 2.0 * (double)d.M * (double)d.N * (double)d.K * d.batch);
  prof.bytes(gemm_bytes(d, 2));
  prof.detail("gemm_g16_kernel<%c%c> %lldx%lldx%lld b%d s%d", TA ? 'T' : 'N', TB ? 'T' : 'N', (long long)d.M,
              (long long)d.N, (long long)d.K, d.batch, splits);
  const dim3 grid((unsigned)ka.nblk, (unsigned)d.batch), block(512);
  if (f16) hipLaunchKernelGGL((gemm_g16_kernel<TA, TB, true>), grid, block, 0, s, ka);
  else hipLaunchKernelGGL((gemm_g16_kernel<TA, TB, false>), grid, block, 0, s, ka);
  return finish_splits(d, ka, splits, s);
}

template <bool TA, bool TB>
int launch_h16(const GemmDesc& d, hipStream_t s, bool f16) {
  static const int cfg_env = env_int("SRK_H16_CFG", 0);
  // the LDS-DMA ping-pong kernel wherever its 256 x 256 tile fills the chip (srk option overrides)
  const int kern = g_opt_gemm16_kernel ? g_opt_gemm16_kernel : (d.M >= 1024 && d.N >= 256 ? 2 : 1);
  if (kern == 2 || cfg_env == 5 || d.batch > 1) return launch_g16<TA, TB>(d, s, f16);   // only g16 is batched
  // measured (profiles/r01zk_gemm_h16_cfg*.txt): 256 x 256 on x W^T and on the weight gradients
  // (TA != TB: gi 143 vs 148 us, dW_ih 128 vs 137), 256 x 128 on dx (204 tiles of 256 x 256 leave
  // CUs idle: 255 vs 147 us), 128 x 128 below 1024 rows
  const int cfg = cfg_env ? cfg_env : d.M < 1024 ? 1 : (TA != TB && d.N >= 256) ? 4 : 3;
  if (cfg == 3) return launch_h16_cfg<TA, TB, 256, 128, 8>(d, s, f16);
  if (cfg == 4) return launch_h16_cfg<TA, TB, 256, 256, 8>(d, s, f16);
  return launch_h16_cfg<TA, TB, 128, 128, 4>(d, s, f16);
}

template <bool TA, bool TB>
int launch_p32(const GemmDesc& d, hipStream_t s) {
  KernelArgs ka;
  int splits = 1;
  const int64_t tiles = ((d.M + 255) / 256) * ((d.N + 255) / 256) * d.batch;
  const int64_t ki = (d.K + kP32BK - 1) / kP32BK;
  // stream-K where one round of 256 x 256 tiles leaves CUs idle but covers at least half of them
  // (dx of the BiGRU layers: 204 tiles on 256 CUs), K long enough to split
  const bool streamk = g_opt_gemm_streamk && d.batch == 1 && !d.rowsum && tiles < kCUs && tiles * 2 >= kCUs && ki >= 32;
  if (int rc = plan_launch(d, 256, 256, kP32BK, 1, ka, &splits, !streamk && tiles * 2 < kCUs, true)) return rc;
  if (streamk) {
    ka.sk_wgs = kCUs;
    ka.sk_ki = (int)ki;
    ka.nblk = kCUs;
    if (int rc = get_scratch((size_t)3 * d.M * d.N, &ka.sk_slab)) return rc;   // <= 3 runs per tile (tiles >= W / 2)
  }
  ProfScope prof("gemm_f32", s, 2.0 * (double)d.M * (double)d.N * (double)d.K * d.batch);
  prof.bytes(gemm_bytes(d, 4));
  prof.detail("gemm_p32_kernel<%c%c> %lldx%lldx%lld b%d s%d%s", TA ? 'T' : 'N', TB ? 'T' : 'N', (long long)d.M,
              (long long)d.N, (long long)d.K, d.batch, splits, streamk ? " streamk" : "");
  hipLaunchKernelGGL((gemm_p32_kernel<TA, TB>), dim3((unsigned)ka.nblk, (unsigned)d.batch), dim3(512), 0, s, ka);
  if (streamk) hipLaunchKernelGGL(sk_fixup_kernel, dim3((unsigned)ka.tiles * kSkFixupSlices), dim3(256), 0, s, ka);
  return finish_splits(d, ka, splits, s);
}

template <bool TA, bool TB>
int dispatch_tile(const GemmDesc& d, hipStream_t s, bool vec) {
  const int prec = d.prec >= 0 ? d.prec : matmul_prec();
  if (prec != kPrecF32) return launch_lp<TA, TB>(d, s, vec, prec == kPrecF16);
  // the LDS-DMA ping-pong kernel where a 256 x 256 grid fills the chip (16-B units, 32-bit buffer
  // offsets, batch 1); srk option gemm32_kernel: 1 register-staged, 2 ping-pong
  const double ext_a = (double)(d.ta ? d.K : d.M) * d.lda * 4, ext_b = (double)(d.tb ? d.N : d.K) * d.ldb * 4;
  const bool p32_ok = vec && ext_a < 2147483000.0 && ext_b < 2147483000.0;
  // measured (tools/gemm_bench.py, cfg2 shapes): ping-pong 6-7 % faster on dx (NN) and dW_ih (TN),
  // 8 % slower on the x W^T projection (NT) and on the 12-tile dW_hh grid (split 16); batched
  // launches (the BiGRU's two dW_hh) and row sums over a batch only exist on the ping-pong kernel
  const int kern32 = g_opt_gemm32_kernel ? g_opt_gemm32_kernel
                                         : (!TB && ((d.M >= 2048 && d.N >= 1024) || d.batch > 1) ? 2 : 1);
  SRK_REQUIRE(!d.rowsum || d.batch == 1 || (p32_ok && kern32 == 2), SRK_ERR_INVALID,
              "gemm: batched row sums need the fp32 ping-pong kernel (16-B operand rows)");
  if (p32_ok && kern32 == 2) return launch_p32<TA, TB>(d, s);
  // 256 x 128 tiles (one 8-wave workgroup per CU, 110 KB of LDS) halve the L2 -> CU operand
  // traffic per flop of the 128 x 128 tile; used when the grid still fills the chip several times
  static const int tile_env = env_int("SRK_GEMM_TILE", 0);
  const int64_t t256 = ((d.M + 255) / 256) * ((d.N + 127) / 128) * d.batch;
  const bool big = tile_env ? tile_env == 256 : (d.M >= 2048 && d.N >= 128 && d.K >= 256 && (t256 >= 512 || d.K >= 4096));
  if (big) return launch<TA, TB, 256, 128, 32>(d, s, vec);
  const int64_t big_tiles = ((d.M + 127) / 128) * ((d.N + 127) / 128) * d.batch;
  if (d.M > 64 && d.N > 64 && (big_tiles >= 64 || d.K >= 2048)) return launch<TA, TB, 128, 128, 32>(d, s, vec);
  return launch<TA, TB, 64, 64, 32>(d, s, vec);
}

}  // namespace

bool gemm_f32_batched_rowsum_ok(const GemmDesc& d) {
  // mirrors gemm_f32 -> dispatch_tile: batched row sums exist only on the fp32-operand ping-pong
  // kernel (fp32 precision, 16-B operand rows, 32-bit buffer extents, not overridden to kernel 1)
  const int prec = d.prec >= 0 ? d.prec : matmul_prec();
  if (prec != kPrecF32 || d.A16 || d.B16 || d.tb || g_opt_gemm32_kernel == 1) return false;
  const bool kc_operand = !d.ta || d.tb;
  const bool vec = (d.lda % 4 == 0) && ((uintptr_t)d.A % 16 == 0) && (d.sA % 4 == 0) && (d.ldb % 4 == 0) &&
                   ((uintptr_t)d.B % 16 == 0) && (d.sB % 4 == 0) && (!kc_operand || d.K % 4 == 0) &&
                   (!d.ta || d.M % 4 == 0) && (d.tb || d.N % 4 == 0);
  const double ext_a = (double)(d.ta ? d.K : d.M) * d.lda * 4, ext_b = (double)(d.tb ? d.N : d.K) * d.ldb * 4;
  // a batched launch spans batch - 1 strides past the first operand
  const double span_a = ext_a + (double)(d.batch - 1) * d.sA * 4, span_b = ext_b + (double)(d.batch - 1) * d.sB * 4;
  return vec && span_a < 2147483000.0 && span_b < 2147483000.0;
}

int gemm_f32(const GemmDesc& d, hipStream_t s) {
  SRK_REQUIRE(d.M >= 0 && d.N >= 0 && d.K >= 0 && d.batch >= 1, SRK_ERR_INVALID, "gemm: bad shape");
  if (d.M == 0 || d.N == 0) return SRK_OK;
  if (d.A16 || d.B16) {   // 16-bit operands in memory
    const int prec = d.prec >= 0 ? d.prec : matmul_prec();
    SRK_REQUIRE(d.A16 && d.B16 && d.C && prec != kPrecF32 && !d.rowsum && (d.batch == 1 || d.bias_mode == 0),
                SRK_ERR_INVALID,
                "gemm: 16-bit operands need both A16 / B16, a 16-bit precision and no row sums (no bias when batched)");
    SRK_REQUIRE(d.batch == 1 || (d.sA % 8 == 0 && d.sB % 8 == 0 && d.sC % 4 == 0), SRK_ERR_INVALID,
                "gemm: batched 16-bit operands need 8-element strides");
    const double ext_a = (double)(d.ta ? d.K : d.M) * d.lda * 2, ext_b = (double)(d.tb ? d.N : d.K) * d.ldb * 2;
    SRK_REQUIRE((uintptr_t)d.A16 % 16 == 0 && (uintptr_t)d.B16 % 16 == 0 && d.lda % 8 == 0 && d.ldb % 8 == 0 &&
                    ((d.ta && d.M % 8 == 0) || (!d.ta && d.K % 8 == 0)) &&
                    ((d.tb && d.K % 8 == 0) || (!d.tb && d.N % 8 == 0)) && ext_a < 2147483648.0 &&
                    ext_b < 2147483648.0,
                SRK_ERR_INVALID, "gemm: 16-bit operands need 16-B aligned rows of 8-element multiples");
    SRK_REQUIRE(d.K > 0, SRK_ERR_INVALID, "gemm: 16-bit operands need K > 0");
    const bool f16 = prec == kPrecF16;
    if (!d.ta && !d.tb) return launch_h16<false, false>(d, s, f16);
    if (!d.ta && d.tb) return launch_h16<false, true>(d, s, f16);
    if (d.ta && !d.tb) return launch_h16<true, false>(d, s, f16);
    return launch_h16<true, true>(d, s, f16);
  }
  SRK_REQUIRE(d.C && (d.K == 0 || (d.A && d.B)), SRK_ERR_INVALID, "gemm: null operand");
  SRK_REQUIRE(d.bias_mode == 0 || d.bias, SRK_ERR_INVALID, "gemm: bias_mode without bias");
  if (const int kind = skinny_kind(d); kind >= 0) {   // one dimension <= 16: VALU kernels
    const int prec = d.prec >= 0 ? d.prec : matmul_prec();
    return prec == kPrecBF16 ? launch_skinny_rnd<1>(d, kind, s)
           : prec == kPrecF16 ? launch_skinny_rnd<2>(d, kind, s) : launch_skinny_rnd<0>(d, kind, s);
  }
  SRK_REQUIRE(!d.rowsum || d.batch == 1 || d.prec == kPrecF32 || (d.prec < 0 && matmul_prec() == kPrecF32),
              SRK_ERR_INVALID, "gemm: batched rowsum needs fp32 operands");
  // 16-B loads need 16-B aligned rows, K % 4 == 0 when an operand is k-contiguous (a clamped k vector
  // stays inside the row) and,
  // along M / N (A when ta, B when !tb), a row count that is a multiple of 4 (a clamped vector is
  // wholly in or wholly out of range).  Otherwise the kernel stages with 4-B loads.
  const bool kc_operand = !d.ta || d.tb;   // some operand is k-contiguous: its vectors run along k
  const bool vec = (d.lda % 4 == 0) && ((uintptr_t)d.A % 16 == 0) && (d.sA % 4 == 0) && (d.ldb % 4 == 0) &&
                   ((uintptr_t)d.B % 16 == 0) && (d.sB % 4 == 0) && (!kc_operand || d.K % 4 == 0) &&
                   (!d.ta || d.M % 4 == 0) && (d.tb || d.N % 4 == 0);
  if (!d.ta && !d.tb) return dispatch_tile<false, false>(d, s, vec);
  if (!d.ta && d.tb) return dispatch_tile<false, true>(d, s, vec);
  if (d.ta && !d.tb) return dispatch_tile<true, false>(d, s, vec);
  return dispatch_tile<true, true>(d, s, vec);
}

int colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, float beta, hipStream_t s) {
  if (N == 0) return SRK_OK;
  const int64_t cblocks = (N + 63) / 64;
  // split the rows when there are too few column blocks to fill the chip (>= 32 rows per split)
  int64_t rsplit = 1;
  if (cblocks < 256 && M >= 64) rsplit = std::min<int64_t>((512 + cblocks - 1) / cblocks, (M + 31) / 32);
  if (rsplit <= 1) {
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)cblocks, 1), dim3(256), 0, s, X, M, N, ldx, out, beta, M,
                       (float*)nullptr);
  } else {
    const int64_t rows_per = (M + rsplit - 1) / rsplit;
    float* part = nullptr;
    if (int rc = get_scratch((size_t)rsplit * N, &part)) return rc;
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)cblocks, (unsigned)rsplit), dim3(256), 0, s, X, M, N, ldx, out,
                       beta, rows_per, part);
    hipLaunchKernelGGL(rowsum_reduce_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, out, beta, part, N,
                       (int)rsplit);
  }
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

}  // namespace srk

extern "C" int srk_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                            int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc,
                            const float* bias, int bias_mode, void* stream) {
  SRK_API_BEGIN
  srk::GemmDesc d;
  d.M = M; d.N = N; d.K = K;
  d.A = A; d.lda = lda; d.ta = trans_a != 0;
  d.B = B; d.ldb = ldb; d.tb = trans_b != 0;
  d.C = C; d.ldc = ldc; d.alpha = alpha; d.beta = beta;
  d.bias = bias; d.bias_mode = bias_mode;
  SRK_REQUIRE(bias_mode >= 0 && bias_mode <= 2, SRK_ERR_INVALID, "gemm: bias_mode must be 0, 1 or 2");
  return srk::gemm_f32(d, srk::as_stream(stream));
  SRK_API_END
}

extern "C" int srk_gemm_rowsum_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha,
                                   const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C,
                                   int64_t ldc, float* rowsum, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(rowsum, SRK_ERR_INVALID, "gemm_rowsum: null rowsum");
  srk::GemmDesc d;
  d.M = M; d.N = N; d.K = K;
  d.A = A; d.lda = lda; d.ta = trans_a != 0;
  d.B = B; d.ldb = ldb; d.tb = trans_b != 0;
  d.C = C; d.ldc = ldc; d.alpha = alpha; d.beta = beta;
  d.rowsum = rowsum; d.rowsum_beta = beta;
  return srk::gemm_f32(d, srk::as_stream(stream));
  SRK_API_END
}

extern "C" int srk_colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, float beta, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(M >= 0 && N >= 0 && (N == 0 || (X && out)), SRK_ERR_INVALID, "colsum: bad args");
  return srk::colsum_f32(X, M, N, ldx, out, beta, srk::as_stream(stream));
  SRK_API_END
}

extern "C" int srk_gemm_16(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha, const uint16_t* A,
                           int64_t lda, const uint16_t* B, int64_t ldb, float beta, float* C, int64_t ldc,
                           const float* bias, int bias_mode, void* stream) {
  SRK_API_BEGIN
  srk::GemmDesc d;
  d.M = M; d.N = N; d.K = K;
  d.A16 = A; d.lda = lda; d.ta = trans_a != 0;
  d.B16 = B; d.ldb = ldb; d.tb = trans_b != 0;
  d.C = C; d.ldc = ldc; d.alpha = alpha; d.beta = beta;
  d.bias = bias; d.bias_mode = bias_mode;
  SRK_REQUIRE(bias_mode >= 0 && bias_mode <= 2, SRK_ERR_INVALID, "gemm: bias_mode must be 0, 1 or 2");
  SRK_REQUIRE(srk::matmul_prec() != srk::kPrecF32, SRK_ERR_INVALID, "gemm_16: set matmul_precision to bf16 / fp16");
  return srk::gemm_f32(d, srk::as_stream(stream));
  SRK_API_END
}

extern "C" int srk_gemm_16_batched(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, float alpha,
                                   const uint16_t* A, int64_t lda, int64_t sA, const uint16_t* B, int64_t ldb,
                                   int64_t sB, float beta, float* C, int64_t ldc, int64_t sC, int batch,
                                   void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(batch >= 1, SRK_ERR_INVALID, "gemm_16_batched: batch must be >= 1");
  srk::GemmDesc d;
  d.M = M; d.N = N; d.K = K;
  d.A16 = A; d.lda = lda; d.ta = trans_a != 0;
  d.B16 = B; d.ldb = ldb; d.tb = trans_b != 0;
  d.C = C; d.ldc = ldc; d.alpha = alpha; d.beta = beta;
  d.batch = batch; d.sA = sA; d.sB = sB; d.sC = sC;
  SRK_REQUIRE(srk::matmul_prec() != srk::kPrecF32, SRK_ERR_INVALID,
              "gemm_16_batched: set matmul_precision to bf16 / fp16");
  return srk::gemm_f32(d, srk::as_stream(stream));
  SRK_API_END
}

namespace srk {
int release_gemm_scratch() {
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  SRK_CHECK_HIP(hipDeviceSynchronize());
  for (Scratch& s : g_scratch) {
    if (s.p) SRK_CHECK_HIP(hipFree(s.p));
    s = Scratch{};
  }
  g_scratch_gen.fetch_add(1);
  return SRK_OK;
}
}  // namespace srk
