// Shared building blocks of the fp32 MFMA tile kernels (gemm.hip, conv.hip): LDS operand images,
// the k-permuted 32x32x2 fragment loop, and the XCD-aware block -> tile map.
//
// A workgroup is 256 threads = 2 x 2 waves; each wave owns (BM/2) x (BN/2) of the output as 32x32
// MFMA tiles (v_mfma_f32_32x32x2_f32: exact fp32 fma chain, 64 FLOP/clk/SIMD).
#pragma once
#include <algorithm>

#include "srk_internal.h"

namespace srk {
namespace tile {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4f ld4(const float* p) { return *reinterpret_cast<const v4f*>(p); }
__device__ __forceinline__ void st4(float* p, v4f v) { *reinterpret_cast<v4f*>(p) = v; }

// LDS images (pitches in floats, all multiples of 4 so every 16-B store is aligned):
//   operand stored k-contiguous in HBM (KC): [row][BK + 4]   (float4 along k)
//   operand stored row-contiguous  (!KC):    [BK][rows + 8]  (float4 along rows)
// MFMA 32x32x2 operand = element (row = lane & 31, k = lane >> 5).  The k order is permuted per
// 8-deep block: sub-step s (0..3) of block kb gives lanes of half h the real k = 8 kb + 4 h + s, the
// same for A and B (any fixed permutation of k is a valid summation order), so a k-contiguous image
// feeds 4 MFMAs from ONE ds_read_b128 per operand, and a row-contiguous image from 4 ds_read_b32 at
// a pitch (rows + 8) that puts the two lane halves on disjoint banks.
template <bool KC, int ROWS, int BK>
struct Img {
  static constexpr int P = KC ? BK + 4 : ROWS + 8;
  static constexpr int FLOATS = KC ? ROWS * P : BK * P;
  __device__ static __forceinline__ v4f frag(const float* s, int row, int kb, int h) {
    if (KC) return ld4(s + row * P + kb * 8 + 4 * h);
    const float* q = s + (kb * 8 + 4 * h) * P + row;
    return v4f{q[0], q[P], q[2 * P], q[3 * P]};
  }
  __device__ static __forceinline__ float elem(const float* s, int row, int k) {
    return KC ? s[row * P + k] : s[k * P + row];
  }
  // element offset of the float4 a staging thread writes (row-major walk of the image's source)
  __device__ static __forceinline__ int store_off(int vi) {
    return KC ? (vi / (BK / 4)) * P + (vi % (BK / 4)) * 4 : (vi / (ROWS / 4)) * P + (vi % (ROWS / 4)) * 4;
  }
};

// Lane-linear LDS images, filled by global_load_lds_dwordx4 (LDS-DMA: a wave-instruction writes
// 1 KB contiguously, lane l at +16 l), so no padding is possible:
//   KC:  [row][BK] with the 16-B quads of each row XOR-swizzled by (row >> 1) & (BK/4 - 1) — the
//        swizzle goes on the GLOBAL source address at load time; a fragment ds_read_b128 of 16 rows
//        then touches 16 distinct bank quads (rows of one parity get distinct quads);
//   !KC: [BK][ROWS] unpadded (each half-wave's ds_read_b32 reads 32 consecutive floats).
template <bool KC, int ROWS, int BK>
struct ImgL {
  static constexpr int P = KC ? BK : ROWS;
  static constexpr int FLOATS = ROWS * BK;
  static constexpr int QMASK = BK / 4 - 1;
  __device__ static __forceinline__ int swz(int row) { return (row >> 1) & QMASK; }
  __device__ static __forceinline__ v4f frag(const float* s, int row, int kb, int h) {
    if (KC) return ld4(s + row * P + (((kb * 2 + h) ^ swz(row)) << 2));
    const float* q = s + (kb * 8 + 4 * h) * P + row;
    return v4f{q[0], q[P], q[2 * P], q[3 * P]};
  }
  __device__ static __forceinline__ float elem(const float* s, int row, int k) {
    return KC ? s[row * P + ((((k >> 2) ^ swz(row))) << 2) + (k & 3)] : s[k * P + row];
  }
};

#ifndef SRK_PIN_PREFETCH
#define SRK_PIN_PREFETCH 1
#endif
constexpr bool kPinPrefetch = SRK_PIN_PREFETCH != 0;

// One BK-deep stage: acc[TM][TN] += A_img[wm0 .. +BM/2][k] * B_img[k][wn0 .. +BN/2], fragments of
// the next 8-deep block are read ahead of this block's MFMAs.
template <class IA, class IB, int TM, int TN, int BK>
__device__ __forceinline__ void mma_stage(const float* As, const float* Bs, f32x16 (&acc)[TM][TN], int wm0, int wn0,
                                          int lane) {
  const int lh = lane >> 5, lc = lane & 31;
  v4f fa[2][TM], fb[2][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) fa[0][i] = IA::frag(As, wm0 + i * 32 + lc, 0, lh);
#pragma unroll
  for (int j = 0; j < TN; ++j) fb[0][j] = IB::frag(Bs, wn0 + j * 32 + lc, 0, lh);
#pragma unroll
  for (int kb = 0; kb < BK / 8; ++kb) {
    const int c = kb & 1;
    if (kb + 1 < BK / 8) {
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[c ^ 1][i] = IA::frag(As, wm0 + i * 32 + lc, kb + 1, lh);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[c ^ 1][j] = IB::frag(Bs, wn0 + j * 32 + lc, kb + 1, lh);
    }
    // pin the prefetch ABOVE this block's MFMAs: left alone, the scheduler sinks the ds_reads
    // below them and the wave then waits on LDS latency with the matrix pipe idle
    if (kPinPrefetch) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[c][i][s], fb[c][j][s], acc[i][j], 0, 0, 0);
  }
}

// Block -> (split, tile_m, tile_n).  Workgroups are dealt round-robin over the 8 XCDs (block b and
// b + 8 share an XCD; speed only, never correctness), so consecutive LOGICAL tiles go to blocks of
// ONE XCD: tiles an XCD runs concurrently share A and B panels in its L2.  Within a split, tiles are
// walked in groups of group_m tile rows (column-major inside a group): resident tiles form a compact
// 2-D patch.
// map_tile_at: the same for a virtual block index b (persistent kernels: b = blockIdx.x + r gridDim.x with a
// grid that is a multiple of 8, so b's XCD is the workgroup's)
__device__ __forceinline__ void map_tile_at(int b, int nblk, int tiles, int tiles_m, int tiles_n, int group_m,
                                            bool remap, int& split, int& tm, int& tn) {
  int lin = b;
  if (remap) {
    const int xcd = b & 7, q = nblk >> 3, r = nblk & 7;
    lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  split = lin / tiles;
  const int t = lin - split * tiles;
  const int gsz_full = group_m * tiles_n;
  const int grp = t / gsz_full, first_m = grp * group_m;
  const int gm = tiles_m - first_m < group_m ? tiles_m - first_m : group_m;
  const int tin = t - grp * gsz_full;
  tm = first_m + tin % gm;
  tn = tin / gm;
}

__device__ __forceinline__ void map_tile(int nblk, int tiles, int tiles_m, int tiles_n, int group_m, bool remap,
                                         int& split, int& tm, int& tn) {
  int lin = blockIdx.x;
  if (remap) {
    const int b = blockIdx.x, xcd = b & 7, q = nblk >> 3, r = nblk & 7;
    lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  split = lin / tiles;
  const int t = lin - split * tiles;
  const int gsz_full = group_m * tiles_n;
  const int grp = t / gsz_full, first_m = grp * group_m;
  const int gm = tiles_m - first_m < group_m ? tiles_m - first_m : group_m;
  const int tin = t - grp * gsz_full;
  tm = first_m + tin % gm;
  tn = tin / gm;
}

// Split-K choice: the split count (<= smax, >= 4 BK-tiles per split) whose last round of
// workgroups is fullest, preferring fewer splits (each split adds an M x N fp32 slab write + read):
// a split must buy >= 10 % more filled resident slots.
inline int choose_splits(int64_t tiles, int64_t K, int BK, int64_t slots, int64_t smax) {
  if (K < 16 * BK) return 1;
  auto eff = [&](int64_t sp) {
    const int64_t w = tiles * sp, rounds = (w + slots - 1) / slots;
    return (double)w / (double)(rounds * slots);
  };
  int splits = 1;
  double best = eff(1);
  smax = std::min<int64_t>(smax, K / (4 * BK));
  for (int64_t sp = 2; sp <= smax; ++sp) {
    const double e = eff(sp);
    if (e > best * 1.10 + 1e-9 && tiles * sp <= 4 * slots) { best = e; splits = (int)sp; }
  }
  return splits;
}

constexpr int kCUs = 256;

}  // namespace tile
}  // namespace srk
