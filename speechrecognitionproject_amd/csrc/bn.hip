// K9: BatchNorm1d (+ optional residual add + ReLU) on channels-last activations [M rows][C]
// (M = N * L), the normalisation layers of models/model_resnet_bgru.py:20-39,49-50 and its
// downsample branches (:67-70).
//
// Training mode uses the batch statistics (biased variance for the normalisation, unbiased for the
// running estimate, momentum 0.1 as nn.BatchNorm1d), computed in ONE pass: per-thread shifted sums
// -> per-chunk (mean, M2) -> Chan's pairwise combination in a fixed order (deterministic, and
// accurate without a second centred pass).  All element kernels move 16 B per lane.
// Eval mode normalises with the running statistics.
//   y = act( (x - mean) * invstd * gamma + beta  [+ residual] ),  act = ReLU or identity
// Backward (training statistics):
//   g = dy * act'(y);  dbeta = sum g;  dgamma = sum g * xhat
//   dx = gamma * invstd / M * (M g - dbeta - xhat * dgamma);  dresidual = g
#include <mutex>

#include "srk_internal.h"

namespace srk {
namespace {

typedef float v4f __attribute__((ext_vector_type(4)));

// Work split: a block = 256 threads = CQ channel quads (4 channels each, 16-B accesses) x RP row
// phases; blockIdx.x walks channel groups of 4*CQ channels, blockIdx.y row chunks.  The chunk count
// is capped (kMaxChunks) so the per-channel finalize reads a short, fixed-order list of partials.
// The reduction kernels keep kUnroll rows' 16-B loads in flight per lane (all issued before any is
// consumed; clamped addresses, masked accumulation in the same row order, so the sums are bitwise
// those of the one-row loop): with one 4-wave block per CU at C = 64 the one-row loop waited out a
// full HBM latency per row.
constexpr int kMaxChunks = 256;
constexpr int kUnroll = 8;

struct BnGeom {
  int C, C4, CQ, RP;   // channels, channel quads, quads per block, row phases per block
  int64_t M, rows_per_chunk;
  int chunks;
};

inline BnGeom bn_geom(int64_t M, int C) {
  BnGeom g;
  g.M = M;
  g.C = C;
  g.C4 = C / 4;
  g.CQ = g.C4 < 64 ? g.C4 : 64;
  g.RP = 256 / g.CQ;
  int64_t rows = (M + kMaxChunks - 1) / kMaxChunks;
  rows = ((rows + g.RP - 1) / g.RP) * g.RP;
  g.rows_per_chunk = rows < g.RP ? g.RP : rows;
  g.chunks = (int)((M + g.rows_per_chunk - 1) / g.rows_per_chunk);
  return g;
}

__device__ __forceinline__ v4f ld4(const float* p) { return *reinterpret_cast<const v4f*>(p); }
__device__ __forceinline__ void st4(float* p, v4f v) { *reinterpret_cast<v4f*>(p) = v; }

// 16-bit copy of an output for the convolution that consumes it next (LP 1 = bf16, 2 = fp16; 0 = none):
// the conversion of conv.hip's to16_kernel (round to nearest even), so the copy is bitwise the one the
// convolution would have made from the fp32 tensor
typedef unsigned u32x2b __attribute__((ext_vector_type(2)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef _Float16 hf4 __attribute__((ext_vector_type(4)));
template <int LP>
__device__ __forceinline__ void st4_16(uint16_t* p, v4f v) {
  if constexpr (LP == 1) *reinterpret_cast<u32x2b*>(p) = __builtin_bit_cast(u32x2b, __builtin_convertvector(v, bf4));
  if constexpr (LP == 2) *reinterpret_cast<u32x2b*>(p) = __builtin_bit_cast(u32x2b, __builtin_convertvector(v, hf4));
}

// Chan et al. pairwise combination of (count, mean, M2) — fixed call order => deterministic.
// The update is spelled out with fmaf (mu = fma(d, nb / nt, mu), m2 += fma(d d, n nb / nt, m2b)), so every
// form that uses it rounds identically whatever the compiler's contraction / vectorisation choices.
__device__ __forceinline__ void chan_step(float n, float& mu, float& m2, float nb, float nt, float mub, float m2b) {
  const float d = mub - mu, r = nb / nt, q = n * nb / nt;
  mu = fmaf(d, r, mu);
  m2 = m2 + fmaf(d * d, q, m2b);
}
__device__ __forceinline__ void chan(float& n, float& mu, float& m2, float nb, float mub, float m2b) {
  if (nb == 0.f) return;
  if (n == 0.f) { n = nb; mu = mub; m2 = m2b; return; }
  const float nt = n + nb;
  chan_step(n, mu, m2, nb, nt, mub, m2b);
  n = nt;
}

// Training statistics, one pass: per thread shifted sums (pivot = the chunk's first row) for its
// 4 channels over its row phase, turned into (n, mean, M2) and combined across row phases in LDS
// (fixed order).  Output per chunk: mean and M2 per channel.
__global__ __launch_bounds__(256) void bn_stats_kernel(const float* __restrict__ x, BnGeom g,
                                                       float* __restrict__ pmean, float* __restrict__ pm2) {
  const int q = threadIdx.x % g.CQ, rp = threadIdx.x / g.CQ;
  const int c4 = blockIdx.x * g.CQ + q;
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_chunk;
  const int64_t r1 = r0 + g.rows_per_chunk < g.M ? r0 + g.rows_per_chunk : g.M;
  __shared__ float sn[256], smu[256][4], sm2[256][4];
  v4f s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
  float n = 0.f;
  v4f piv = {0.f, 0.f, 0.f, 0.f};
  if (c4 < g.C4) {
    piv = ld4(x + r0 * g.C + c4 * 4);
    for (int64_t r = r0 + rp; r < r1; r += kUnroll * g.RP) {
      v4f v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t ru = r + u * g.RP;
        v[u] = ld4(x + (ru < r1 ? ru : r) * g.C + c4 * 4);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (r + u * g.RP < r1) {
          const v4f d = v[u] - piv;
          s1 += d;
          s2 += d * d;
          n += 1.f;
        }
      }
    }
  }
  sn[threadIdx.x] = n;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float m = n > 0.f ? s1[e] / n : 0.f;
    smu[threadIdx.x][e] = piv[e] + m;
    sm2[threadIdx.x][e] = n > 0.f ? s2[e] - s1[e] * m : 0.f;
  }
  __syncthreads();
  if (rp == 0 && c4 < g.C4) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float nn = 0.f, mu = 0.f, m2 = 0.f;
      for (int k = 0; k < g.RP; ++k) chan(nn, mu, m2, sn[k * g.CQ + q], smu[k * g.CQ + q][e], sm2[k * g.CQ + q][e]);
      pmean[(int64_t)blockIdx.y * g.C + c4 * 4 + e] = mu;
      pm2[(int64_t)blockIdx.y * g.C + c4 * 4 + e] = m2;
    }
  }
}

// The reduction kernels below load the partials of kPre chunks before any is combined (an in-order sum
// that no longer waits out one load latency per chunk).
constexpr int kPre = 32;

// Combine the chunk partials of channel c in chunk order (Chan), one lane (srk option bn_tree = 0).
__device__ __forceinline__ void combine_chunks(const float* __restrict__ pmean, const float* __restrict__ pm2,
                                               const BnGeom& g, int c, float& n, float& mu, float& m2) {
  n = 0.f;
  mu = 0.f;
  m2 = 0.f;
  for (int k0 = 0; k0 < g.chunks; k0 += kPre) {
    float vm[kPre], v2[kPre];
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int64_t k = k0 + u < g.chunks ? k0 + u : g.chunks - 1;
      vm[u] = pmean[k * g.C + c];
      v2[u] = pm2[k * g.C + c];
    }
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      if (k0 + u < g.chunks) {
        const int64_t r0 = (int64_t)(k0 + u) * g.rows_per_chunk;
        const float nb = (float)((r0 + g.rows_per_chunk < g.M ? g.rows_per_chunk : g.M - r0));
        chan(n, mu, m2, nb, vm[u], v2[u]);
      }
    }
  }
}

// combine_chunks's arithmetic, bit for bit, without its dependent divides: every chunk has >= 1 row, so
// past chunk 0 (taken as is: chan's n == 0 case) the counts n, nb and the ratios nb / nt, n nb / nt are
// data-independent — computed off the (mu, m2) chain, which keeps only chan_step's subtract / fma / fma / add
// per chunk (chan_step itself, so the same roundings).  The in-order form that bn_finalize runs by
// default (bn_tree = 0): ~54 us per BatchNorm layer with the divides in the chain (r04k cfg4 bf16).
__device__ __forceinline__ void combine_chunks_fast(const float* __restrict__ pmean, const float* __restrict__ pm2,
                                                    const BnGeom& g, int c, float& n, float& mu, float& m2) {
  const float rpc = (float)g.rows_per_chunk;
  const float last = (float)(g.M - (int64_t)(g.chunks - 1) * g.rows_per_chunk);
  n = g.chunks == 1 ? last : rpc;
  mu = pmean[c];
  m2 = pm2[c];
  for (int k0 = 1; k0 < g.chunks; k0 += kPre) {
    float vm[kPre], v2[kPre];
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int64_t k = k0 + u < g.chunks ? k0 + u : g.chunks - 1;
      vm[u] = pmean[k * g.C + c];
      v2[u] = pm2[k * g.C + c];
    }
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      if (k0 + u < g.chunks) {
        const float nb = k0 + u == g.chunks - 1 ? last : rpc;
        const float nt = n + nb;
        chan_step(n, mu, m2, nb, nt, vm[u], v2[u]);
        n = nt;
      }
    }
  }
}

// Combine the chunk partials of channel c (Chan's pairwise formula) as a fixed pairwise tree, one wave
// per channel: lane l combines chunks 4l .. 4l+3 in order (kMaxChunks = 256 = 4 x 64), then the lanes pair up at distance 1, 2, .. 32 (lane l takes lane
// l + d when l % 2d == 0).  Deterministic (the tree does not depend on timing) and shallower: 3 + 6
// dependent Chan steps instead of 256 — the serial chain's dependent divides were ~54 us per BatchNorm
// layer (r04k cfg4 bf16).  The result sits in lane 0.
static_assert(kMaxChunks == 4 * 64, "combine_chunks_tree: four chunks per lane");
__device__ __forceinline__ void combine_chunks_tree(const float* __restrict__ pmean, const float* __restrict__ pm2,
                                                    const BnGeom& g, int c, float& n, float& mu, float& m2) {
  const int lane = threadIdx.x & 63;
  n = 0.f;
  mu = 0.f;
  m2 = 0.f;
  float vm[4], v2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = 4 * lane + u < g.chunks ? 4 * lane + u : g.chunks - 1;
    vm[u] = pmean[(int64_t)k * g.C + c];
    v2[u] = pm2[(int64_t)k * g.C + c];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = 4 * lane + u;
    if (k < g.chunks) {
      const int64_t r0 = (int64_t)k * g.rows_per_chunk;
      chan(n, mu, m2, (float)(r0 + g.rows_per_chunk < g.M ? g.rows_per_chunk : g.M - r0), vm[u], v2[u]);
    }
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float nb = __shfl_down(n, d, 64), mb = __shfl_down(mu, d, 64), m2b = __shfl_down(m2, d, 64);
    if ((lane & (2 * d - 1)) == 0) chan(n, mu, m2, nb, mb, m2b);
  }
}

// Biased variance for the normalisation, unbiased for the running estimate (nn.BatchNorm1d,
// momentum update).  Block = 4 waves = 4 channels (combine_chunks_tree).
// TREE: 0 = in order (combine_chunks_fast), 1 = pairwise tree, 2 = in order with the divides in the chain
// (combine_chunks: the bitwise reference of form 0)
template <int TREE>
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ pmean,
                                                          const float* __restrict__ pm2, BnGeom g, float eps,
                                                          float momentum, float* __restrict__ mean,
                                                          float* __restrict__ invstd, float* __restrict__ running_mean,
                                                          float* __restrict__ running_var) {
  const int c = TREE == 1 ? blockIdx.x * 4 + (threadIdx.x >> 6) : blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= g.C) return;
  float n, mu, m2;
  if (TREE == 1) {
    combine_chunks_tree(pmean, pm2, g, c, n, mu, m2);
    if ((threadIdx.x & 63) != 0) return;
  } else if (TREE == 2) {
    combine_chunks(pmean, pm2, g, c, n, mu, m2);
  } else {
    combine_chunks_fast(pmean, pm2, g, c, n, mu, m2);
  }
  const float var = m2 / (float)g.M;
  mean[c] = mu;
  invstd[c] = 1.0f / sqrtf(var + eps);
  if (running_mean) {
    const float unbiased = g.M > 1 ? m2 / (float)(g.M - 1) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
  }
}

template <bool I32>
__device__ __forceinline__ int chan_of(int64_t o, int C) {
  return I32 ? (int)((unsigned)o % (unsigned)C) : (int)(o % C);
}

template <bool I32, int LP>
__global__ void bn_apply_kernel(const float* __restrict__ x, int64_t M, int C, const float* __restrict__ mean,
                                const float* __restrict__ invstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, const float* __restrict__ residual, int relu,
                                float* __restrict__ y, uint16_t* __restrict__ y16, uint8_t* __restrict__ mask) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 * 4 >= M * C) return;
  const int c = chan_of<I32>(i4 * 4, C);
  const v4f mu = ld4(mean + c), is = ld4(invstd + c), ga = ld4(gamma + c), be = ld4(beta + c);
  v4f v = (ld4(x + i4 * 4) - mu) * is * ga + be;
  if (residual) v += ld4(residual + i4 * 4);
  if (relu) {
    unsigned bits = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      bits |= (v[e] > 0.f ? 1u : 0u) << e;   // y > 0 exactly (NaN -> 0, as the ReLU below)
      v[e] = v[e] > 0.f ? v[e] : 0.f;
    }
    if (mask) mask[i4] = (uint8_t)bits;
  }
  st4(y + i4 * 4, v);
  if constexpr (LP != 0) st4_16<LP>(y16 + i4 * 4, v);
}

__global__ void bn_eval_stats_kernel(const float* __restrict__ rm, const float* __restrict__ rv, int C, float eps,
                                     float* __restrict__ mean, float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  invstd[c] = 1.0f / sqrtf(rv[c] + eps);
}

// Backward partials: per chunk and channel, sum g and sum g * xhat, g = dy * act'(y).
__global__ __launch_bounds__(256) void bn_bwd_partial_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                             const uint8_t* __restrict__ mask,
                                                             const float* __restrict__ dy, BnGeom g,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd, int relu,
                                                             float* __restrict__ p0, float* __restrict__ p1) {
  const int q = threadIdx.x % g.CQ, rp = threadIdx.x / g.CQ;
  const int c4 = blockIdx.x * g.CQ + q;
  const int64_t r0 = (int64_t)blockIdx.y * g.rows_per_chunk;
  const int64_t r1 = r0 + g.rows_per_chunk < g.M ? r0 + g.rows_per_chunk : g.M;
  __shared__ v4f s0[256], s1[256];
  v4f a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  if (c4 < g.C4) {
    const v4f mu = ld4(mean + c4 * 4), is = ld4(invstd + c4 * 4);
    for (int64_t r = r0 + rp; r < r1; r += kUnroll * g.RP) {
      v4f vd[kUnroll], vy[kUnroll], vx[kUnroll];
      unsigned mb[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t ru = r + u * g.RP;
        const int64_t o = (ru < r1 ? ru : r) * g.C + c4 * 4;
        vd[u] = ld4(dy + o);
        if (relu && mask) mb[u] = mask[o >> 2];
        else if (relu) vy[u] = ld4(y + o);
        vx[u] = ld4(x + o);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        if (r + u * g.RP < r1) {
          v4f gr = vd[u];
          if (relu && mask) {
#pragma unroll
            for (int e = 0; e < 4; ++e) gr[e] = (mb[u] >> e) & 1u ? gr[e] : 0.f;
          } else if (relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) gr[e] = vy[u][e] <= 0.f ? 0.f : gr[e];
          }
          a0 += gr;
          a1 += gr * ((vx[u] - mu) * is);
        }
      }
    }
  }
  s0[threadIdx.x] = a0;
  s1[threadIdx.x] = a1;
  __syncthreads();
  if (rp == 0 && c4 < g.C4) {
    v4f t0 = {0.f, 0.f, 0.f, 0.f}, t1 = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < g.RP; ++k) {
      t0 += s0[k * g.CQ + q];
      t1 += s1[k * g.CQ + q];
    }
    st4(p0 + (int64_t)blockIdx.y * g.C + c4 * 4, t0);
    st4(p1 + (int64_t)blockIdx.y * g.C + c4 * 4, t1);
  }
}

// acc_dbeta / acc_dgamma (nullable): the parameters' .grad buffers, which the same sums are added into
// (autograd's accumulation fused here instead of one add kernel per parameter)
__global__ void bn_dgamma_kernel(const float* __restrict__ p0, const float* __restrict__ p1, int chunks, int C,
                                 float* __restrict__ dbeta, float* __restrict__ dgamma, float* __restrict__ acc_dbeta,
                                 float* __restrict__ acc_dgamma) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  for (int k0 = 0; k0 < chunks; k0 += kPre) {   // loads ahead of the in-order sums (see combine_chunks)
    float v0[kPre], v1[kPre];
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int64_t k = k0 + u < chunks ? k0 + u : chunks - 1;
      v0[u] = p0[k * C + c];
      v1[u] = p1[k * C + c];
    }
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      if (k0 + u < chunks) {
        a += v0[u];
        b += v1[u];
      }
    }
  }
  dbeta[c] = a;
  dgamma[c] = b;
  if (acc_dbeta) acc_dbeta[c] += a;
  if (acc_dgamma) acc_dgamma[c] += b;
}

template <bool I32, int LP>
__global__ void bn_dx_kernel(const float* __restrict__ x, const float* __restrict__ y, const uint8_t* __restrict__ mask,
                             const float* __restrict__ dy,
                             int64_t M, int C, const float* __restrict__ mean, const float* __restrict__ invstd,
                             const float* __restrict__ gamma, const float* __restrict__ dbeta,
                             const float* __restrict__ dgamma, int relu, int train, float m_norm,
                             const float* __restrict__ m_norm_dev, float* __restrict__ dx,
                             float* __restrict__ dres, uint16_t* __restrict__ dx16) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 * 4 >= M * C) return;
  const int64_t o = i4 * 4;
  const int c = chan_of<I32>(o, C);
  v4f gr = ld4(dy + o);
  if (relu && mask) {   // the forward's ReLU bits (srk_batchnorm_fwd16_mask): 1/16 of y's bytes
    const unsigned mb = mask[i4];
#pragma unroll
    for (int e = 0; e < 4; ++e) gr[e] = (mb >> e) & 1u ? gr[e] : 0.f;
  } else if (relu) {
    const v4f yv = ld4(y + o);
#pragma unroll
    for (int e = 0; e < 4; ++e) gr[e] = yv[e] <= 0.f ? 0.f : gr[e];
  }
  if (dres) st4(dres + o, gr);
  if (!dx) return;
  const v4f is = ld4(invstd + c), ga = ld4(gamma + c);
  if (train) {
    const v4f xhat = (ld4(x + o) - ld4(mean + c)) * is;
    const float mn = m_norm_dev ? m_norm_dev[0] : m_norm;   // rows the statistics span (all ranks' for SyncBN)
    const float inv_m = 1.0f / mn;
    const v4f db = ld4(dbeta + c), dg = ld4(dgamma + c);
    const v4f v = ga * is * inv_m * (mn * gr - db - xhat * dg);
    st4(dx + o, v);
    if constexpr (LP != 0) st4_16<LP>(dx16 + o, v);
  } else {
    const v4f v = ga * is * gr;
    st4(dx + o, v);
    if constexpr (LP != 0) st4_16<LP>(dx16 + o, v);
  }
}

// ---- SyncBatchNorm pieces (torch.nn.SyncBatchNorm over data-parallel ranks).  One rank's (count,
// mean, M2) per channel from the chunk partials; the ranks' triples are gathered by the caller and
// combined in rank order (Chan, fixed order: every rank computes identical statistics).
__global__ __launch_bounds__(256) void bn_local_stats_kernel(const float* __restrict__ pmean,
                                                             const float* __restrict__ pm2, BnGeom g,
                                                             float* __restrict__ stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;   // one lane per channel, in chunk order (the finalize's)
  if (c >= g.C) return;
  float n, mu, m2;
  combine_chunks_fast(pmean, pm2, g, c, n, mu, m2);
  stats[c] = n;
  stats[g.C + c] = mu;
  stats[2 * g.C + c] = m2;
}

__global__ void bn_combine_kernel(const float* __restrict__ all, int world, int C, float eps, float momentum,
                                  float* __restrict__ running_mean, float* __restrict__ running_var,
                                  float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ total) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int r = 0; r < world; ++r) {
    const float* s = all + (size_t)r * 3 * C;
    chan(n, mu, m2, s[c], s[C + c], s[2 * C + c]);
  }
  const float var = n > 0.f ? m2 / n : 0.f;
  if (c == 0 && total) total[0] = n;
  mean[c] = mu;
  invstd[c] = 1.0f / sqrtf(var + eps);
  if (running_mean) {
    const float unbiased = n > 1.f ? m2 / (n - 1.f) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
  }
}

struct BnScratch {
  float* p = nullptr;
  size_t floats = 0;
};
BnScratch g_bs[64];
std::mutex g_bs_mu;

int bn_scratch(size_t floats, float** out) {
  int dev = 0;
  SRK_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_bs_mu);
  BnScratch& s = g_bs[dev & 63];
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

// the element kernels by index width (32-bit channel arithmetic below 2^32 elements) and 16-bit copy
template <int LP>
void launch_apply_lp(int64_t M, int C, hipStream_t s, const float* x, const float* mean, const float* invstd,
                     const float* gamma, const float* beta, const float* residual, int relu, float* y, uint16_t* y16,
                     uint8_t* mask) {
  const int64_t n4 = M * C / 4;
  hipLaunchKernelGGL((M * C < (1LL << 32) ? bn_apply_kernel<true, LP> : bn_apply_kernel<false, LP>),
                     dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, x, M, C, mean, invstd, gamma, beta, residual,
                     relu, y, y16, mask);
}
void launch_apply(int LP, int64_t M, int C, hipStream_t s, const float* x, const float* mean, const float* invstd,
                  const float* gamma, const float* beta, const float* residual, int relu, float* y, uint16_t* y16,
                  uint8_t* mask = nullptr) {
  if (LP == 1) launch_apply_lp<1>(M, C, s, x, mean, invstd, gamma, beta, residual, relu, y, y16, mask);
  else if (LP == 2) launch_apply_lp<2>(M, C, s, x, mean, invstd, gamma, beta, residual, relu, y, y16, mask);
  else launch_apply_lp<0>(M, C, s, x, mean, invstd, gamma, beta, residual, relu, y, nullptr, mask);
}
template <int LP>
void launch_dx_lp(int64_t M, int C, hipStream_t s, const float* x, const float* y, const uint8_t* mask, const float* dy,
                  const float* mean, const float* invstd, const float* gamma, const float* dbeta, const float* dgamma,
                  int relu, int train, float m_norm, const float* m_norm_dev, float* dx, float* dres, uint16_t* dx16) {
  const int64_t n4 = M * C / 4;
  hipLaunchKernelGGL((M * C < (1LL << 32) ? bn_dx_kernel<true, LP> : bn_dx_kernel<false, LP>),
                     dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, x, y, mask, dy, M, C, mean, invstd, gamma,
                     dbeta, dgamma, relu, train, m_norm, m_norm_dev, dx, dres, dx16);
}
void launch_dx(int LP, int64_t M, int C, hipStream_t s, const float* x, const float* y, const uint8_t* mask,
               const float* dy, const float* mean, const float* invstd, const float* gamma, const float* dbeta,
               const float* dgamma, int relu, int train, float m_norm, const float* m_norm_dev, float* dx, float* dres,
               uint16_t* dx16) {
  if (LP == 1) launch_dx_lp<1>(M, C, s, x, y, mask, dy, mean, invstd, gamma, dbeta, dgamma, relu, train, m_norm, m_norm_dev, dx, dres, dx16);
  else if (LP == 2) launch_dx_lp<2>(M, C, s, x, y, mask, dy, mean, invstd, gamma, dbeta, dgamma, relu, train, m_norm, m_norm_dev, dx, dres, dx16);
  else launch_dx_lp<0>(M, C, s, x, y, mask, dy, mean, invstd, gamma, dbeta, dgamma, relu, train, m_norm, m_norm_dev, dx, dres, nullptr);
}

// 16-bit copy requested and possible: the matmul precision's type (1 bf16, 2 fp16), else 0
int copy16_type(const void* p16) {
  const int prec = matmul_prec();
  if (!p16 || prec == kPrecF32 || reinterpret_cast<uintptr_t>(p16) % 16) return 0;
  return prec == kPrecBF16 ? 1 : 2;
}

}  // namespace
}  // namespace srk

extern "C" {

int srk_batchnorm_fwd(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta, float eps,
                      float momentum, int training, float* running_mean, float* running_var, const float* residual,
                      int relu, float* y, float* save_mean, float* save_invstd, void* stream) {
  return srk_batchnorm_fwd16(x, M, C, gamma, beta, eps, momentum, training, running_mean, running_var, residual, relu,
                             y, nullptr, nullptr, save_mean, save_invstd, stream);
}

int srk_batchnorm_fwd16(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta, float eps,
                        float momentum, int training, float* running_mean, float* running_var, const float* residual,
                        int relu, float* y, void* y16, int* y16_written, float* save_mean, float* save_invstd,
                        void* stream) {
  return srk_batchnorm_fwd16_mask(x, M, C, gamma, beta, eps, momentum, training, running_mean, running_var, residual,
                                  relu, y, y16, y16_written, nullptr, save_mean, save_invstd, stream);
}

int srk_batchnorm_fwd16_mask(const float* x, int64_t M, int64_t C, const float* gamma, const float* beta, float eps,
                             float momentum, int training, float* running_mean, float* running_var,
                             const float* residual, int relu, float* y, void* y16, int* y16_written,
                             uint8_t* relu_mask, float* save_mean, float* save_invstd, void* stream) {
  SRK_API_BEGIN
  if (y16_written) *y16_written = 0;
  SRK_REQUIRE(M > 0 && C > 0 && C <= (1 << 24), SRK_ERR_INVALID, "batchnorm: bad shape");
  SRK_REQUIRE(C % 4 == 0, SRK_ERR_INVALID, "batchnorm: channels must be a multiple of 4");
  SRK_REQUIRE(x && gamma && beta && y && save_mean && save_invstd && running_mean && running_var, SRK_ERR_INVALID,
              "batchnorm: null pointer");
  hipStream_t s = srk::as_stream(stream);
  const int lp = srk::copy16_type(y16);
  const bool mk = relu && relu_mask;
  srk::ProfScope prof("batchnorm_fwd", s,
                      ((training ? 12.0 : 8.0) + (lp ? 2.0 : 0.0) + (mk ? 0.25 : 0.0)) * (double)M * C);
  const srk::BnGeom g = srk::bn_geom(M, (int)C);
  if (training) {
    float* part = nullptr;
    if (int rc = srk::bn_scratch((size_t)2 * g.chunks * C, &part)) return rc;
    hipLaunchKernelGGL(srk::bn_stats_kernel, dim3((unsigned)((g.C4 + g.CQ - 1) / g.CQ), (unsigned)g.chunks), dim3(256),
                       0, s, x, g, part, part + (size_t)g.chunks * C);
    // one wave per channel (tree) or one lane per channel in 64-lane blocks (in order: C / 64 waves over the chip)
    if (srk::g_opt_bn_tree == 1)
      hipLaunchKernelGGL(srk::bn_finalize_kernel<1>, dim3((unsigned)((C + 3) / 4)), dim3(256), 0, s, part,
                         part + (size_t)g.chunks * C, g, eps, momentum, save_mean, save_invstd, running_mean,
                         running_var);
    else if (srk::g_opt_bn_tree == 2)
      hipLaunchKernelGGL(srk::bn_finalize_kernel<2>, dim3((unsigned)((C + 63) / 64)), dim3(64), 0, s, part,
                         part + (size_t)g.chunks * C, g, eps, momentum, save_mean, save_invstd, running_mean,
                         running_var);
    else
      hipLaunchKernelGGL(srk::bn_finalize_kernel<0>, dim3((unsigned)((C + 63) / 64)), dim3(64), 0, s, part,
                         part + (size_t)g.chunks * C, g, eps, momentum, save_mean, save_invstd, running_mean,
                         running_var);
  } else {
    hipLaunchKernelGGL(srk::bn_eval_stats_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, running_mean,
                       running_var, (int)C, eps, save_mean, save_invstd);
  }
  srk::launch_apply(lp, M, (int)C, s, x, save_mean, save_invstd, gamma, beta, residual, relu, y,
                    static_cast<uint16_t*>(y16), mk ? relu_mask : nullptr);
  SRK_CHECK_HIP(hipGetLastError());
  if (lp && y16_written) *y16_written = 1;
  return SRK_OK;
  SRK_API_END
}

int srk_batchnorm_bwd(const float* x, const float* y, const float* dy, int64_t M, int64_t C, const float* gamma,
                      const float* save_mean, const float* save_invstd, int training, int relu, float* dx,
                      float* dgamma, float* dbeta, float* dresidual, void* stream) {
  return srk_batchnorm_bwd16(x, y, dy, M, C, gamma, save_mean, save_invstd, training, relu, dx, nullptr, nullptr,
                             dgamma, dbeta, dresidual, stream);
}

int srk_batchnorm_bwd16(const float* x, const float* y, const float* dy, int64_t M, int64_t C, const float* gamma,
                        const float* save_mean, const float* save_invstd, int training, int relu, float* dx,
                        void* dx16, int* dx16_written, float* dgamma, float* dbeta, float* dresidual, void* stream) {
  return srk_batchnorm_bwd16_acc(x, y, dy, M, C, gamma, save_mean, save_invstd, training, relu, dx, dx16, dx16_written,
                                 dgamma, dbeta, dresidual, nullptr, nullptr, stream);
}

int srk_batchnorm_bwd16_acc(const float* x, const float* y, const float* dy, int64_t M, int64_t C, const float* gamma,
                            const float* save_mean, const float* save_invstd, int training, int relu, float* dx,
                            void* dx16, int* dx16_written, float* dgamma, float* dbeta, float* dresidual,
                            float* dgamma_acc, float* dbeta_acc, void* stream) {
  return srk_batchnorm_bwd16_mask(x, y, nullptr, dy, M, C, gamma, save_mean, save_invstd, training, relu, dx, dx16,
                                  dx16_written, dgamma, dbeta, dresidual, dgamma_acc, dbeta_acc, stream);
}

int srk_batchnorm_bwd16_mask(const float* x, const float* y, const uint8_t* relu_mask, const float* dy, int64_t M,
                             int64_t C, const float* gamma, const float* save_mean, const float* save_invstd,
                             int training, int relu, float* dx, void* dx16, int* dx16_written, float* dgamma,
                             float* dbeta, float* dresidual, float* dgamma_acc, float* dbeta_acc, void* stream) {
  SRK_API_BEGIN
  if (dx16_written) *dx16_written = 0;
  SRK_REQUIRE(M > 0 && C > 0 && C % 4 == 0, SRK_ERR_INVALID, "batchnorm_bwd: bad shape (C % 4 == 0 required)");
  SRK_REQUIRE(x && (y || (relu && relu_mask)) && dy && gamma && save_mean && save_invstd && dgamma && dbeta,
              SRK_ERR_INVALID, "batchnorm_bwd: null pointer");
  hipStream_t s = srk::as_stream(stream);
  const int lp = dx ? srk::copy16_type(dx16) : 0;
  const uint8_t* mk = relu ? relu_mask : nullptr;
  // algorithmic bytes: x, dy and y (or its mask bits) read twice, dx written (+ its 16-bit copy)
  srk::ProfScope prof("batchnorm_bwd", s, ((mk ? 12.5 : 16.0) + (lp ? 2.0 : 0.0)) * (double)M * C);
  const srk::BnGeom g = srk::bn_geom(M, (int)C);
  float* part = nullptr;
  if (int rc = srk::bn_scratch((size_t)2 * g.chunks * C, &part)) return rc;
  hipLaunchKernelGGL(srk::bn_bwd_partial_kernel, dim3((unsigned)((g.C4 + g.CQ - 1) / g.CQ), (unsigned)g.chunks),
                     dim3(256), 0, s, x, y, mk, dy, g, save_mean, save_invstd, relu, part, part + (size_t)g.chunks * C);
  hipLaunchKernelGGL(srk::bn_dgamma_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, part,
                     part + (size_t)g.chunks * C, g.chunks, (int)C, dbeta, dgamma, dbeta_acc, dgamma_acc);
  srk::launch_dx(lp, M, (int)C, s, x, y, mk, dy, save_mean, save_invstd, gamma, dbeta, dgamma, relu, training,
                 (float)M, nullptr, dx, dresidual, static_cast<uint16_t*>(dx16));
  SRK_CHECK_HIP(hipGetLastError());
  if (lp && dx16_written) *dx16_written = 1;
  return SRK_OK;
  SRK_API_END
}

int srk_batchnorm_stats(const float* x, int64_t M, int64_t C, float* stats, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(M > 0 && C > 0 && C % 4 == 0 && C <= (1 << 24), SRK_ERR_INVALID,
              "batchnorm_stats: bad shape (C % 4 == 0 required)");
  SRK_REQUIRE(M < (1LL << 24), SRK_ERR_INVALID, "batchnorm_stats: > 2^24 rows per rank (fp32 counts)");
  SRK_REQUIRE(x && stats, SRK_ERR_INVALID, "batchnorm_stats: null pointer");
  hipStream_t s = srk::as_stream(stream);
  srk::ProfScope prof("batchnorm_fwd", s, 4.0 * (double)M * C);
  const srk::BnGeom g = srk::bn_geom(M, (int)C);
  float* part = nullptr;
  if (int rc = srk::bn_scratch((size_t)2 * g.chunks * C, &part)) return rc;
  hipLaunchKernelGGL(srk::bn_stats_kernel, dim3((unsigned)((g.C4 + g.CQ - 1) / g.CQ), (unsigned)g.chunks), dim3(256), 0,
                     s, x, g, part, part + (size_t)g.chunks * C);
  hipLaunchKernelGGL(srk::bn_local_stats_kernel, dim3((unsigned)((C + 63) / 64)), dim3(64), 0, s, part,
                     part + (size_t)g.chunks * C, g, stats);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_batchnorm_combine(const float* stats_all, int world, int64_t C, float eps, float momentum,
                          float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                          float* total_count, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(world >= 1 && C > 0, SRK_ERR_INVALID, "batchnorm_combine: bad shape");
  SRK_REQUIRE(stats_all && save_mean && save_invstd && ((running_mean == nullptr) == (running_var == nullptr)),
              SRK_ERR_INVALID, "batchnorm_combine: null pointer");
  hipStream_t s = srk::as_stream(stream);
  hipLaunchKernelGGL(srk::bn_combine_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, stats_all, world,
                     (int)C, eps, momentum, running_mean, running_var, save_mean, save_invstd, total_count);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_batchnorm_apply(const float* x, int64_t M, int64_t C, const float* save_mean, const float* save_invstd,
                        const float* gamma, const float* beta, const float* residual, int relu, float* y,
                        void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(M > 0 && C > 0 && C % 4 == 0, SRK_ERR_INVALID, "batchnorm_apply: bad shape (C % 4 == 0 required)");
  SRK_REQUIRE(x && save_mean && save_invstd && gamma && beta && y, SRK_ERR_INVALID, "batchnorm_apply: null pointer");
  hipStream_t s = srk::as_stream(stream);
  srk::ProfScope prof("batchnorm_fwd", s, 8.0 * (double)M * C);
  srk::launch_apply(0, M, (int)C, s, x, save_mean, save_invstd, gamma, beta, residual, relu, y, nullptr);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_batchnorm_bwd_reduce(const float* x, const float* y, const float* dy, int64_t M, int64_t C,
                             const float* save_mean, const float* save_invstd, int relu, float* sums, void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(M > 0 && C > 0 && C % 4 == 0, SRK_ERR_INVALID, "batchnorm_bwd_reduce: bad shape");
  SRK_REQUIRE(x && y && dy && save_mean && save_invstd && sums, SRK_ERR_INVALID, "batchnorm_bwd_reduce: null pointer");
  hipStream_t s = srk::as_stream(stream);
  srk::ProfScope prof("batchnorm_bwd", s, 12.0 * (double)M * C);
  const srk::BnGeom g = srk::bn_geom(M, (int)C);
  float* part = nullptr;
  if (int rc = srk::bn_scratch((size_t)2 * g.chunks * C, &part)) return rc;
  hipLaunchKernelGGL(srk::bn_bwd_partial_kernel, dim3((unsigned)((g.C4 + g.CQ - 1) / g.CQ), (unsigned)g.chunks),
                     dim3(256), 0, s, x, y, nullptr, dy, g, save_mean, save_invstd, relu, part,
                     part + (size_t)g.chunks * C);
  hipLaunchKernelGGL(srk::bn_dgamma_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, part,
                     part + (size_t)g.chunks * C, g.chunks, (int)C, sums, sums + C, nullptr, nullptr);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_batchnorm_bwd_dx(const float* x, const float* y, const float* dy, int64_t M, int64_t C,
                         const float* total_count, const float* gamma, const float* save_mean,
                         const float* save_invstd, const float* sums, int relu, float* dx, float* dresidual,
                         void* stream) {
  SRK_API_BEGIN
  SRK_REQUIRE(M > 0 && C > 0 && C % 4 == 0, SRK_ERR_INVALID, "batchnorm_bwd_dx: bad shape");
  SRK_REQUIRE(x && y && dy && total_count && gamma && save_mean && save_invstd && sums && (dx || dresidual),
              SRK_ERR_INVALID, "batchnorm_bwd_dx: null pointer");
  hipStream_t s = srk::as_stream(stream);
  srk::ProfScope prof("batchnorm_bwd", s, 16.0 * (double)M * C);
  srk::launch_dx(0, M, (int)C, s, x, y, nullptr, dy, save_mean, save_invstd, gamma, sums, sums + C, relu, 1, 0.f,
                 total_count, dx, dresidual, nullptr);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"

namespace srk {
int release_bn_scratch() {
  std::lock_guard<std::mutex> lk(g_bs_mu);
  SRK_CHECK_HIP(hipDeviceSynchronize());
  for (BnScratch& s : g_bs) {
    if (s.p) SRK_CHECK_HIP(hipFree(s.p));
    s.p = nullptr;
    s.floats = 0;
  }
  g_scratch_gen.fetch_add(1);
  return SRK_OK;
}
}  // namespace srk
