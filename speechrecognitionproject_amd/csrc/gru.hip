// K5: bidirectional GRU layer forward / backward (PyTorch gate convention [r; z; n], h0 = 0),
// replacing nn.GRU(bidirectional=True, batch_first=True) at models/model_mfcc_bgru.py:25,35,
// model_spec_bgru.py:23,33 and model_resnet_bgru.py:130,135.
//
//   r = sigmoid(W_ir x + b_ir + W_hr h + b_hr)      z = sigmoid(W_iz x + b_iz + W_hz h + b_hz)
//   n = tanh(W_in x + b_in + r * (W_hn h + b_hn))   h' = (1 - z) * n + z * h
//
// Forward  = one MFMA GEMM for the input projections of BOTH directions and all T steps
//            (gi = x W_ih_cat^T + b_ih, [B*T, 6H]), then T launches of a fused recurrence step
//            kernel: gh = h_{t-1} W_hh^T on the matrix cores with the gate math as its epilogue.
// Backward = T launches of a fused step kernel (dh_{t} = dy_t + dgh_{t+1} W_hh + dh_{t+1} z_{t+1},
//            then the gate derivatives as epilogue), followed by the weight-gradient GEMMs
//            (dW_ih = dgi^T x, dW_hh = dgh^T h_prev with K = B*T) and column sums for the biases.
//
// Workspace (fp32, caller-owned; sizes in srk_gru_workspace_floats):
//   fwd:  gi [B*T, 6H] | gates [2][T][B][4H] (r, z, n, W_hn h + b_hn)       — kept for backward
//   bwd:  dgi [B*T, 6H] | dgh [2][B][T][3H] | dgh_edge [2][B][3H] | dhz [2][B][H]
#include <algorithm>
#include <mutex>

#include "gemm.h"
#include "gru_internal.h"

namespace srk {
namespace {

// Recurrence step tiling.  One workgroup = 64 batch rows x 16 hidden units of one direction
// (all three gates: 48 columns of W_hh for the forward step), 4 waves = 4 x 16 rows.
// Both operands are staged ROW-major in LDS (row pitch BK+4 floats) and read as float4: for
// MFMA k-substep s a lane with k-quad q uses k = kbase + 4q + s, for A and B alike (any fixed
// permutation of k is a valid GEMM order), so one ds_read_b128 feeds four v_mfma_f32_16x16x4_f32.
// Workgroup -> (direction, batch group, unit slice) is XCD-aware: the 32 workgroups that share
// an XCD (blockIdx % 8, observed round-robin dispatch) take the slices of ONE (direction, group)
// pair, so that direction's W_hh (3 MB fp32) stays resident in that XCD's 4 MB L2 from one step
// launch to the next.  (Placement only changes speed, never results.)
constexpr int kRows = 64;    // batch rows per workgroup
constexpr int kUnits = 16;   // hidden units per workgroup
constexpr int kBK = 128;     // k per LDS stage
constexpr int kPitch = kBK + 4;

struct GruArgs {
  int B, T, H, in;
  int G, S;             // batch groups (ceil(B/64)), unit slices (H/16)
  const float* y_in;    // fwd: y (h_prev source); bwd: y
  float* y;             // fwd output [B][T][2H]
  const float* gi;      // [B*T][6H]
  const float* w_hh;    // [2][3H][H]
  const float* b_hh;    // [2][3H]
  float* gates;         // [2][T][B][4H]
  const float* dy;      // [B][T][2H]
  float* dgi;           // [B*T][6H]
  float* dgh;           // [2][B][T][3H]
  float* dgh_edge;      // [2][B][3H]
  float* dhz;           // [2][B][H]
};

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// Native 4-float vector: HIP's float4 is a struct whose copies lower to memcpy, which SROA cannot
// keep in registers (a float4 staging array ends up in scratch); ext_vector loads/stores do not.
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4f ld4(const float* p) { return *reinterpret_cast<const v4f*>(p); }
__device__ __forceinline__ void st4(float* p, v4f v) { *reinterpret_cast<v4f*>(p) = v; }

__device__ __forceinline__ void map_block(const GruArgs& a, int& dir, int& group, int& slice) {
  const int nwg = 2 * a.G * a.S;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  const int pair = wgid / a.S;
  slice = wgid % a.S;
  dir = pair / a.G;
  group = pair % a.G;
}

// ------------------------------------------------------------------ forward step
// gh[b, g*H + j] = sum_k h_prev[b, k] W_hh[g*H + j, k];  epilogue = the GRU cell.
__global__ __launch_bounds__(256) void gru_fwd_step_kernel(GruArgs a, int step) {
  constexpr int WR = 3 * kUnits;                        // W rows (gate columns) per workgroup
  constexpr int VA = kRows * kBK / 4 / 256;             // float4 per thread per stage: 8
  constexpr int VW = WR * kBK / 4 / 256;                // 6
  __shared__ __attribute__((aligned(16))) float smem[2 * (kRows + WR) * kPitch];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  int dir, group, slice;
  map_block(a, dir, group, slice);
  const int B = a.B, T = a.T, H = a.H;
  const int t = dir == 0 ? step : T - 1 - step;
  const int tprev = dir == 0 ? t - 1 : t + 1;
  const int b0 = group * kRows, j0 = slice * kUnits;
  const float* __restrict__ W = a.w_hh + (size_t)dir * 3 * H * H;

  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 acc[3];
#pragma unroll
  for (int g = 0; g < 3; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (step > 0) {
    v4f ra[VA], rw[VW];
    auto load = [&](int k0) {
#pragma unroll
      for (int i = 0; i < VA; ++i) {
        const int v = tid + i * 256, row = v / (kBK / 4), kq = (v % (kBK / 4)) * 4;
        const int b = b0 + row;
        const v4f x = ld4(a.y_in + ((size_t)(b < B ? b : B - 1) * T + tprev) * 2 * H + dir * H + k0 + kq);
        ra[i] = b < B ? x : v4f{0.f, 0.f, 0.f, 0.f};   // clamped row + select: no exec-masked loads
      }
#pragma unroll
      for (int i = 0; i < VW; ++i) {
        const int v = tid + i * 256, c = v / (kBK / 4), kq = (v % (kBK / 4)) * 4;
        const int g = c / kUnits, jj = c % kUnits;
        rw[i] = ld4(W + (size_t)(g * H + j0 + jj) * H + k0 + kq);
      }
    };
    auto store = [&](int buf) {
      float* As = smem + buf * (kRows + WR) * kPitch;
      float* Ws = As + kRows * kPitch;
#pragma unroll
      for (int i = 0; i < VA; ++i) {
        const int v = tid + i * 256, row = v / (kBK / 4), kq = (v % (kBK / 4)) * 4;
        st4(As + row * kPitch + kq, ra[i]);
      }
#pragma unroll
      for (int i = 0; i < VW; ++i) {
        const int v = tid + i * 256, c = v / (kBK / 4), kq = (v % (kBK / 4)) * 4;
        st4(Ws + c * kPitch + kq, rw[i]);
      }
    };
    const int nk = H / kBK;
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load((kt + 1) * kBK);
      const float* As = smem + cur * (kRows + WR) * kPitch;
      const float* Ws = As + kRows * kPitch;
#pragma unroll
      for (int kb = 0; kb < kBK; kb += 16) {
        const v4f av = ld4(As + (wave * 16 + lr) * kPitch + kb + 4 * lq);
        v4f wv[3];
#pragma unroll
        for (int g = 0; g < 3; ++g) wv[g] = ld4(Ws + (g * kUnits + lr) * kPitch + kb + 4 * lq);
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, wv[g].x, acc[g], 0, 0, 0);
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, wv[g].y, acc[g], 0, 0, 0);
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, wv[g].z, acc[g], 0, 0, 0);
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, wv[g].w, acc[g], 0, 0, 0);
        }
      }
      asm volatile("" ::: "memory");      // keep the stage-k+1 LDS store (and its vmcnt wait)
      __builtin_amdgcn_sched_barrier(0);   // after this stage's MFMAs
      if (kt + 1 < nk) store(cur ^ 1);
      __syncthreads();
    }
  }

  // epilogue: lane owns rows 16*wave + 4*lq + r, unit j = j0 + lr, all three gates
  const int j = j0 + lr;
  const float bhr = a.b_hh[dir * 3 * H + j], bhz = a.b_hh[dir * 3 * H + H + j], bhn = a.b_hh[dir * 3 * H + 2 * H + j];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = b0 + wave * 16 + lq * 4 + r;
    if (b >= B) continue;
    const float* gi = a.gi + ((size_t)b * T + t) * 6 * H + dir * 3 * H;
    const float ghn = acc[2][r] + bhn;
    const float rg = sigmoidf_(gi[j] + (acc[0][r] + bhr));
    const float zg = sigmoidf_(gi[H + j] + (acc[1][r] + bhz));
    const float ng = tanhf(gi[2 * H + j] + rg * ghn);
    const float hp = step > 0 ? a.y_in[((size_t)b * T + tprev) * 2 * H + dir * H + j] : 0.f;
    const float h = (1.0f - zg) * ng + zg * hp;
    a.y[((size_t)b * T + t) * 2 * H + dir * H + j] = h;
    float* gs = a.gates + (((size_t)dir * T + t) * B + b) * 4 * H;
    gs[j] = rg;
    gs[H + j] = zg;
    gs[2 * H + j] = ng;
    gs[3 * H + j] = ghn;
  }
}

// ------------------------------------------------------------------ backward step
// dh_rec[b, j] = sum_c dgh_next[b, c] W_hh[c, j] (c over 3H);  epilogue = the cell derivatives.
__global__ __launch_bounds__(256) void gru_bwd_step_kernel(GruArgs a, int step) {
  constexpr int VA = kRows * kBK / 4 / 256;             // 8
  constexpr int VW = kBK * kUnits / 4 / 256;            // 2
  __shared__ __attribute__((aligned(16))) float smem[2 * (kRows + kUnits) * kPitch];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  int dir, group, slice;
  map_block(a, dir, group, slice);
  const int B = a.B, T = a.T, H = a.H;
  const int t = dir == 0 ? T - 1 - step : step;          // time processed now
  const int tnext = dir == 0 ? t + 1 : t - 1;           // processed by the previous step
  const int tprev = dir == 0 ? t - 1 : t + 1;           // h_prev source
  const bool edge = (step == T - 1);                    // h_prev = 0 here
  const int b0 = group * kRows, j0 = slice * kUnits;
  const float* __restrict__ W = a.w_hh + (size_t)dir * 3 * H * H;
  const float* __restrict__ dghn = a.dgh + (size_t)dir * B * T * 3 * H;   // [B][T][3H] of this dir

  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  if (step > 0) {
    v4f ra[VA], rw[VW];
    auto load = [&](int k0) {
#pragma unroll
      for (int i = 0; i < VA; ++i) {
        const int v = tid + i * 256, row = v / (kBK / 4), kq = (v % (kBK / 4)) * 4;
        const int b = b0 + row;
        const v4f x = ld4(dghn + ((size_t)(b < B ? b : B - 1) * T + tnext) * 3 * H + k0 + kq);
        ra[i] = b < B ? x : v4f{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < VW; ++i) {   // W_hh[k0 + kr][j0 .. j0+15], 4 units per float4
        const int v = tid + i * 256, kr = v / (kUnits / 4), jq = (v % (kUnits / 4)) * 4;
        rw[i] = ld4(W + (size_t)(k0 + kr) * H + j0 + jq);
      }
    };
    auto store = [&](int buf) {
      float* As = smem + buf * (kRows + kUnits) * kPitch;
      float* Ws = As + kRows * kPitch;    // [unit][k]
#pragma unroll
      for (int i = 0; i < VA; ++i) {
        const int v = tid + i * 256, row = v / (kBK / 4), kq = (v % (kBK / 4)) * 4;
        st4(As + row * kPitch + kq, ra[i]);
      }
#pragma unroll
      for (int i = 0; i < VW; ++i) {
        const int v = tid + i * 256, kr = v / (kUnits / 4), jq = (v % (kUnits / 4)) * 4;
        Ws[(jq + 0) * kPitch + kr] = rw[i].x;
        Ws[(jq + 1) * kPitch + kr] = rw[i].y;
        Ws[(jq + 2) * kPitch + kr] = rw[i].z;
        Ws[(jq + 3) * kPitch + kr] = rw[i].w;
      }
    };
    const int nk = 3 * H / kBK;
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load((kt + 1) * kBK);
      const float* As = smem + cur * (kRows + kUnits) * kPitch;
      const float* Ws = As + kRows * kPitch;
#pragma unroll
      for (int kb = 0; kb < kBK; kb += 16) {
        const v4f av = ld4(As + (wave * 16 + lr) * kPitch + kb + 4 * lq);
        const v4f wv = ld4(Ws + lr * kPitch + kb + 4 * lq);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, wv.x, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, wv.y, acc[1], 0, 0, 0);
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, wv.z, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, wv.w, acc[1], 0, 0, 0);
      }
      asm volatile("" ::: "memory");      // keep the stage-k+1 LDS store (and its vmcnt wait)
      __builtin_amdgcn_sched_barrier(0);   // after this stage's MFMAs
      if (kt + 1 < nk) store(cur ^ 1);
      __syncthreads();
    }
  }

  const int j = j0 + lr;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = b0 + wave * 16 + lq * 4 + r;
    if (b >= B) continue;
    float* dhz = a.dhz + ((size_t)dir * B + b) * H + j;
    float dh = a.dy[((size_t)b * T + t) * 2 * H + dir * H + j];
    if (step > 0) dh += (acc[0][r] + acc[1][r]) + *dhz;
    const float* gs = a.gates + (((size_t)dir * T + t) * B + b) * 4 * H;
    const float rg = gs[j], zg = gs[H + j], ng = gs[2 * H + j], ghn = gs[3 * H + j];
    const float hp = edge ? 0.f : a.y_in[((size_t)b * T + tprev) * 2 * H + dir * H + j];
    const float dn = dh * (1.0f - zg);
    const float daz = dh * (hp - ng) * zg * (1.0f - zg);
    const float dan = dn * (1.0f - ng * ng);
    const float dar = dan * ghn * rg * (1.0f - rg);
    float* dgi = a.dgi + ((size_t)b * T + t) * 6 * H + dir * 3 * H;
    dgi[j] = dar;
    dgi[H + j] = daz;
    dgi[2 * H + j] = dan;
    float* dg = edge ? a.dgh_edge + ((size_t)dir * B + b) * 3 * H
                     : a.dgh + (((size_t)dir * B + b) * T + t) * 3 * H;
    dg[j] = dar;
    dg[H + j] = daz;
    dg[2 * H + j] = dan * rg;
    if (edge) {   // keep the h_prev = 0 row out of the dW_hh GEMM (see layer_bwd)
      float* z0 = a.dgh + (((size_t)dir * B + b) * T + t) * 3 * H;
      z0[j] = 0.f; z0[H + j] = 0.f; z0[2 * H + j] = 0.f;
    }
    *dhz = dh * zg;
  }
}

int check_dims(int64_t B, int64_t T, int64_t in, int64_t H) {
  SRK_REQUIRE(B > 0 && T > 0 && in > 0 && H > 0, SRK_ERR_INVALID, "gru: dims must be positive");
  SRK_REQUIRE(H % kBK == 0, SRK_ERR_INVALID, "gru: hidden size must be a multiple of 128");
  SRK_REQUIRE(B * T * 6 * H < ((int64_t)1 << 40), SRK_ERR_INVALID, "gru: problem too large");
  return SRK_OK;
}

// Input widths that are not a multiple of 4 (the 39 MFCC features of model_mfcc_bgru.py:25):
// the input-projection GEMMs run on a copy of x / W_ih padded with zero columns to a multiple of
// 4, so they take the 16-B vector (and LDS-DMA / buffer-load) paths; a zero column adds exact
// zeros to every dot product.  dW_ih is produced at the padded width and its first `in` columns
// are written (or added) into the caller's tensor.
__global__ void pad_cols_kernel(const float* __restrict__ src, int64_t rows, int cols, float* __restrict__ dst,
                                int colsp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * colsp) return;
  const int64_t r = i / colsp;
  const int c = (int)(i - r * colsp);
  dst[i] = c < cols ? src[r * cols + c] : 0.f;
}
__global__ void unpad_cols_kernel(const float* __restrict__ src, int64_t rows, int colsp, float* __restrict__ dst,
                                  int cols, int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols) return;
  const int64_t r = i / cols;
  const int c = (int)(i - r * cols);
  const float v = src[r * colsp + c];
  dst[i] = accumulate ? dst[i] + v : v;
}
// bf16 / fp16 mode: fp32 [rows][cols] -> 16-bit [rows][colsp] (zero columns past cols), rounded to
// nearest-even — the GEMM operands of the layer that are not produced by the recurrence kernels.
template <bool F16>
__global__ void to16_kernel(const float* __restrict__ src, int64_t rows, int cols, uint16_t* __restrict__ dst,
                            int colsp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * colsp) return;
  const int64_t r = i / colsp;
  const int c = (int)(i - r * colsp);
  const float v = c < cols ? src[r * cols + c] : 0.f;
  if (F16) {
    const _Float16 h = (_Float16)v;
    dst[i] = __builtin_bit_cast(uint16_t, h);
  } else {
    const __bf16 h = (__bf16)v;
    dst[i] = __builtin_bit_cast(uint16_t, h);
  }
}
// Dense case (no column padding, 8 | n, 16-B aligned): 8 elements per thread, two 16-B loads and one
// 16-B store, no index division.
template <bool F16>
__global__ void to16_vec8_kernel(const float* __restrict__ src, int64_t n8, uint16_t* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((ext_vector_type(8))) typename std::conditional<F16, _Float16, __bf16>::type e8;
  const f4 a = *reinterpret_cast<const f4*>(src + 8 * i), b = *reinterpret_cast<const f4*>(src + 8 * i + 4);
  const e8 h = __builtin_convertvector((__attribute__((ext_vector_type(8))) float){a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w}, e8);
  *reinterpret_cast<u4*>(dst + 8 * i) = __builtin_bit_cast(u4, h);
}

int to16(const float* src, int64_t rows, int64_t cols, uint16_t* dst, int64_t colsp, hipStream_t s) {
  const int64_t n = rows * colsp;
  if (cols == colsp && n % 8 == 0 && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0) {
    const int64_t n8 = n / 8;
    if (matmul_prec() == kPrecF16)
      hipLaunchKernelGGL(to16_vec8_kernel<true>, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, src, n8, dst);
    else
      hipLaunchKernelGGL(to16_vec8_kernel<false>, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, s, src, n8, dst);
    SRK_CHECK_HIP(hipGetLastError());
    return SRK_OK;
  }
  if (matmul_prec() == kPrecF16)
    hipLaunchKernelGGL(to16_kernel<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, rows, (int)cols,
                       dst, (int)colsp);
  else
    hipLaunchKernelGGL(to16_kernel<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, rows, (int)cols,
                       dst, (int)colsp);
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}
// Bias gradients from the 16-bit backward kernel's partials [part][2 dir][4][H] (sums of dar, daz,
// dan, dan * r), summed over the valid (chunk, group) parts in order: db_ih = (dar, daz, dan),
// db_hh = (dar, daz, dan * r); `accumulate` adds into the caller's tensors.
__device__ __forceinline__ void dbias_reduce_at(int i, const float* __restrict__ part, int nparts, int B, int H,
                                                int rows_per_part, float* __restrict__ db_ih,
                                                float* __restrict__ db_hh, int accumulate) {
  if (i >= 2 * 3 * H) return;   // i over [2 dir][3][H]
  const int dir = i / (3 * H), g = (i / H) % 3, j = i % H;
  const int per_chunk = 256 / rows_per_part;
  float si = 0.f, sh = 0.f;
  for (int p = 0; p < nparts; ++p) {
    if ((p / per_chunk) * 256 + (p % per_chunk) * rows_per_part >= B) continue;   // (chunk, group) without rows
    const float* q = part + ((size_t)p * 2 + dir) * 4 * H;
    si += q[g * H + j];
    sh += q[(g == 2 ? 3 : g) * H + j];
  }
  db_ih[i] = accumulate ? db_ih[i] + si : si;
  db_hh[i] = accumulate ? db_hh[i] + sh : sh;
}
__global__ void dbias_reduce_kernel(const float* __restrict__ part, int nparts, int B, int H, int rows_per_part,
                                    float* __restrict__ db_ih, float* __restrict__ db_hh, int accumulate) {
  dbias_reduce_at(blockIdx.x * blockDim.x + threadIdx.x, part, nparts, B, H, rows_per_part, db_ih, db_hh, accumulate);
}

// Both reductions of the fused 16-bit backward in one launch.  Blocks [0, dw_blocks): dW_hh[dir] (+)= sum
// over the partials [part][2 dir][3H][H] in part order (deterministic), 4 consecutive columns per thread
// (part p = chunk * 8 + group covers batch rows 256 chunk + 32 group ..; parts past the batch were never
// written and are skipped).  The rest: the bias gradients, as dbias_reduce_kernel.
__global__ void dwhh_dbias_reduce_kernel(const float* __restrict__ part, int nparts, int B, int64_t per_dir,
                                         float* __restrict__ dw, int accumulate, int dw_blocks,
                                         const float* __restrict__ bpart, int bparts, int H, int rows_per_part,
                                         float* __restrict__ db_ih, float* __restrict__ db_hh) {
  if ((int)blockIdx.x >= dw_blocks) {
    dbias_reduce_at(((int)blockIdx.x - dw_blocks) * blockDim.x + threadIdx.x, bpart, bparts, B, H, rows_per_part,
                    db_ih, db_hh, accumulate);
    return;
  }
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i4 * 4 >= 2 * per_dir) return;
  const int64_t o = i4 * 4, dir = o / per_dir, e = o - dir * per_dir;
  v4f acc = accumulate ? *reinterpret_cast<const v4f*>(dw + o) : v4f{0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < nparts; ++p) {
    if ((p / 8) * 256 + (p % 8) * 32 >= B) continue;
    acc += *reinterpret_cast<const v4f*>(part + ((size_t)p * 2 + dir) * per_dir + e);
  }
  *reinterpret_cast<v4f*>(dw + o) = acc;
}

// grow-only scratch of the fused backward's dW_hh partials (graph-safe: bumps g_scratch_gen on growth)
struct GruScratch {
  float* p = nullptr;
  size_t floats = 0;
};
GruScratch g_gs[64];
std::mutex g_gs_mu;

int gru_scratch(size_t floats, float** out) {
  int dev = 0;
  SRK_CHECK_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_gs_mu);
  GruScratch& sc = g_gs[dev & 63];
  if (sc.floats < floats) {
    if (sc.p) {
      SRK_CHECK_HIP(hipDeviceSynchronize());
      SRK_CHECK_HIP(hipFree(sc.p));
    }
    sc.floats = floats + floats / 4;
    SRK_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&sc.p), sc.floats * sizeof(float)));
    g_scratch_gen.fetch_add(1);
  }
  *out = sc.p;
  return SRK_OK;
}

inline int64_t pad4(int64_t v) { return (v + 3) / 4 * 4; }
inline bool padded_in(int64_t in) { return in % 4 != 0; }
int pad_cols(const float* src, int64_t rows, int64_t cols, float* dst, hipStream_t s) {
  const int64_t n = rows * pad4(cols);
  hipLaunchKernelGGL(pad_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, rows, (int)cols, dst,
                     (int)pad4(cols));
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
}

}  // namespace

int release_gru_scratch() {
  std::lock_guard<std::mutex> lk(g_gs_mu);
  SRK_CHECK_HIP(hipDeviceSynchronize());
  for (GruScratch& sc : g_gs) {
    if (sc.p) SRK_CHECK_HIP(hipFree(sc.p));
    sc.p = nullptr;
    sc.floats = 0;
  }
  g_scratch_gen.fetch_add(1);
  return SRK_OK;
}
}  // namespace srk

using srk::GemmDesc;

extern "C" {

// Both workspaces end with a 64-float-aligned block of kCounterFloats arrival counters (the
// persistent recurrence kernels' step ordering; see gru_persistent.hip).
// Before them, 64-float aligned, the persistent kernels' hand-off ring in MFMA-fragment order
// (fwd: h [2 dir][kHandoffSlots][rows][H], bwd: dg [2 dir][kHandoffSlots][rows][3H]).
static int64_t fwd_xbuf_off(int64_t B, int64_t T, int64_t H) { return (B * T * 6 * H + 2 * T * B * 4 * H + 63) / 64 * 64; }
static int64_t bwd_xbuf_off(int64_t B, int64_t T, int64_t H) {
  return (B * T * 6 * H + 2 * B * T * 3 * H + 2 * B * 3 * H + 2 * B * H + 63) / 64 * 64;
}
// (rows padded to the 64-row groups of one launch chunk: <= 512 rows, or B rounded up to 64)
static int64_t xbuf_rows(int64_t B) { return std::min<int64_t>((B + 63) / 64 * 64, 512); }
static int64_t fwd_counter_off(int64_t B, int64_t T, int64_t H) {
  return fwd_xbuf_off(B, T, H) + 2 * srk::kHandoffSlots * xbuf_rows(B) * H;
}
static int64_t bwd_counter_off(int64_t B, int64_t T, int64_t H) {
  return bwd_xbuf_off(B, T, H) + 6 * srk::kHandoffSlots * xbuf_rows(B) * H;
}

// After the counters, for an input width that is not a multiple of 4 (srk::padded_in):
//   fwd: x padded [B*T][in4] (kept for the backward's dW_ih) | W_ih padded [6H][in4]
//   bwd: W_ih padded [6H][in4] | dW_ih padded [6H][in4] | dx padded [B*T][in4]
static int64_t pad_off(int64_t B, int64_t T, int64_t H, int backward) {
  return ((backward ? bwd_counter_off(B, T, H) : fwd_counter_off(B, T, H)) + srk::kCounterFloats + 63) / 64 * 64;
}

// Then the bf16 / fp16 ("h16") region, used when the 16-bit persistent kernels run (use_h16):
//   fwd: x16 [B*T][in8] | W_ih16 [6H][in8] | y16 [B*T][2H]          (16-bit, kept for the backward)
//   bwd: bias partials [8 * chunks][2][4][H] | dW_ih [6H][in8] | dx [B*T][in8]   (fp32; the last two
//        only when in8 != in); dgi16 / dgh16 alias the fp32 dgi region (unused in this mode).
static int64_t pad_end(int64_t B, int64_t T, int64_t in, int64_t H, int backward) {
  int64_t e = pad_off(B, T, H, backward) + 64;
  if (srk::padded_in(in)) {
    const int64_t in4 = srk::pad4(in);
    e += (backward ? 2 * 6 * H * in4 + B * T * in4 : B * T * in4 + 6 * H * in4) + 64;
  }
  return (e + 63) / 64 * 64;
}
static int64_t up64(int64_t v) { return (v + 63) / 64 * 64; }
static int64_t in8_of(int64_t in) { return (in + 7) / 8 * 8; }
static int64_t h16_floats(int64_t B, int64_t T, int64_t in, int64_t H, int backward) {
  const int64_t in8 = in8_of(in), BT = B * T;
  if (!backward) return up64(BT * in8 / 2 + 1) + up64(6 * H * in8 / 2 + 1) + up64(BT * 2 * H / 2 + 1);
  const int64_t chunks = (B + 255) / 256;
  return up64(chunks * 8 * 2 * 4 * H) + (in8 != in ? up64(6 * H * in8) + up64(BT * in8) : 0);   // <= 8 parts per chunk
}
// The 16-bit path: a 16-bit precision, the persistent kernels (both directions of the layer), and
// 32-bit byte offsets for the 16-bit GEMM operands.
static bool use_h16(int64_t B, int64_t T, int64_t in, int64_t H) {
  return srk::matmul_prec() != srk::kPrecF32 && srk::g_opt_gru_persistent &&
         srk::gru_persistent_supported(B, T, H, false) && srk::gru_persistent_supported(B, T, H, true) &&
         (double)B * T * 6 * H * 2 < 2147483647.0 && (double)B * T * in8_of(in) * 2 < 2147483647.0;
}

int64_t srk_gru_workspace_floats(int64_t B, int64_t T, int64_t in, int64_t H, int backward) {
  return pad_end(B, T, in, H, backward) + (H == 512 ? h16_floats(B, T, in, H, backward) + 64 : 0);
}

int srk_gru_layer_fwd(const float* x, int64_t B, int64_t T, int64_t in, int64_t H, const float* w_ih,
                      const float* w_hh, const float* b_ih, const float* b_hh, float* y, float* ws, void* stream) {
  return srk_gru_layer_fwd_x16(x, nullptr, B, T, in, H, w_ih, w_hh, b_ih, b_hh, y, ws, stream);
}

int64_t srk_gru_y16_offset(int64_t B, int64_t T, int64_t in, int64_t H) {
  if (srk::check_dims(B, T, in, H) || H != 512 || !use_h16(B, T, in, H)) return -1;
  const int64_t in8 = in8_of(in), BT = B * T;
  return pad_end(B, T, in, H, 0) + up64(BT * in8 / 2 + 1) + up64(6 * H * in8 / 2 + 1);
}

int srk_gru_layer_fwd_x16(const float* x, const void* x16_in, int64_t B, int64_t T, int64_t in, int64_t H,
                          const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, float* y,
                          float* ws, void* stream) {
  SRK_API_BEGIN
  if (int rc = srk::check_dims(B, T, in, H)) return rc;
  SRK_REQUIRE(x && w_ih && w_hh && b_ih && b_hh && y && ws, SRK_ERR_INVALID, "gru_fwd: null pointer");
  hipStream_t s = srk::as_stream(stream);
  float* gi = ws;
  float* gates = ws + B * T * 6 * H;
  uint16_t* y16 = nullptr;
  if (use_h16(B, T, in, H)) {   // 16-bit operands in memory: x, W_ih rounded once, h written by the kernel
    const int64_t in8 = in8_of(in), BT = B * T;
    uint16_t* x16 = reinterpret_cast<uint16_t*>(ws + pad_end(B, T, in, H, 0));
    uint16_t* w16 = x16 + 2 * up64(BT * in8 / 2 + 1);
    y16 = w16 + 2 * up64(6 * H * in8 / 2 + 1);
    // x16_in: the producer's copy of x (the previous layer's y16), used as it is: in == in8 only
    SRK_REQUIRE(!x16_in || (in8 == in && reinterpret_cast<uintptr_t>(x16_in) % 16 == 0), SRK_ERR_INVALID,
                "gru_fwd: a ready 16-bit x needs in % 8 == 0 and 16-B alignment");
    if (x16_in) x16 = const_cast<uint16_t*>(static_cast<const uint16_t*>(x16_in));
    else if (int rc = srk::to16(x, BT, in, x16, in8, s)) return rc;
    const bool fuse = in <= srk::kFusedIn;   // the kernel projects the input itself (no gi GEMM)
    // W16: the gi GEMM's operand; with the fused projection only the backward's dx needs it (rounded there)
    if (!fuse) {
      if (int rc = srk::to16(w_ih, 6 * H, in, w16, in8, s)) return rc;
      GemmDesc g;   // gi[B*T, 6H] = x16 * W16^T + b_ih
      g.M = BT; g.N = 6 * H; g.K = in8;
      g.A16 = x16; g.lda = in8;
      g.B16 = w16; g.ldb = in8; g.tb = true;
      g.C = gi; g.ldc = 6 * H;
      g.bias = b_ih; g.bias_mode = 1;
      if (int rc = srk::gemm_f32(g, s)) return rc;
    }
    srk::GruPArgs p{};
    p.B = (int)B; p.T = (int)T; p.H = (int)H;
    p.gi = gi; p.w_hh = w_hh; p.b_hh = b_hh; p.y = y; p.gates = gates; p.y16 = y16;
    if (fuse) { p.x_in = x; p.w_ih = w_ih; p.b_ih = b_ih; p.in = (int)in; }
    p.xbuf = ws + fwd_xbuf_off(B, T, H);
    p.counters = reinterpret_cast<unsigned*>(ws + fwd_counter_off(B, T, H));
    return srk::gru_persistent_launch(p, false, s);
  }
  const float* xa = x;
  const float* wa = w_ih;
  int64_t ink = in;
  if (srk::padded_in(in)) {   // zero-pad the input width to a multiple of 4 (vector GEMM paths)
    ink = srk::pad4(in);
    float* xp = ws + pad_off(B, T, H, 0);
    float* wp = xp + B * T * ink;
    if (int rc = srk::pad_cols(x, B * T, in, xp, s)) return rc;
    if (int rc = srk::pad_cols(w_ih, 6 * H, in, wp, s)) return rc;
    xa = xp;
    wa = wp;
  }
  // both directions of the layer persistent or neither: the persistent fp32 kernels hand the saved
  // gates over unit-interleaved, the per-step kernels in the plain layout
  const bool persistent = srk::g_opt_gru_persistent && srk::gru_persistent_supported(B, T, H, false) &&
                          srk::gru_persistent_supported(B, T, H, true);
  const bool fuse = persistent && in <= srk::kFusedIn;   // the kernel projects the input itself
  if (!fuse) {
    GemmDesc g;   // gi[B*T, 6H] = x[B*T, in] * W_ih_cat[6H, in]^T + b_ih_cat
    g.M = B * T; g.N = 6 * H; g.K = ink;
    g.A = xa; g.lda = ink;
    g.B = wa; g.ldb = ink; g.tb = true;
    g.C = gi; g.ldc = 6 * H;
    g.bias = b_ih; g.bias_mode = 1;
    if (int rc = srk::gemm_f32(g, s)) return rc;
  }
  if (persistent) {
    srk::GruPArgs p{};
    p.B = (int)B; p.T = (int)T; p.H = (int)H;
    p.gi = gi; p.w_hh = w_hh; p.b_hh = b_hh; p.y = y; p.gates = gates;
    if (fuse) { p.x_in = x; p.w_ih = w_ih; p.b_ih = b_ih; p.in = (int)in; }
    p.xbuf = ws + fwd_xbuf_off(B, T, H);
    p.counters = reinterpret_cast<unsigned*>(ws + fwd_counter_off(B, T, H));
    return srk::gru_persistent_launch(p, false, s);
  }
  srk::GruArgs a{};
  a.B = (int)B; a.T = (int)T; a.H = (int)H; a.in = (int)in;
  a.y_in = y; a.y = y; a.gi = gi; a.w_hh = w_hh; a.b_hh = b_hh; a.gates = gates;
  a.G = (int)((B + srk::kRows - 1) / srk::kRows);
  a.S = (int)(H / srk::kUnits);
  const dim3 grid((unsigned)(2 * a.G * a.S));
  for (int step = 0; step < T; ++step) {
    srk::ProfScope prof("gru_fwd_step", s, step > 0 ? 2.0 * 2.0 * (double)B * 3 * H * H : 0.0);   // 2 dirs x [B,H]x[H,3H]
    hipLaunchKernelGGL(srk::gru_fwd_step_kernel, grid, dim3(256), 0, s, a, step);
  }
  SRK_CHECK_HIP(hipGetLastError());
  return SRK_OK;
  SRK_API_END
}

int srk_gru_layer_bwd(const float* x, int64_t B, int64_t T, int64_t in, int64_t H, const float* w_ih,
                      const float* w_hh, const float* y, const float* ws_fwd, const float* dy, float* dx,
                      float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, int accumulate, float* ws,
                      void* stream) {
  return srk_gru_layer_bwd_x16(x, nullptr, B, T, in, H, w_ih, w_hh, y, ws_fwd, dy, dx, dw_ih, dw_hh, db_ih, db_hh,
                               accumulate, ws, stream);
}

int srk_gru_layer_bwd_x16(const float* x, const void* x16_in, int64_t B, int64_t T, int64_t in, int64_t H,
                          const float* w_ih, const float* w_hh, const float* y, const float* ws_fwd, const float* dy,
                          float* dx, float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, int accumulate,
                          float* ws, void* stream) {
  SRK_API_BEGIN
  if (int rc = srk::check_dims(B, T, in, H)) return rc;
  SRK_REQUIRE(x && w_ih && w_hh && y && ws_fwd && dy && dw_ih && dw_hh && db_ih && db_hh && ws, SRK_ERR_INVALID,
              "gru_bwd: null pointer");
  hipStream_t s = srk::as_stream(stream);
  const int64_t BT = B * T;
  if (use_h16(B, T, in, H)) {
    // 16-bit path: the kernel writes dgi16 / dgh16 (aliasing the fp32 dgi region) and the bias-
    // gradient partials; every GEMM reads 16-bit operands (x16 / W16 / y16 from the forward).
    const int64_t in8 = in8_of(in);
    const uint16_t* x16 = reinterpret_cast<const uint16_t*>(ws_fwd + pad_end(B, T, in, H, 0));
    const uint16_t* w16 = x16 + 2 * up64(BT * in8 / 2 + 1);
    const uint16_t* y16 = w16 + 2 * up64(6 * H * in8 / 2 + 1);
    if (x16_in) x16 = static_cast<const uint16_t*>(x16_in);   // the forward's ready copy (srk_gru_layer_fwd_x16)
    uint16_t* dgi16 = reinterpret_cast<uint16_t*>(ws);
    uint16_t* dgh16 = dgi16 + BT * 6 * H;
    float* part = ws + pad_end(B, T, in, H, 1);
    const int64_t chunks = (B + 255) / 256;
    float* dwpad = part + up64(chunks * 8 * 2 * 4 * H);
    float* dxpad = dwpad + up64(6 * H * in8);
    srk::GruPArgs p{};
    p.B = (int)B; p.T = (int)T; p.H = (int)H;
    p.w_hh = w_hh; p.y_in = y; p.gates = const_cast<float*>(ws_fwd + BT * 6 * H); p.dy = dy;
    p.dgi16 = dgi16; p.dgh16 = dgh16; p.dbias = part;
    p.xbuf = ws + bwd_xbuf_off(B, T, H);
    p.counters = reinterpret_cast<unsigned*>(ws + bwd_counter_off(B, T, H));
    int rc;
    // the recurrent weight gradient accumulated inside the recurrence kernel (partials per row group)
    const int dw_parts = srk::gru_dwhh_fused_parts(B, T);
    if (dw_parts) {
      if ((rc = srk::gru_scratch((size_t)dw_parts * 2 * 3 * H * H, &p.dw_part))) return rc;
      p.y16_in = y16;
    }
    if ((rc = srk::gru_persistent_launch(p, true, s))) return rc;
    const int prows = srk::gru_bias_part_rows(B);
    if (dw_parts) {   // dW_hh and the bias gradients from their partials: one launch
      const int64_t per_dir = 3 * H * H, n4 = 2 * per_dir / 4;
      const int dw_blocks = (int)((n4 + 255) / 256);
      srk::ProfScope prof("gru_dwhh_reduce", s, 4.0 * (dw_parts + 2) * 2 * per_dir);
      hipLaunchKernelGGL(srk::dwhh_dbias_reduce_kernel, dim3((unsigned)(dw_blocks + (6 * H + 255) / 256)), dim3(256),
                         0, s, p.dw_part, dw_parts, (int)B, per_dir, dw_hh, (int)accumulate, dw_blocks, part,
                         (int)(chunks * (256 / prows)), (int)H, prows, db_ih, db_hh);
    } else {
      hipLaunchKernelGGL(srk::dbias_reduce_kernel, dim3((unsigned)((6 * H + 255) / 256)), dim3(256), 0, s, part,
                         (int)(chunks * (256 / prows)), (int)B, (int)H, prows, db_ih, db_hh, accumulate);
    }
    SRK_CHECK_HIP(hipGetLastError());
    const float beta = accumulate ? 1.f : 0.f;
    {  // dW_ih [6H, in] = dgi16^T x16
      GemmDesc g;
      g.M = 6 * H; g.N = in8; g.K = BT;
      g.A16 = dgi16; g.lda = 6 * H; g.ta = true;
      g.B16 = x16; g.ldb = in8;
      g.C = in8 == in ? dw_ih : dwpad; g.ldc = in8; g.beta = in8 == in ? beta : 0.f;
      if ((rc = srk::gemm_f32(g, s))) return rc;
      if (in8 != in) {
        const int64_t n = 6 * H * in;
        hipLaunchKernelGGL(srk::unpad_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dwpad, 6 * H,
                           (int)in8, dw_ih, (int)in, (int)accumulate);
        SRK_CHECK_HIP(hipGetLastError());
      }
    }
    {   // dW_hh[dir] = dgh16[dir]^T h_prev16 (edge rows of dgh16 are zero), both directions in ONE
        // batched launch: dir 0 pairs dgh16 row r + 1 with y16 row r, dir 1 dgh16 row r with y16 row
        // r + 1 (its reverse half); a 24-tile grid split 10 ways fills the CUs where two 12-tile
        // launches ran one after the other
      GemmDesc g;
      g.M = 3 * H; g.N = H; g.K = BT - 1;
      g.ta = true; g.lda = 3 * H; g.ldb = 2 * H;
      g.A16 = dgh16 + 3 * H;                 // dir 1: dgh16 + BT 3H
      g.B16 = y16;                           // dir 1: y16 + 3H (row 1, reverse half)
      g.C = dw_hh; g.ldc = H; g.beta = beta;
      g.batch = 2; g.sA = BT * 3 * H - 3 * H; g.sB = 3 * H; g.sC = 3 * H * H;
      if (dw_parts) {
        // done: the recurrence kernel accumulated it (dwhh_dbias_reduce_kernel above)
      } else if (g.K > 0 && srk::g_opt_gru_dwhh_batched) {
        if ((rc = srk::gemm_f32(g, s))) return rc;
      } else if (g.K > 0) {   // one launch per direction (A/B and tests)
        g.batch = 1;
        for (int dir = 0; dir < 2; ++dir, g.A16 += g.sA, g.B16 += g.sB, g.C += g.sC)
          if ((rc = srk::gemm_f32(g, s))) return rc;
      } else if (!accumulate) {
        SRK_CHECK_HIP(hipMemsetAsync(g.C, 0, sizeof(float) * 2 * 3 * H * H, s));
      }
    }
    if (dx) {   // dx [BT, in] = dgi16 W16
      if (in <= srk::kFusedIn) {   // the fused-projection forward left W16 unwritten: round it here
        if ((rc = srk::to16(w_ih, 6 * H, in, const_cast<uint16_t*>(w16), in8, s))) return rc;
      }
      GemmDesc g;
      g.M = BT; g.N = in8; g.K = 6 * H;
      g.A16 = dgi16; g.lda = 6 * H;
      g.B16 = w16; g.ldb = in8;
      g.C = in8 == in ? dx : dxpad; g.ldc = in8;
      if ((rc = srk::gemm_f32(g, s))) return rc;
      if (in8 != in) {
        const int64_t n = BT * in;
        hipLaunchKernelGGL(srk::unpad_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dxpad, BT,
                           (int)in8, dx, (int)in, 0);
        SRK_CHECK_HIP(hipGetLastError());
      }
    }
    return SRK_OK;
  }
  float* dgi = ws;
  float* dgh = dgi + BT * 6 * H;
  float* dgh_edge = dgh + 2 * BT * 3 * H;
  float* dhz = dgh_edge + 2 * B * 3 * H;
  srk::GruArgs a{};
  a.B = (int)B; a.T = (int)T; a.H = (int)H; a.in = (int)in;
  a.y_in = y; a.w_hh = w_hh; a.gates = const_cast<float*>(ws_fwd + BT * 6 * H);
  a.dy = dy; a.dgi = dgi; a.dgh = dgh; a.dgh_edge = dgh_edge; a.dhz = dhz;
  a.G = (int)((B + srk::kRows - 1) / srk::kRows);
  a.S = (int)(H / srk::kUnits);
  if (srk::g_opt_gru_persistent && srk::gru_persistent_supported(B, T, H, false) &&
      srk::gru_persistent_supported(B, T, H, true)) {   // as the forward decided (the gates' layout)
    srk::GruPArgs p{};
    p.B = (int)B; p.T = (int)T; p.H = (int)H;
    p.w_hh = w_hh; p.y_in = y; p.gates = a.gates; p.dy = dy; p.dgi = dgi; p.dgh = dgh; p.dgh_edge = dgh_edge;
    p.xbuf = ws + bwd_xbuf_off(B, T, H);
    p.counters = reinterpret_cast<unsigned*>(ws + bwd_counter_off(B, T, H));
    if (int rc = srk::gru_persistent_launch(p, true, s)) return rc;
  } else {
  const dim3 grid((unsigned)(2 * a.G * a.S));
  for (int step = 0; step < T; ++step) {
    srk::ProfScope prof("gru_bwd_step", s, step > 0 ? 2.0 * 2.0 * (double)B * 3 * H * H : 0.0);   // 2 dirs x [B,3H]x[3H,H]
    hipLaunchKernelGGL(srk::gru_bwd_step_kernel, grid, dim3(256), 0, s, a, step);
  }
  SRK_CHECK_HIP(hipGetLastError());
  }

  int rc;
  const float beta = accumulate ? 1.f : 0.f;   // autograd .grad accumulation in the GEMM epilogues
  const bool pad = srk::padded_in(in);
  const int64_t in4 = srk::pad4(in);
  float* wpad = pad ? ws + pad_off(B, T, H, 1) : nullptr;   // [6H][in4]
  float* dwpad = pad ? wpad + 6 * H * in4 : nullptr;         // [6H][in4]
  float* dxpad = pad ? dwpad + 6 * H * in4 : nullptr;        // [BT][in4]
  {  // dW_ih_cat[6H, in] = dgi^T [6H, BT] * x [BT, in]; db_ih fused as the row sums of dgi^T
    GemmDesc g;
    g.M = 6 * H; g.N = pad ? in4 : in; g.K = BT;
    g.A = dgi; g.lda = 6 * H; g.ta = true;
    g.B = pad ? ws_fwd + pad_off(B, T, H, 0) : x; g.ldb = pad ? in4 : in;   // the forward's padded x
    g.C = pad ? dwpad : dw_ih; g.ldc = pad ? in4 : in; g.beta = pad ? 0.f : beta;
    g.rowsum = db_ih; g.rowsum_beta = beta;
    if ((rc = srk::gemm_f32(g, s))) return rc;
    if (pad) {
      const int64_t n = 6 * H * in;
      hipLaunchKernelGGL(srk::unpad_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dwpad, 6 * H,
                         (int)in4, dw_ih, (int)in, (int)accumulate);
      SRK_CHECK_HIP(hipGetLastError());
    }
  }
  {
    // dW_hh[dir][3H, H] = sum_(b,t) dgh[b][t]^T h_prev[b][t]; h_prev of row (b,t) is y row (b,t-1)
    // (dir 0) or (b,t+1) (dir 1); the edge rows of dgh are zero so the batch seams contribute 0.
    // db_hh = row sums of dgh^T (fused) + the edge rows kept aside in dgh_edge.  Both directions run
    // as ONE batch-2 launch (dir 1 = dir 0's operands + sA / sB; option gru_dwhh_batched).
    GemmDesc g;
    g.M = 3 * H; g.N = H; g.K = BT - 1;
    g.ta = true; g.lda = 3 * H; g.ldb = 2 * H;
    g.A = dgh + 3 * H;      // dir 1: dgh + BT 3H
    g.B = y;                // dir 1: y + 3H (row 1, reverse half)
    g.C = dw_hh; g.ldc = H; g.beta = beta;
    g.rowsum = db_hh; g.rowsum_beta = beta;
    g.batch = 2; g.sA = BT * 3 * H - 3 * H; g.sB = 3 * H; g.sC = 3 * H * H; g.sRS = 3 * H;
    // (the batched row sums exist on the ping-pong kernel only: 16-B rows, 32-bit buffer offsets)
    const bool batched = srk::g_opt_gru_dwhh_batched && srk::gemm_f32_batched_rowsum_ok(g);
    if (g.K > 0 && batched) {
      if ((rc = srk::gemm_f32(g, s))) return rc;
    } else if (g.K > 0) {
      g.batch = 1;
      for (int dir = 0; dir < 2; ++dir, g.A += g.sA, g.B += g.sB, g.C += g.sC, g.rowsum += g.sRS)
        if ((rc = srk::gemm_f32(g, s))) return rc;
    } else if (!accumulate) {
      SRK_CHECK_HIP(hipMemsetAsync(dw_hh, 0, sizeof(float) * 2 * 3 * H * H, s));
      SRK_CHECK_HIP(hipMemsetAsync(db_hh, 0, sizeof(float) * 2 * 3 * H, s));
    }
    for (int dir = 0; dir < 2; ++dir)
      if ((rc = srk::colsum_f32(dgh_edge + (size_t)dir * B * 3 * H, B, 3 * H, 3 * H, db_hh + dir * 3 * H, 1.f, s)))
        return rc;
  }
  if (dx) {  // dx[BT, in] = dgi[BT, 6H] * W_ih_cat[6H, in]
    GemmDesc g;
    g.M = BT; g.N = pad ? in4 : in; g.K = 6 * H;
    g.A = dgi; g.lda = 6 * H;
    if (pad && (rc = srk::pad_cols(w_ih, 6 * H, in, wpad, s))) return rc;
    g.B = pad ? wpad : w_ih; g.ldb = pad ? in4 : in;
    g.C = pad ? dxpad : dx; g.ldc = pad ? in4 : in;
    if ((rc = srk::gemm_f32(g, s))) return rc;
    if (pad) {
      const int64_t n = BT * in;
      hipLaunchKernelGGL(srk::unpad_cols_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dxpad, BT,
                         (int)in4, dx, (int)in, 0);
      SRK_CHECK_HIP(hipGetLastError());
    }
  }
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
