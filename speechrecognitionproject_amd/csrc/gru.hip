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

}  // namespace
}  // namespace srk

using srk::GemmDesc;

extern "C" {

// Both workspaces end with a 64-float-aligned block of kCounterFloats arrival counters (the
// persistent recurrence kernels' step ordering; see gru_persistent.hip).
// Before them, 64-float aligned, the persistent kernels' hand-off ping-pong buffer in MFMA-fragment
// order (fwd: h [2 dir][2][rows][H], bwd: dg [2 dir][2][rows][3H]).
static int64_t fwd_xbuf_off(int64_t B, int64_t T, int64_t H) { return (B * T * 6 * H + 2 * T * B * 4 * H + 63) / 64 * 64; }
static int64_t bwd_xbuf_off(int64_t B, int64_t T, int64_t H) {
  return (B * T * 6 * H + 2 * B * T * 3 * H + 2 * B * 3 * H + 2 * B * H + 63) / 64 * 64;
}
// (rows padded to the 64-row groups of one launch chunk: <= 256 rows, or B rounded up to 64)
static int64_t xbuf_rows(int64_t B) { return std::min<int64_t>((B + 63) / 64 * 64, 256); }
static int64_t fwd_counter_off(int64_t B, int64_t T, int64_t H) { return fwd_xbuf_off(B, T, H) + 4 * xbuf_rows(B) * H; }
static int64_t bwd_counter_off(int64_t B, int64_t T, int64_t H) { return bwd_xbuf_off(B, T, H) + 12 * xbuf_rows(B) * H; }

int64_t srk_gru_workspace_floats(int64_t B, int64_t T, int64_t in, int64_t H, int backward) {
  (void)in;
  return (backward ? bwd_counter_off(B, T, H) : fwd_counter_off(B, T, H)) + srk::kCounterFloats + 64;
}

int srk_gru_layer_fwd(const float* x, int64_t B, int64_t T, int64_t in, int64_t H, const float* w_ih,
                      const float* w_hh, const float* b_ih, const float* b_hh, float* y, float* ws, void* stream) {
  SRK_API_BEGIN
  if (int rc = srk::check_dims(B, T, in, H)) return rc;
  SRK_REQUIRE(x && w_ih && w_hh && b_ih && b_hh && y && ws, SRK_ERR_INVALID, "gru_fwd: null pointer");
  hipStream_t s = srk::as_stream(stream);
  float* gi = ws;
  float* gates = ws + B * T * 6 * H;
  GemmDesc g;   // gi[B*T, 6H] = x[B*T, in] * W_ih_cat[6H, in]^T + b_ih_cat
  g.M = B * T; g.N = 6 * H; g.K = in;
  g.A = x; g.lda = in;
  g.B = w_ih; g.ldb = in; g.tb = true;
  g.C = gi; g.ldc = 6 * H;
  g.bias = b_ih; g.bias_mode = 1;
  if (int rc = srk::gemm_f32(g, s)) return rc;
  if (srk::g_opt_gru_persistent && srk::gru_persistent_supported(B, T, H, false)) {
    srk::GruPArgs p{};
    p.B = (int)B; p.T = (int)T; p.H = (int)H;
    p.gi = gi; p.w_hh = w_hh; p.b_hh = b_hh; p.y = y; p.gates = gates;
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
  SRK_API_BEGIN
  if (int rc = srk::check_dims(B, T, in, H)) return rc;
  SRK_REQUIRE(x && w_ih && w_hh && y && ws_fwd && dy && dw_ih && dw_hh && db_ih && db_hh && ws, SRK_ERR_INVALID,
              "gru_bwd: null pointer");
  hipStream_t s = srk::as_stream(stream);
  const int64_t BT = B * T;
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
  if (srk::g_opt_gru_persistent && srk::gru_persistent_supported(B, T, H, true)) {
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
  {  // dW_ih_cat[6H, in] = dgi^T [6H, BT] * x [BT, in]; db_ih fused as the row sums of dgi^T
    GemmDesc g;
    g.M = 6 * H; g.N = in; g.K = BT;
    g.A = dgi; g.lda = 6 * H; g.ta = true;
    g.B = x; g.ldb = in;
    g.C = dw_ih; g.ldc = in; g.beta = beta;
    g.rowsum = db_ih; g.rowsum_beta = beta;
    if ((rc = srk::gemm_f32(g, s))) return rc;
  }
  for (int dir = 0; dir < 2; ++dir) {
    // dW_hh[dir][3H, H] = sum_(b,t) dgh[b][t]^T h_prev[b][t]; h_prev of row (b,t) is y row (b,t-1)
    // (dir 0) or (b,t+1) (dir 1); the edge rows of dgh are zero so the batch seams contribute 0.
    // db_hh = row sums of dgh^T (fused) + the edge rows kept aside in dgh_edge.
    const float* dg = dgh + (size_t)dir * BT * 3 * H;
    float* dbh = db_hh + dir * 3 * H;
    GemmDesc g;
    g.M = 3 * H; g.N = H; g.K = BT - 1;
    g.ta = true; g.lda = 3 * H; g.ldb = 2 * H;
    g.A = dir == 0 ? dg + 3 * H : dg;
    g.B = dir == 0 ? y + dir * H : y + 2 * H + dir * H;
    g.C = dw_hh + (size_t)dir * 3 * H * H; g.ldc = H; g.beta = beta;
    g.rowsum = dbh; g.rowsum_beta = beta;
    if (g.K > 0) {
      if ((rc = srk::gemm_f32(g, s))) return rc;
    } else if (!accumulate) {
      SRK_CHECK_HIP(hipMemsetAsync(g.C, 0, sizeof(float) * 3 * H * H, s));
      SRK_CHECK_HIP(hipMemsetAsync(dbh, 0, sizeof(float) * 3 * H, s));
    }
    if ((rc = srk::colsum_f32(dgh_edge + (size_t)dir * B * 3 * H, B, 3 * H, 3 * H, dbh, 1.f, s))) return rc;
  }
  if (dx) {  // dx[BT, in] = dgi[BT, 6H] * W_ih_cat[6H, in]
    GemmDesc g;
    g.M = BT; g.N = in; g.K = 6 * H;
    g.A = dgi; g.lda = 6 * H;
    g.B = w_ih; g.ldb = in;
    g.C = dx; g.ldc = in;
    if ((rc = srk::gemm_f32(g, s))) return rc;
  }
  return SRK_OK;
  SRK_API_END
}

}  // extern "C"
