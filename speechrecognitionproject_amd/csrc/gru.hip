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
#include "gemm.h"

namespace srk {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBMB = 32;   // batch rows per workgroup
constexpr int kBJ = 32;    // hidden units per workgroup
constexpr int kBK = 32;    // k per LDS stage

struct GruArgs {
  int B, T, H, in;
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

// ------------------------------------------------------------------ forward step
__global__ __launch_bounds__(256) void gru_fwd_step_kernel(GruArgs a, int step) {
  __shared__ float As[2][kBK][kBMB + 16];
  __shared__ float Bs[2][kBK][3 * kBJ + 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane >> 4, lc = lane & 15;
  const int rh = wave & 1, ch = wave >> 1;
  const int dir = blockIdx.z;
  const int B = a.B, T = a.T, H = a.H;
  const int t = dir == 0 ? step : T - 1 - step;
  const int tprev = dir == 0 ? t - 1 : t + 1;
  const int b0 = blockIdx.x * kBMB, j0 = blockIdx.y * kBJ;
  const float* __restrict__ W = a.w_hh + (size_t)dir * 3 * H * H;

  f32x4 acc[3];
#pragma unroll
  for (int g = 0; g < 3; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (step > 0) {
    // A = h_prev rows (y[b][tprev][dir*H + k]), B = W_hh rows {g*H + j0 + jj}
    float4 ra, rb[3];
    auto load = [&](int k0) {
      {
        const int row = tid >> 3, kq = (tid & 7) * 4;
        const int b = b0 + row;
        ra = b < B ? *reinterpret_cast<const float4*>(a.y_in + ((size_t)b * T + tprev) * 2 * H + dir * H + k0 + kq)
                   : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int vi = tid + i * 256;
        const int c = vi >> 3, kq = (vi & 7) * 4;
        const int g = c / kBJ, jj = c % kBJ;
        rb[i] = *reinterpret_cast<const float4*>(W + (size_t)(g * H + j0 + jj) * H + k0 + kq);
      }
    };
    auto store = [&](int buf) {
      {
        const int row = tid >> 3, kq = (tid & 7) * 4;
        As[buf][kq + 0][row] = ra.x; As[buf][kq + 1][row] = ra.y;
        As[buf][kq + 2][row] = ra.z; As[buf][kq + 3][row] = ra.w;
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int vi = tid + i * 256;
        const int c = vi >> 3, kq = (vi & 7) * 4;
        Bs[buf][kq + 0][c] = rb[i].x; Bs[buf][kq + 1][c] = rb[i].y;
        Bs[buf][kq + 2][c] = rb[i].z; Bs[buf][kq + 3][c] = rb[i].w;
      }
    };
    const int nk = H / kBK;
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load((kt + 1) * kBK);
#pragma unroll
      for (int kk = 0; kk < kBK; kk += 4) {
        const float av = As[cur][kk + lr][rh * 16 + lc];
#pragma unroll
        for (int g = 0; g < 3; ++g)
          acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, Bs[cur][kk + lr][g * kBJ + ch * 16 + lc], acc[g], 0, 0, 0);
      }
      if (kt + 1 < nk) store(cur ^ 1);
      __syncthreads();
    }
  }

  // epilogue: lane owns rows rh*16 + 4*lr + r, unit j = j0 + ch*16 + lc, all three gates
  const int j = j0 + ch * 16 + lc;
  const float bhr = a.b_hh[dir * 3 * H + j], bhz = a.b_hh[dir * 3 * H + H + j], bhn = a.b_hh[dir * 3 * H + 2 * H + j];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = b0 + rh * 16 + lr * 4 + r;
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
__global__ __launch_bounds__(256) void gru_bwd_step_kernel(GruArgs a, int step) {
  __shared__ float As[2][kBK][kBMB + 16];
  __shared__ float Bs[2][kBK][kBJ + 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane >> 4, lc = lane & 15;
  const int rh = wave & 1, ch = wave >> 1;
  const int dir = blockIdx.z;
  const int B = a.B, T = a.T, H = a.H;
  const int t = dir == 0 ? T - 1 - step : step;          // time processed now
  const int tnext = dir == 0 ? t + 1 : t - 1;           // processed by the previous step
  const int tprev = dir == 0 ? t - 1 : t + 1;           // h_prev source
  const bool edge = (step == T - 1);                    // h_prev = 0 here
  const int b0 = blockIdx.x * kBMB, j0 = blockIdx.y * kBJ;
  const float* __restrict__ W = a.w_hh + (size_t)dir * 3 * H * H;
  const float* __restrict__ dghn = a.dgh + (size_t)dir * B * T * 3 * H;   // [B][T][3H] of this dir

  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  if (step > 0) {
    // dh_rec[b][j] = sum_c dgh[b][tnext][c] * W_hh[c][j],  c in [0, 3H)
    float4 ra, rb;
    auto load = [&](int k0) {
      const int row = tid >> 3, q = (tid & 7) * 4;
      const int b = b0 + row;
      ra = b < B ? *reinterpret_cast<const float4*>(dghn + ((size_t)b * T + tnext) * 3 * H + k0 + q)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
      rb = *reinterpret_cast<const float4*>(W + (size_t)(k0 + row) * H + j0 + q);
    };
    auto store = [&](int buf) {
      const int row = tid >> 3, q = (tid & 7) * 4;
      As[buf][q + 0][row] = ra.x; As[buf][q + 1][row] = ra.y;
      As[buf][q + 2][row] = ra.z; As[buf][q + 3][row] = ra.w;
      *reinterpret_cast<float4*>(&Bs[buf][row][q]) = rb;
    };
    const int nk = 3 * H / kBK;
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load((kt + 1) * kBK);
#pragma unroll
      for (int kk = 0; kk < kBK; kk += 4)
        acc[(kk >> 2) & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(As[cur][kk + lr][rh * 16 + lc],
                                                                   Bs[cur][kk + lr][ch * 16 + lc],
                                                                   acc[(kk >> 2) & 1], 0, 0, 0);
      if (kt + 1 < nk) store(cur ^ 1);
      __syncthreads();
    }
  }

  const int j = j0 + ch * 16 + lc;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = b0 + rh * 16 + lr * 4 + r;
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
  SRK_REQUIRE(H % kBJ == 0 && H % kBK == 0, SRK_ERR_INVALID, "gru: hidden size must be a multiple of 32");
  SRK_REQUIRE(B * T * 6 * H < ((int64_t)1 << 40), SRK_ERR_INVALID, "gru: problem too large");
  return SRK_OK;
}

}  // namespace
}  // namespace srk

using srk::GemmDesc;

extern "C" {

int64_t srk_gru_workspace_floats(int64_t B, int64_t T, int64_t in, int64_t H, int backward) {
  (void)in;
  if (!backward) return B * T * 6 * H + 2 * T * B * 4 * H;
  return B * T * 6 * H + 2 * B * T * 3 * H + 2 * B * 3 * H + 2 * B * H;
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
  srk::GruArgs a{};
  a.B = (int)B; a.T = (int)T; a.H = (int)H; a.in = (int)in;
  a.y_in = y; a.y = y; a.gi = gi; a.w_hh = w_hh; a.b_hh = b_hh; a.gates = gates;
  const dim3 grid((unsigned)((B + srk::kBMB - 1) / srk::kBMB), (unsigned)(H / srk::kBJ), 2);
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
                      float* dw_ih, float* dw_hh, float* db_ih, float* db_hh, float* ws, void* stream) {
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
  const dim3 grid((unsigned)((B + srk::kBMB - 1) / srk::kBMB), (unsigned)(H / srk::kBJ), 2);
  for (int step = 0; step < T; ++step) {
    srk::ProfScope prof("gru_bwd_step", s, step > 0 ? 2.0 * 2.0 * (double)B * 3 * H * H : 0.0);   // 2 dirs x [B,3H]x[3H,H]
    hipLaunchKernelGGL(srk::gru_bwd_step_kernel, grid, dim3(256), 0, s, a, step);
  }
  SRK_CHECK_HIP(hipGetLastError());

  int rc;
  {  // dW_ih_cat[6H, in] = dgi^T [6H, BT] * x [BT, in]
    GemmDesc g;
    g.M = 6 * H; g.N = in; g.K = BT;
    g.A = dgi; g.lda = 6 * H; g.ta = true;
    g.B = x; g.ldb = in;
    g.C = dw_ih; g.ldc = in;
    if ((rc = srk::gemm_f32(g, s))) return rc;
  }
  if ((rc = srk::colsum_f32(dgi, BT, 6 * H, 6 * H, db_ih, 0.f, s))) return rc;
  for (int dir = 0; dir < 2; ++dir) {
    // dW_hh[dir][3H, H] = sum_(b,t) dgh[b][t]^T h_prev[b][t]; h_prev of row (b,t) is y row (b,t-1)
    // (dir 0) or (b,t+1) (dir 1); the edge rows of dgh are zero so the batch seams contribute 0.
    const float* dg = dgh + (size_t)dir * BT * 3 * H;
    GemmDesc g;
    g.M = 3 * H; g.N = H; g.K = BT - 1;
    g.ta = true; g.lda = 3 * H; g.ldb = 2 * H;
    g.A = dir == 0 ? dg + 3 * H : dg;
    g.B = dir == 0 ? y + dir * H : y + 2 * H + dir * H;
    g.C = dw_hh + (size_t)dir * 3 * H * H; g.ldc = H;
    if (g.K > 0 && (rc = srk::gemm_f32(g, s))) return rc;
    if (g.K == 0) SRK_CHECK_HIP(hipMemsetAsync(g.C, 0, sizeof(float) * 3 * H * H, s));
    float* dbh = db_hh + dir * 3 * H;
    if ((rc = srk::colsum_f32(dg, BT, 3 * H, 3 * H, dbh, 0.f, s))) return rc;
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
