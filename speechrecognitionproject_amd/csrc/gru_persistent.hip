// K5, persistent form: ONE launch runs all T steps of a bidirectional GRU layer's recurrence
// (forward or backward), replacing the T per-step launches of gru.hip for the shapes the
// reference uses (H = 512; models/model_mfcc_bgru.py:25, model_spec_bgru.py:23,
// model_resnet_bgru.py:130).  Same arithmetic, same operand order, same outputs as the per-step
// kernels — only the schedule changes:
//
//  * each workgroup owns (direction, 64 batch rows, 16 hidden units) for the whole sequence and
//    keeps ITS slice of W_hh resident in LDS (fwd: the 3 x 16 gate rows x H, bwd: the 16 unit
//    columns x 3H) — ~97 KB per workgroup, 3 MB per direction, read from HBM once per layer
//    instead of once per step;
//  * the recurrent state crosses workgroups through a ping-pong buffer laid out in MFMA-FRAGMENT
//    order: for each 16-row block and 16-wide k block, the 64 lanes' float4 A-operands are one
//    contiguous 1 KB chunk ([group][row block][k block][lane][4]), so every consumer load is a fully
//    coalesced 1 KB wave access (the natural [row][k] layout puts 16 rows in each quarter-wave:
//    measured 3-4 us of load time per step, independent of caching); written write-through (`sc1`,
//    16 B per lane, after an LDS transpose) and read back with `sc1` loads (the outputs y / dgh get
//    plain stores for the later GEMMs); one agent-scope arrival counter per (direction,
//    64-row group) orders the steps (MI355X_MICROARCH.md "Valid forms", table row 1: one lane of
//    each storing workgroup adds after every storing wave drained; consumers poll with an `sc1`
//    load; every load of the handed-off bytes is an `sc1` load; one workgroup per CU);
//  * the register-resident carries (fwd: h_{t-1} of the lane's own cells, bwd: dh*z) never touch
//    memory.
//
// Co-residency: the grid (2 directions x 64-row groups x H/16 slices, <= one workgroup per CU)
// must be resident at once; the host checks the occupancy query against the CU count and falls
// back to the per-step kernels otherwise, and splits larger batches into 64*G-row chunk launches.
// Every spin is bounded: a workgroup that waits ~2 s gives up, bumps g_spin_timeouts (read by
// srk_spin_timeouts()) and raises the host-pinned health word, then carries on so a fault can never
// hang the GPU.  The results of that launch are invalid, so a timeout is FATAL to the caller:
// srk_health_check() (no device sync) returns SRK_ERR_TIMEOUT from then on; the optimizer step,
// training.py's loss flush and bench.py check it and raise.
#include <cstdlib>
#include <type_traits>
#include <mutex>
#include <utility>

#include "gru_internal.h"

namespace srk {

__device__ unsigned long long g_spin_timeouts = 0;

namespace {

typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = 64;     // batch rows per workgroup (4 waves x 16)
constexpr int kUnits = 16;    // hidden units per workgroup
constexpr int kSc1 = 16;      // buffer-instruction aux bit: sc1 (write-through / L1-bypass)
constexpr unsigned kSpinLimit = 1u << 24;   // x s_sleep(2) (~128 clk) ~= 2 s at 2.4 GHz

__device__ __forceinline__ v4f ld4(const float* p) { return *reinterpret_cast<const v4f*>(p); }
__device__ __forceinline__ void st4(float* p, v4f v) { *reinterpret_cast<v4f*>(p) = v; }
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
// 16-bit kernels: the hardware exp / reciprocal forms (v_exp_f32, v_rcp_f32: ~1 ulp, far inside the
// 16-bit operand tolerance) keep the cell epilogue short on the step-to-step chain; the fp32 kernels
// keep the libm forms.
__device__ __forceinline__ float sigmoid_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) { return 2.0f * sigmoid_fast(2.0f * x) - 1.0f; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ v4f ld4_sc1(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  return __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, kSc1));
}
__device__ __forceinline__ void st4_sc1(__amdgpu_buffer_rsrc_t r, unsigned byte_off, v4f v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, (int)byte_off, 0, kSc1);
}

// One lane of the workgroup waits until *cnt >= target (relaxed agent-scope = sc1 load), then
// the whole workgroup passes a barrier.  Bounded.
// A wait that gave up: count it and raise the host-visible health word (a vector store to
// host-coherent memory at system scope).
__device__ __forceinline__ void spin_gave_up(const GruPArgs& a) {
  atomicAdd(&g_spin_timeouts, 1ull);
  if (a.health) __hip_atomic_store(a.health, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void wait_count(const GruPArgs& a, unsigned* cnt, unsigned target) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins >= a.spin_limit) {
        spin_gave_up(a);
        break;
      }
    }
  }
  __syncthreads();
}

// Every storing wave drains its sc1 stores, the workgroup meets, one lane arrives.
__device__ __forceinline__ void arrive(unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-producer flags (a.flags): producer (dir, group, slice) stores step + 1 into ITS word of
// [2][G][32] after every storing wave drained (one lane, behind the workgroup barrier: an sc1
// store); the consumer's wave 0 polls all S words of its (dir, group) at once (lane i <-> slice i,
// sc1 loads) until every one is >= step, then the workgroup meets.  MI355X_MICROARCH.md "Valid
// forms" row 1 (a sharded flag, every shard polled).  Replaces the atomic add at the memory side.
__device__ __forceinline__ void sync_wait(const GruPArgs& a, unsigned* cnt, int dir, int group, int S, int step,
                                          bool local) {
  if (!a.flags && !local) {
    wait_count(a, cnt, (unsigned)S * step);
    return;
  }
  if (threadIdx.x < 64) {
    unsigned* f = a.counters + pw_flag64(dir, a.G, group, 0);
    const int lane = threadIdx.x;
    unsigned spins = 0;
    while (true) {
      const unsigned v = lane < S ? __hip_atomic_load(f + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0xffffffffu;
      if (__all(v >= (unsigned)step)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins >= a.spin_limit) {
        if (lane == 0) spin_gave_up(a);
        break;
      }
    }
  }
  __syncthreads();
}
__device__ __forceinline__ void sync_arrive(const GruPArgs& a, unsigned* cnt, int dir, int group, int slice, int step,
                                            bool local) {
  if (!a.flags && !local) {
    arrive(cnt);
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* f = a.counters + pw_flag64(dir, a.G, group, slice);
    if (local)   // XCD-local: a plain store, kept in the XCD's L2 where the consumers' sc1 polls read it
      __builtin_amdgcn_raw_buffer_store_b32((unsigned)(step + 1), rsrc(reinterpret_cast<const float*>(f)), 0, 0, 0);
    else
      __hip_atomic_store(f, (unsigned)(step + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Hand-off payload store: write-through (sc1) in the placement-independent protocol; a plain store
// in the XCD-local one (the line stays in the XCD's L2, where every consumer's sc1 load finds it).
__device__ __forceinline__ void st4_ho(__amdgpu_buffer_rsrc_t r, unsigned byte_off, v4f v, bool local) {
  if (local) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, (int)byte_off, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, (int)byte_off, 0, kSc1);
}

// Diagnostics (tools/gru_trace.py): thread 0 stamps s_memrealtime (100 MHz) at step start (0), after
// the arrival wait (1), after its MFMAs retired (2), after the cell epilogue (3) and after
// publishing (4).  Off (null) in production.
__device__ __forceinline__ void stamp(const GruPArgs& a, int step, int i) {
  if (a.trace && threadIdx.x == 0)
    a.trace[((size_t)blockIdx.x * a.T + step) * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

// Diagnostics: the workgroup's (direction, group) pair and slice, in trace slot 5 of its step 0.
__device__ __forceinline__ void trace_id(const GruPArgs& a, int dir, int group, int slice) {
  if (a.trace && threadIdx.x == 0)
    a.trace[(size_t)blockIdx.x * a.T * 8 + 5] = ((unsigned long long)(dir * a.G + group) << 8) | (unsigned)slice;
}

// (direction, group, slice) of this workgroup: the S slices of one (direction, group) pair are
// dealt to blocks of ONE XCD (blocks b, b+8, ... share an XCD under round-robin dispatch), so the
// handed-off rows stay in that XCD's L2.  Speed only; the protocol does not depend on it.
__device__ __forceinline__ void map_block(int G, int S, int& dir, int& group, int& slice) {
  const int nwg = 2 * G * S;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  const int pair = wgid / S;
  slice = wgid % S;
  dir = pair / G;
  group = pair % G;
}

// Placement.  Default: map_block (speed-only XCD affinity; every hand-off byte goes write-through,
// MI355X_MICROARCH.md "Valid forms" row 1, correct under any placement).  With xcd_local and a full
// 256-workgroup grid, a census first asks the hardware which XCD each workgroup runs on
// (HW_REG_XCC_ID) and hands out slots per XCD; when every XCD holds exactly 32 workgroups, XCD x
// runs (direction, group) pairs x * 32 / S .. (S slices per pair: one pair of 32 slices, or two of
// 16) — then producers and consumers of a pair provably share one L2, the
// hand-off bytes and flags are PLAIN stores that stay in that L2 (no write-through to the Infinity
// Cache and back) and consumers keep reading them with sc1 (L1-bypassing) loads.  Otherwise every
// workgroup (they all read the same final census) falls back to the default protocol.
__device__ __forceinline__ void place(const GruPArgs& a, int S, int& dir, int& group, int& slice, bool& local) {
  __shared__ int info[2];
  const int nwg = 2 * a.G * S;
  if (a.xcd_local && nwg == 256) {
    if (threadIdx.x == 0) {
      unsigned xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
      unsigned* cen = a.counters + kCensusOff;
      const unsigned slot = __hip_atomic_fetch_add(cen + xcc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // wait for the per-XCD counts themselves to add up to the grid: the counts only grow and sum
      // to nwg at most, so a sum of nwg means every count read in that pass is final (a separate
      // total counter would not order the per-XCD adds it counts)
      unsigned n[8], spins = 0;
      while (true) {
        unsigned sum = 0;
        for (int x = 0; x < 8; ++x) {
          n[x] = __hip_atomic_load(cen + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sum += n[x];
        }
        if (sum >= (unsigned)nwg) break;
        __builtin_amdgcn_s_sleep(2);
        if (++spins >= a.spin_limit) {
          spin_gave_up(a);
          break;
        }
      }
      bool even = true;
      for (int x = 0; x < 8; ++x) even = even && n[x] == (unsigned)(nwg / 8);
      info[0] = even ? (int)xcc : -1;
      info[1] = (int)slot;
    }
    __syncthreads();
    const int xcc = __builtin_amdgcn_readfirstlane(info[0]);
    if (xcc >= 0) {   // XCD x hosts pairs x * (32 / S) .. : 32 workgroups = 32 / S whole (direction, group) pairs
      const int slot = __builtin_amdgcn_readfirstlane(info[1]);
      const int pair = xcc * (32 / S) + slot / S;
      local = true;
      dir = pair / a.G;
      group = pair % a.G;
      slice = slot % S;
      return;
    }
  }
  local = false;
  map_block(a.G, S, dir, group, slice);
}

// The saved gates (r, z, n, W_hn h + b_hn) of a lane's 4 cells, stored AFTER the step's arrival:
// nothing in this launch reads them, so their write latency leaves the step-to-step chain.
__device__ __forceinline__ void store_gates(const GruPArgs& a, const float (&gsv)[4][4], int dir, int t, int brow0,
                                            int b_last, int j) {
  const int H = a.H;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = brow0 + r;
    if (b > b_last) continue;
    float* gs = a.gates + (((size_t)dir * a.T + t) * a.B + b) * 4 * H;
    gs[j] = gsv[r][0];
    gs[H + j] = gsv[r][1];
    gs[2 * H + j] = gsv[r][2];
    gs[3 * H + j] = gsv[r][3];
  }
}

// The 16-bit 32 x 32 kernels keep the saved gates unit-interleaved, [dir][t][b][H][4]: one 16-B store
// per cell here and one 16-B load in the backward kernel instead of four dword accesses each.
__device__ __forceinline__ void store_gates_il(const GruPArgs& a, const float (&gsv)[4][4], int dir, int t, int brow0,
                                               int b_last, int j) {
  const int H = a.H;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = brow0 + r;
    if (b > b_last) continue;
    float* gs = a.gates + (((size_t)dir * a.T + t) * a.B + b) * 4 * H;
    *reinterpret_cast<v4f*>(gs + 4 * j) = v4f{gsv[r][0], gsv[r][1], gsv[r][2], gsv[r][3]};
  }
}

// The input-projection gradients dgi (dar, daz, dan) of a lane's 4 cells, likewise after the arrival.
__device__ __forceinline__ void store_dgi(const GruPArgs& a, const float (&dv)[4][3], int dir, int t, int brow0,
                                          int b_last, int j) {
  const int H = a.H;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = brow0 + r;
    if (b > b_last) continue;
    float* dgi = a.dgi + ((size_t)b * a.T + t) * 6 * H + dir * 3 * H;
    dgi[j] = dv[r][0];
    dgi[H + j] = dv[r][1];
    dgi[2 * H + j] = dv[r][2];
  }
}

// ------------------------------------------------------------------ fused input projection
// For inputs of <= kFusedIn features the forward kernels compute the step's input projection for
// their 64 rows x 48 gate units on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: lane = (row lr,
// k-quad lq), the same output layout as the recurrent accumulators), from x_t (global, L2-resident)
// and an LDS copy of the W_ih slice, BEFORE the step's wait: it does not depend on h and runs in
// the hand-off latency.  RND rounds both operands to bf16 / fp16 first (the 16-bit kernels' GEMM
// semantics: 16-bit operands, fp32 accumulation).
constexpr int kXP = kFusedIn + 1;   // LDS pitch of the W_ih slice (odd: conflict-free column reads)

template <int RND>
__device__ __forceinline__ float rnd16(float v) {
  if (RND == 1) return (float)(__bf16)v;
  if (RND == 2) return (float)(_Float16)v;
  return v;
}

template <int RND>
__device__ __forceinline__ void stage_wih(const GruPArgs& a, float* Wx, int dir, int j0, int H) {
  const float* W = a.w_ih + (size_t)dir * 3 * H * a.in;
  for (int v = threadIdx.x; v < 3 * kUnits * kFusedIn; v += 256) {
    const int c = v / kFusedIn, k = v % kFusedIn, g = c / kUnits, jj = c % kUnits;
    Wx[c * kXP + k] = k < a.in ? rnd16<RND>(W[(size_t)(g * H + j0 + jj) * a.in + k]) : 0.f;
  }
}

// x_t of the lane's row (k = 4 m + lq); issued one step ahead so the loads are in flight during the
// previous step
__device__ __forceinline__ void load_x(const GruPArgs& a, int t, int brow, int lq, float (&xv)[kFusedIn / 4]) {
  const float* xr = a.x_in + ((size_t)brow * a.T + t) * a.in;
#pragma unroll
  for (int m = 0; m < kFusedIn / 4; ++m) {
    const int k = 4 * m + lq;
    xv[m] = (4 * m < a.in && k < a.in) ? xr[k] : 0.f;
  }
}

template <int RND>
__device__ __forceinline__ void fused_gi(const GruPArgs& a, const float* Wx, const float (&xv0)[kFusedIn / 4], int lr,
                                         int lq, float bir, float biz, float bin, float (&gr)[4], float (&gz)[4],
                                         float (&gn)[4]) {
  float xv[kFusedIn / 4];
#pragma unroll
  for (int m = 0; m < kFusedIn / 4; ++m) xv[m] = rnd16<RND>(xv0[m]);
  f32x4 ax[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int m = 0; m < kFusedIn / 4; ++m) {
    if (4 * m >= a.in) break;   // uniform
#pragma unroll
    for (int g = 0; g < 3; ++g)
      ax[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[m], Wx[(g * kUnits + lr) * kXP + 4 * m + lq], ax[g], 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    gr[r] = ax[0][r] + bir;
    gz[r] = ax[1][r] + biz;
    gn[r] = ax[2][r] + bin;
  }
}

// ------------------------------------------------------------------ forward
// LDS: W slice [48][H + 4] (gate g, unit jj -> row g*16 + jj), then the h transpose tile [64][20].
template <int H>
__global__ __launch_bounds__(256, 1) void gru_fwd_persistent_kernel(GruPArgs a) {
  constexpr int WP = H + 4, HTP = kUnits + 4, NKB = H / 16;
  constexpr int RNDX = 0;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ws = smem;
  float* hT = smem + 3 * kUnits * WP;
  float* Wx = hT + 64 * HTP;   // fused input projection: W_ih slice [48][kXP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
  int dir, group, slice;
  bool local;
  place(a, H / kUnits, dir, group, slice, local);
  trace_id(a, dir, group, slice);
  const int T = a.T, j0 = slice * kUnits, j = j0 + lr;
  const int b0 = a.b_begin + group * kRows;
  const int b_last = a.b_end - 1;
  unsigned* cnt = a.counters + pw_counter(dir, a.G, group);

  {  // this slice of W_hh[dir] -> LDS (read once per layer)
    const float* W = a.w_hh + (size_t)dir * 3 * H * H;
    for (int v = tid; v < 3 * kUnits * H / 4; v += 256) {
      const int c = v / (H / 4), kq = (v % (H / 4)) * 4, g = c / kUnits, jj = c % kUnits;
      st4(Ws + c * WP + kq, ld4(W + (size_t)(g * H + j0 + jj) * H + kq));
    }
  }
  const bool fused = a.x_in != nullptr;
  if (fused) stage_wih<RNDX>(a, Wx, dir, j0, H);
  float xnext[kFusedIn / 4];   // x of the next step (fused projection), loaded a step ahead
  if (fused) load_x(a, dir == 0 ? 0 : a.T - 1, min(a.b_begin + group * kRows + wave * 16 + lr, a.b_end - 1), lq, xnext);
  const float bir = fused ? a.b_ih[dir * 3 * H + j] : 0.f, biz = fused ? a.b_ih[dir * 3 * H + H + j] : 0.f,
              bin = fused ? a.b_ih[dir * 3 * H + 2 * H + j] : 0.f;
  const float bhr = a.b_hh[dir * 3 * H + j], bhz = a.b_hh[dir * 3 * H + H + j], bhn = a.b_hh[dir * 3 * H + 2 * H + j];
  __syncthreads();

  const int B = a.B;
  const int Gp = a.G;   // 64-row groups in this launch (the hand-off buffer is padded to Gp * 64 rows)
  const __amdgpu_buffer_rsrc_t rx = rsrc(a.xbuf + (size_t)dir * 2 * Gp * 64 * H);   // [2][Gp][4][H/16][64][4]
  float hreg[4] = {0.f, 0.f, 0.f, 0.f};                 // h_{t-1} of the lane's own 4 cells
  float gsv[4][4];                                      // this step's gates, stored after the arrival

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    const int tprev = dir == 0 ? t - 1 : t + 1;
    stamp(a, step, 0);
    float gr[4], gz[4], gn[4];
    if (fused) {   // this step's input projection, before the wait (independent of h)
      fused_gi<RNDX>(a, Wx, xnext, lr, lq, bir, biz, bin, gr, gz, gn);
      if (step + 1 < T) load_x(a, dir == 0 ? t + 1 : t - 1, min(b0 + wave * 16 + lr, b_last), lq, xnext);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {   // input projections of the lane's cells (written by an earlier launch)
        const int b = min(b0 + wave * 16 + lq * 4 + r, b_last);
        const float* gi = a.gi + ((size_t)b * T + t) * 6 * H + dir * 3 * H;
        gr[r] = gi[j];
        gz[r] = gi[H + j];
        gn[r] = gi[2 * H + j];
      }
    }
    f32x4 acc[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (step > 0) {
      sync_wait(a, cnt, dir, group, H / kUnits, step, local);
      stamp(a, step, 1);
      // h_{t-1}[row 16 wave + lr][k], k = 16 kb + 4 lq + s  (k-permuted: one b128 feeds 4 MFMAs)
      // fragment chunk (group, row block = wave, k block) of the previous step's buffer; lane = lane
      const unsigned base = (unsigned)(((((size_t)((step - 1) & 1) * Gp + group) * 4 + wave) * NKB * 64 + lane) * 16);
      // The 32 workgroups of a (direction, group) read the SAME 64 rows: each walks k starting at a
      // different block (rot = its slice) so they do not all hit the same L2 lines / channel at once
      // (measured: the hand-off loads, not the MFMAs, set the step time).  The k order is fixed per
      // slice, so results stay deterministic.
      const int rot = slice % NKB;
      v4f hv[NKB];
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) hv[kb] = ld4_sc1(rx, base + ((kb + rot) & (NKB - 1)) * 1024);
      __builtin_amdgcn_sched_barrier(0);   // all loads in flight before the first MFMA (no sinking)
      // W fragments one k-block ahead of their MFMAs (issued first, behind a hard scheduling fence,
      // so a block's MFMAs never wait on LDS); within a block the 12 MFMAs rotate over the three
      // gate accumulators (dependent issue distance 3 x 32 cycles > the 40-cycle latency), pinned
      // with scheduling groups (the default scheduler batches one accumulator).
      v4f wv[2][3];
#pragma unroll
      for (int g = 0; g < 3; ++g) wv[0][g] = ld4(Ws + (g * kUnits + lr) * WP + rot * 16 + 4 * lq);
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        const int c = kb & 1;
        if (kb + 1 < NKB) {
          const int kn = (kb + 1 + rot) & (NKB - 1);
#pragma unroll
          for (int g = 0; g < 3; ++g) wv[c ^ 1][g] = ld4(Ws + (g * kUnits + lr) * WP + kn * 16 + 4 * lq);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int g = 0; g < 3; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[kb][s], wv[c][g][s], acc[g], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 12; ++i) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (a.trace) {
        asm volatile("" ::"v"(acc[0][0]), "v"(acc[1][0]), "v"(acc[2][0]));
        stamp(a, step, 2);
      }
    }
    // cell epilogue: lane owns rows 16*wave + 4*lq + r, unit j
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wave * 16 + lq * 4 + r, b = b0 + rl;
      const float ghn = acc[2][r] + bhn;
      const float rg = sigmoidf_(gr[r] + (acc[0][r] + bhr));
      const float zg = sigmoidf_(gz[r] + (acc[1][r] + bhz));
      const float ng = tanhf(gn[r] + rg * ghn);
      const float h = (1.0f - zg) * ng + zg * hreg[r];
      hreg[r] = h;
      hT[rl * HTP + lr] = h;
      gsv[r][0] = rg;
      gsv[r][1] = zg;
      gsv[r][2] = ng;
      gsv[r][3] = ghn;
    }
    __syncthreads();
    stamp(a, step, 3);
    v4f hv4;
    const int yrl = tid >> 2, yuq = (tid & 3) * 4;
    {  // h_t -> the hand-off buffer (write-through): thread = (row tid/4, units 4*(tid%4) .. +3)
      hv4 = ld4(hT + yrl * HTP + yuq);
      if (step + 1 < T && b0 + yrl <= b_last)   // fragment slot (row block rl/16, k block = slice, lane = (uq/4)*16 + rl%16)
        st4_ho(rx, (unsigned)(((((size_t)(step & 1) * Gp + group) * 4 + (yrl >> 4)) * NKB * 64 + slice * 64 +
                                (yuq >> 2) * 16 + (yrl & 15)) * 16), hv4, local);
    }
    sync_arrive(a, cnt, dir, group, slice, step, local);   // waits for the hand-off stores only: y and the gates go out after it (no consumer in this launch)
    stamp(a, step, 4);
    if (b0 + yrl <= b_last) st4(a.y + ((size_t)(b0 + yrl) * T + t) * 2 * H + dir * H + j0 + yuq, hv4);
    store_gates_il(a, gsv, dir, t, b0 + wave * 16 + lq * 4, b_last, j);   // unit-interleaved: read by gru_bwd_persistent_kernel
  }
}

// ------------------------------------------------------------------ backward
// dh[b][j] = dy[b][t][dir, j] + sum_c dgh_next[b][c] W_hh[c][j] + (dh z)_next[b][j]
// LDS: W^T slice [16][3H + 4] (unit jj, gate row c), then the dg transpose tile [64][3][16 + 4].
template <int H>
__global__ __launch_bounds__(256, 1) void gru_bwd_persistent_kernel(GruPArgs a) {
  constexpr int WP = 3 * H + 4, DTP = kUnits + 4, NKB = 3 * H / 16, CH = 16;   // CH k-blocks per chunk
  static_assert(NKB % CH == 0, "chunking");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Wt = smem;
  float* dT = smem + kUnits * WP;   // [64][4][DTP]: dar, daz, dan * r (the hand-off / dgh), dan (dgi)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
  int dir, group, slice;
  bool local;
  place(a, H / kUnits, dir, group, slice, local);
  trace_id(a, dir, group, slice);
  const int T = a.T, B = a.B, j0 = slice * kUnits, j = j0 + lr;
  const int b0 = a.b_begin + group * kRows;
  const int b_last = a.b_end - 1;
  unsigned* cnt = a.counters + pw_counter(dir, a.G, group);

  {  // W_hh[dir][c][j0 .. j0+15] for all 3H rows c, stored transposed [jj][c]
    const float* W = a.w_hh + (size_t)dir * 3 * H * H;
    for (int v = tid; v < 3 * H * kUnits / 4; v += 256) {
      const int c = v / (kUnits / 4), jq = (v % (kUnits / 4)) * 4;
      const v4f w = ld4(W + (size_t)c * H + j0 + jq);
      Wt[(jq + 0) * WP + c] = w.x;
      Wt[(jq + 1) * WP + c] = w.y;
      Wt[(jq + 2) * WP + c] = w.z;
      Wt[(jq + 3) * WP + c] = w.w;
    }
  }
  __syncthreads();

  float* dgh_dir = a.dgh + (size_t)dir * B * T * 3 * H;   // [B][T][3H] of this direction
  const int Gp = a.G;
  const __amdgpu_buffer_rsrc_t rg_ = rsrc(a.xbuf + (size_t)dir * 2 * Gp * 64 * 3 * H);   // [2][Gp][4][3H/16][64][4]
  float dhz[4] = {0.f, 0.f, 0.f, 0.f};

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? T - 1 - step : step;
    const int tnext = dir == 0 ? t + 1 : t - 1;
    const int tprev = dir == 0 ? t - 1 : t + 1;
    const bool edge = (step == T - 1);   // h_prev = 0 here
    stamp(a, step, 0);
    // epilogue operands (written by earlier launches): gates, dy, h_prev
    float g_r[4], g_z[4], g_n[4], g_h[4], dyv[4], hpv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = min(b0 + wave * 16 + lq * 4 + r, b_last);
      const float* gs = a.gates + (((size_t)dir * T + t) * B + b) * 4 * H;   // unit-interleaved (store_gates_il)
      const v4f gv = *reinterpret_cast<const v4f*>(gs + 4 * j);
      g_r[r] = gv.x;
      g_z[r] = gv.y;
      g_n[r] = gv.z;
      g_h[r] = gv.w;
      dyv[r] = a.dy[((size_t)b * T + t) * 2 * H + dir * H + j];
      hpv[r] = edge ? 0.f : a.y_in[((size_t)b * T + tprev) * 2 * H + dir * H + j];
    }
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if (step > 0) {
      sync_wait(a, cnt, dir, group, H / kUnits, step, local);
      stamp(a, step, 1);
      const unsigned base = (unsigned)(((((size_t)((step - 1) & 1) * Gp + group) * 4 + wave) * NKB * 64 + lane) * 16);
      // k rotation per slice (see the forward kernel): block index kr(i) = (i + rot) mod NKB
      const int rot = (slice * (NKB / (H / kUnits))) % NKB;
      auto kr = [&](int i) { const int v = i + rot; return v >= NKB ? v - NKB : v; };
      v4f dv[2][CH];
#pragma unroll
      for (int kb = 0; kb < CH; ++kb) dv[0][kb] = ld4_sc1(rg_, base + kr(kb) * 1024);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ch = 0; ch < NKB / CH; ++ch) {
        const int cur = ch & 1;
        if (ch + 1 < NKB / CH) {
#pragma unroll
          for (int kb = 0; kb < CH; ++kb) dv[cur ^ 1][kb] = ld4_sc1(rg_, base + kr((ch + 1) * CH + kb) * 1024);
        }
        __builtin_amdgcn_sched_barrier(0);   // next chunk's loads in flight before this chunk's MFMAs
        v4f wv[2];
        wv[0] = ld4(Wt + lr * WP + kr(ch * CH) * 16 + 4 * lq);
#pragma unroll
        for (int kb = 0; kb < CH; ++kb) {
          const int c = kb & 1;
          if (kb + 1 < CH) wv[c ^ 1] = ld4(Wt + lr * WP + kr(ch * CH + kb + 1) * 16 + 4 * lq);
          __builtin_amdgcn_sched_barrier(0);
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[cur][kb].x, wv[c].x, acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[cur][kb].y, wv[c].y, acc[1], 0, 0, 0);
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[cur][kb].z, wv[c].z, acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[cur][kb].w, wv[c].w, acc[1], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (a.trace) {
        asm volatile("" ::"v"(acc[0][0]), "v"(acc[1][0]));
        stamp(a, step, 2);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wave * 16 + lq * 4 + r, b = b0 + rl;
      float dh = dyv[r];
      if (step > 0) dh += (acc[0][r] + acc[1][r]) + dhz[r];
      const float rg = g_r[r], zg = g_z[r], ng = g_n[r], ghn = g_h[r], hp = hpv[r];
      const float dn = dh * (1.0f - zg);
      const float daz = dh * (hp - ng) * zg * (1.0f - zg);
      const float dan = dn * (1.0f - ng * ng);
      const float dar = dan * ghn * rg * (1.0f - rg);
      dhz[r] = dh * zg;
      dT[(rl * 4 + 0) * DTP + lr] = dar;
      dT[(rl * 4 + 1) * DTP + lr] = daz;
      dT[(rl * 4 + 2) * DTP + lr] = dan * rg;
      dT[(rl * 4 + 3) * DTP + lr] = dan;
    }
    __syncthreads();
    stamp(a, step, 3);
    // dgh row slice (gates x 16 units) of 64 rows: 768 float4, 3 per thread.  Interior steps go
    // write-through into the hand-off buffer (the next step's operand) before the arrival, and to
    // dgh (the dW_hh GEMM's operand) after it; the edge step has no consumer: it goes to dgh_edge
    // and zeroes its dgh row (kept out of the dW_hh GEMM, see srk_gru_layer_bwd).
    v4f val[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int v = tid + i * 256, rl = v / 12, g = (v % 12) / 4, uq = (v % 4) * 4, b = b0 + rl;
      val[i] = ld4(dT + (rl * 4 + g) * DTP + uq);
      if (b > b_last || edge) continue;
      st4_ho(rg_, (unsigned)(((((size_t)(step & 1) * Gp + group) * 4 + (rl >> 4)) * NKB * 64 +
                               (g * (H / 16) + slice) * 64 + (uq >> 2) * 16 + (rl & 15)) * 16), val[i], local);
    }
    sync_arrive(a, cnt, dir, group, slice, step, local);
    stamp(a, step, 4);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int v = tid + i * 256, rl = v / 12, g = (v % 12) / 4, uq = (v % 4) * 4, b = b0 + rl;
      if (b > b_last) continue;
      if (!edge) {
        st4(dgh_dir + ((size_t)b * T + t) * 3 * H + g * H + j0 + uq, val[i]);
      } else {
        st4(a.dgh_edge + ((size_t)dir * B + b) * 3 * H + g * H + j0 + uq, val[i]);
        st4(dgh_dir + ((size_t)b * T + t) * 3 * H + g * H + j0 + uq, v4f{0.f, 0.f, 0.f, 0.f});
      }
      // dgi (dar, daz, dan): the same 16-B row pieces from the staged image (a dword store per
      // cell and gate otherwise)
      st4(a.dgi + ((size_t)b * T + t) * 6 * H + dir * 3 * H + g * H + j0 + uq,
          g == 2 ? ld4(dT + (rl * 4 + 3) * DTP + uq) : val[i]);
    }
  }
}

// ------------------------------------------------------------------ fp32, two row chains per workgroup
// The fp32 recurrence is bound by its MFMAs (B = 256: 12.3k MFMA cycles per SIMD per step, 5.1-5.6 us)
// plus a serial tail the 4-wave kernels above leave the matrix cores idle in: the wait for the
// slowest producer, the cell epilogue and the publish (~3.5 us of a 10.5 us step, tools/gru_trace.py).
// Here a workgroup (direction, 64-row group, 16-unit slice — the same 256-workgroup grid and W_hh
// slice in LDS) runs 8 waves as two INDEPENDENT chains of 32 rows: wave w = (chain c = w >> 2, row
// block rb, k half kh) multiplies its 16 rows by the 48 gate columns over HALF of k (the h of slices
// 16 kh .. 16 kh + 15), so each SIMD hosts one wave of each chain and one chain's MFMAs fill the other
// chain's wait / epilogue / publish.  No workgroup barrier in the step loop:
//  * a wave polls the per-wave flags of just its producers ((slice, kh') of its chain and row block in
//    its k half: 32 words) and loads 16 fragment chunks of the hand-off;
//  * the k-half pair (kh = 0, 1) adds its partial sums through LDS (double-buffered, an LDS flag per
//    wave) in a fixed order (p0 + p1), after which wave kh owns units 8 kh .. 8 kh + 7 of its rows;
//  * the owner lanes run the cell update, transpose their 16 x 8 h block through a per-wave LDS tile
//    into the fragment layout (512 contiguous bytes of the chunk) and publish it with one flag word.
// Hand-off ring of kHandoffSlots = 3: a producer waits only for its own k half, so without the third
// slot it could overwrite step s - 1's data while a consumer in the other half still reads it; two
// steps ahead it cannot (every slice's step s + 1 needed both halves' step s through its k-half pair).
__device__ __forceinline__ void dc_wave_lds_fence() {   // this wave's LDS writes before its later LDS reads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// diagnostics: wave 4 (chain 1's first wave) stamps its arrival-wait end into trace slot 7
__device__ __forceinline__ void dc_stamp_chain1(const GruPArgs& a, int step) {
  if (a.trace && threadIdx.x == 256)
    a.trace[((size_t)blockIdx.x * a.T + step) * 8 + 7] = __builtin_amdgcn_s_memrealtime();
}

// optional phase offset between the two chains: chain 1 starts a.dc_offset ticks late; optional static
// priority of one chain (a.dc_prio = 1 + c): the two waves of a SIMD then do not split the matrix pipe
// evenly when their MFMA phases overlap — the favoured chain runs its phase at full rate and the other
// fills the gaps, which holds the chains out of phase (MI355X_MICROARCH.md, two waves per SIMD)
__device__ __forceinline__ void dc_chain_delay(const GruPArgs& a, int c) {
  if (c == 1 && a.dc_offset) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < a.dc_offset) __builtin_amdgcn_s_sleep(2);
  }
  if (a.dc_prio == 1 + c) __builtin_amdgcn_s_setprio(1);
}

constexpr int kDcXF = 24;   // floats a lane hands its pair partner: 3 gate accumulators x 4 rows (+ the fused projection's)

__device__ __forceinline__ void dc_wait(const GruPArgs& a, const unsigned* f, int step) {
  const int lane = threadIdx.x & 63;
  unsigned spins = 0;
  while (true) {
    const unsigned v = lane < 32 ? __hip_atomic_load(f + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0xffffffffu;
    if (__all(v >= (unsigned)step)) break;
    __builtin_amdgcn_s_sleep(1);
    if (++spins >= a.spin_limit) {
      if (lane == 0) spin_gave_up(a);
      break;
    }
  }
}

// pair barrier of the two k-half waves through an LDS word per wave (monotonic step counts)
__device__ __forceinline__ void dc_pair_sync(const GruPArgs& a, unsigned* pf, int w, int step) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(pf + w, (unsigned)(step + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  unsigned spins = 0;
  while (__hip_atomic_load(pf + (w ^ 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (unsigned)(step + 1)) {
    __builtin_amdgcn_s_sleep(0);
    if (++spins >= 4 * a.spin_limit) {
      if ((threadIdx.x & 63) == 0) spin_gave_up(a);
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ void dc_flag(const GruPArgs& a, unsigned* f, int step, bool local) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) {
    if (local)
      __builtin_amdgcn_raw_buffer_store_b32((unsigned)(step + 1), rsrc(reinterpret_cast<const float*>(f)), 0, 0, 0);
    else
      __hip_atomic_store(f, (unsigned)(step + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// flags of (dir, group, chain, row block): [32 slices][2 k halves] words
__device__ __forceinline__ unsigned* dc_flags(const GruPArgs& a, int dir, int group, int c, int rb) {
  return a.counters + pw_flag_dc(dir, a.G, group, c, rb, 0);
}

size_t dc_fwd_lds_floats(int H) { return (size_t)48 * (H + 4) + 16 * 32 * kDcXF + 8 * 128 + 16; }

// LDS: W slice [48][H + 4] | combine [2 c][2 rb][2 parity][2 sender kh][32 slots][kDcXF] |
// transpose tiles [8 waves][16][8] | pair flags [8]
template <int H, bool FUSED>
__global__ __launch_bounds__(512, 1) void gru_fwd_persistent_dc_kernel(GruPArgs a) {
  constexpr int WP = H + 4, NKB = H / 16, KB2 = NKB / 2;
  static_assert(KB2 == 16, "the k half is 16 k blocks (H = 512)");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ws = smem;
  float* xch = Ws + 48 * WP;
  float* tp = xch + 16 * 32 * kDcXF;
  unsigned* pf = reinterpret_cast<unsigned*>(tp + 8 * 128);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = w >> 2, rb = (w >> 1) & 1, kh = w & 1;
  const int lr = lane & 15, lq = lane >> 4;
  int dir, group, slice;
  bool local;
  place(a, H / kUnits, dir, group, slice, local);
  trace_id(a, dir, group, slice);
  const int T = a.T, j0 = slice * kUnits, j = j0 + lr;
  const int rbase = a.b_begin + group * kRows + 32 * c + 16 * rb;   // the wave's 16-row block
  const int b_last = a.b_end - 1;
  const bool own = (lr >> 3) == kh;   // after the combine this lane's unit belongs to this wave

  {  // this slice of W_hh[dir] -> LDS (read once per layer)
    const float* W = a.w_hh + (size_t)dir * 3 * H * H;
    for (int v = tid; v < 3 * kUnits * H / 4; v += 512) {
      const int cc = v / (H / 4), kq = (v % (H / 4)) * 4, g = cc / kUnits, jj = cc % kUnits;
      st4(Ws + cc * WP + kq, ld4(W + (size_t)(g * H + j0 + jj) * H + kq));
    }
  }
  if (tid < 8) pf[tid] = 0;
  // fused input projection (in <= 64): this wave's k half of the input quads, W_ih in registers
  constexpr bool fused = FUSED;
  const int nq = fused ? (a.in + 3) / 4 : 0, mh = (nq + 1) / 2;
  const int m0 = kh ? mh : 0, m1 = kh ? nq : mh;   // quads [m0, m1), at most 8
  constexpr int NX = FUSED ? 8 : 1;
  float wx[3][NX];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int k = 4 * (m0 + i) + lq;
      wx[g][i] = (fused && m0 + i < m1 && k < a.in) ? a.w_ih[((size_t)dir * 3 * H + g * H + j) * a.in + k] : 0.f;
    }
  float xv[NX];
  auto load_xh = [&](int t) {
    const float* xr = a.x_in + ((size_t)min(rbase + lr, b_last) * T + t) * a.in;
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int k = 4 * (m0 + i) + lq;
      xv[i] = (m0 + i < m1 && k < a.in) ? xr[k] : 0.f;
    }
  };
  if constexpr (FUSED) load_xh(dir == 0 ? 0 : T - 1);
  const float bir = fused ? a.b_ih[dir * 3 * H + j] : 0.f, biz = fused ? a.b_ih[dir * 3 * H + H + j] : 0.f,
              bin = fused ? a.b_ih[dir * 3 * H + 2 * H + j] : 0.f;
  const float bhr = a.b_hh[dir * 3 * H + j], bhz = a.b_hh[dir * 3 * H + H + j], bhn = a.b_hh[dir * 3 * H + 2 * H + j];
  __syncthreads();
  dc_chain_delay(a, c);

  const int Gp = a.G;
  const __amdgpu_buffer_rsrc_t rx = rsrc(a.xbuf + (size_t)dir * kHandoffSlots * Gp * 64 * H);   // [3][Gp][4][NKB][64][4]
  unsigned* myflags = dc_flags(a, dir, group, c, rb);
  const int rot = slice & (KB2 - 1);   // per-slice k rotation within the half (spreads the L2 channels)
  const int slot_id = (lr & 7) + 8 * lq;
  float* mytp = tp + w * 128;
  float hreg[4] = {0.f, 0.f, 0.f, 0.f};

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    stamp(a, step, 0);
    float gr[4], gz[4], gn[4];
    f32x4 ax[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if constexpr (FUSED) {   // this wave's k half of the step's input projection, before the wait
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        if (m0 + i >= m1) break;   // uniform
#pragma unroll
        for (int g = 0; g < 3; ++g) ax[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[i], wx[g][i], ax[g], 0, 0, 0);
      }
      if (step + 1 < T) load_xh(dir == 0 ? t + 1 : t - 1);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {   // input projections of the lane's cells (written by the gi GEMM)
        const int b = min(rbase + lq * 4 + r, b_last);
        const float* gi = a.gi + ((size_t)b * T + t) * 6 * H + dir * 3 * H;
        gr[r] = gi[j];
        gz[r] = gi[H + j];
        gn[r] = gi[2 * H + j];
      }
    }
    f32x4 acc[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if (step > 0) {
      dc_wait(a, myflags + 32 * kh, step);
      stamp(a, step, 1);
      dc_stamp_chain1(a, step);
      const unsigned base =
          (unsigned)((((((size_t)((step - 1) % kHandoffSlots) * Gp + group) * 4 + 2 * c + rb) * NKB + KB2 * kh) * 64 + lane) * 16);
      v4f hv[KB2];
#pragma unroll
      for (int i = 0; i < KB2; ++i) hv[i] = ld4_sc1(rx, base + ((i + rot) & (KB2 - 1)) * 1024);
      __builtin_amdgcn_sched_barrier(0);
      v4f wv[2][3];
#pragma unroll
      for (int g = 0; g < 3; ++g) wv[0][g] = ld4(Ws + (g * kUnits + lr) * WP + (KB2 * kh + rot) * 16 + 4 * lq);
#pragma unroll
      for (int i = 0; i < KB2; ++i) {
        const int cur = i & 1;
        if (i + 1 < KB2) {
          const int kn = KB2 * kh + ((i + 1 + rot) & (KB2 - 1));
#pragma unroll
          for (int g = 0; g < 3; ++g) wv[cur ^ 1][g] = ld4(Ws + (g * kUnits + lr) * WP + kn * 16 + 4 * lq);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int g = 0; g < 3; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[i][s], wv[cur][g][s], acc[g], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 12; ++q) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (a.trace) {
        asm volatile("" ::"v"(acc[0][0]), "v"(acc[1][0]), "v"(acc[2][0]));
        stamp(a, step, 2);
      }
    }
    // k-half combine: the partner's lanes get this wave's partial sums of their units
    {
      const int par = step & 1;
      float* out = xch + ((((c * 2 + rb) * 2 + par) * 2 + kh) * 32 + slot_id) * kDcXF;
      const float* in = xch + ((((c * 2 + rb) * 2 + par) * 2 + (kh ^ 1)) * 32 + slot_id) * kDcXF;
      if (!own) {
#pragma unroll
        for (int g = 0; g < 3; ++g) st4(out + 4 * g, v4f{acc[g][0], acc[g][1], acc[g][2], acc[g][3]});
        if (fused)
#pragma unroll
          for (int g = 0; g < 3; ++g) st4(out + 12 + 4 * g, v4f{ax[g][0], ax[g][1], ax[g][2], ax[g][3]});
      }
      dc_pair_sync(a, pf, w, step);
      if (own) {
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const v4f o = ld4(in + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[g][r] = kh == 0 ? acc[g][r] + o[r] : o[r] + acc[g][r];
        }
        if (fused) {
#pragma unroll
          for (int g = 0; g < 3; ++g) {
            const v4f o = ld4(in + 12 + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) ax[g][r] = kh == 0 ? ax[g][r] + o[r] : o[r] + ax[g][r];
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gr[r] = ax[0][r] + bir;
            gz[r] = ax[1][r] + biz;
            gn[r] = ax[2][r] + bin;
          }
        }
      }
    }
    // cell update of the owner lanes (rows 4 lq + r of the block, unit j), h -> the transpose tile
    float gsv[4][4];
    if (own) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ghn = acc[2][r] + bhn;
        float rg, zg, ng;
        if (a.fast_cell) {
          rg = sigmoid_fast(gr[r] + (acc[0][r] + bhr));
          zg = sigmoid_fast(gz[r] + (acc[1][r] + bhz));
          ng = tanh_fast(gn[r] + rg * ghn);
        } else {
          rg = sigmoidf_(gr[r] + (acc[0][r] + bhr));
          zg = sigmoidf_(gz[r] + (acc[1][r] + bhz));
          ng = tanhf(gn[r] + rg * ghn);
        }
        const float h = (1.0f - zg) * ng + zg * hreg[r];
        hreg[r] = h;
        mytp[(4 * lq + r) * 8 + (lr & 7)] = h;
        gsv[r][0] = rg;
        gsv[r][1] = zg;
        gsv[r][2] = ng;
        gsv[r][3] = ghn;
      }
    }
    dc_wave_lds_fence();
    stamp(a, step, 3);
    // publish: lane l < 32 = (q = l >> 4, row = l & 15) holds units 8 kh + 4 q .. + 3 of its row; the
    // chunk (row block, k block = slice) has them at fragment lanes 32 kh + l
    const int prow = lane & 15, pq = (lane >> 4) & 1;
    const v4f hv4 = ld4(mytp + prow * 8 + 4 * pq);
    const bool prow_ok = rbase + prow <= b_last;
    if (lane < 32 && step + 1 < T && prow_ok)
      st4_ho(rx, (unsigned)((((((size_t)(step % kHandoffSlots) * Gp + group) * 4 + 2 * c + rb) * NKB + slice) * 64 +
                             32 * kh + lane) * 16), hv4, local);
    dc_flag(a, myflags + 2 * slice + kh, step, local);
    stamp(a, step, 4);
    if (lane < 32 && prow_ok) st4(a.y + ((size_t)(rbase + prow) * T + t) * 2 * H + dir * H + j0 + 8 * kh + 4 * pq, hv4);
    if (own) store_gates_il(a, gsv, dir, t, rbase + 4 * lq, b_last, j);
  }
}


// The backward recurrence in the same two-chain form: wave (c, rb, kh) sums dg_next . W_hh over the
// k half of slices 16 kh .. 16 kh + 15 (all three gates of each: 48 of the 96 k blocks, 8 chunks in
// flight per buffer), the pair combines through LDS, the owner lanes (units 8 kh .. 8 kh + 7) run the
// cell backward and publish (dar, daz, dan * r) of their 16 rows x 8 units into the three gate chunks.
size_t dc_bwd_lds_floats(int H) { return (size_t)16 * (3 * H + 4) + 16 * 32 * 4 + 8 * 512 + 16; }

template <int H>
__global__ __launch_bounds__(512, 1) void gru_bwd_persistent_dc_kernel(GruPArgs a) {
  constexpr int WP = 3 * H + 4, NKB = 3 * H / 16, S = H / kUnits, CH = 8, NCH = 3 * (S / 2) / CH;   // 48 blocks, 6 chunks
  static_assert(S == 32 && NCH * CH == 48, "H = 512");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Wt = smem;                        // [16 units][3H + 4]
  float* xch = Wt + 16 * WP;               // [2 c][2 rb][2 parity][2 sender][32 slots][4]
  float* tp = xch + 16 * 32 * 4;           // [8 waves][16 rows][4 (dar, daz, dan r, dan)][8 units]
  unsigned* pf = reinterpret_cast<unsigned*>(tp + 8 * 512);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = w >> 2, rb = (w >> 1) & 1, kh = w & 1;
  const int lr = lane & 15, lq = lane >> 4;
  int dir, group, slice;
  bool local;
  place(a, S, dir, group, slice, local);
  trace_id(a, dir, group, slice);
  const int T = a.T, B = a.B, j0 = slice * kUnits, j = j0 + lr;
  const int rbase = a.b_begin + group * kRows + 32 * c + 16 * rb;
  const int b_last = a.b_end - 1;
  const bool own = (lr >> 3) == kh;

  {  // W_hh[dir][c][j0 .. j0+15] for all 3H rows c, stored transposed [jj][c]
    const float* W = a.w_hh + (size_t)dir * 3 * H * H;
    for (int v = tid; v < 3 * H * kUnits / 4; v += 512) {
      const int cc = v / (kUnits / 4), jq = (v % (kUnits / 4)) * 4;
      const v4f wv = ld4(W + (size_t)cc * H + j0 + jq);
      Wt[(jq + 0) * WP + cc] = wv.x;
      Wt[(jq + 1) * WP + cc] = wv.y;
      Wt[(jq + 2) * WP + cc] = wv.z;
      Wt[(jq + 3) * WP + cc] = wv.w;
    }
  }
  if (tid < 8) pf[tid] = 0;
  __syncthreads();
  dc_chain_delay(a, c);

  float* dgh_dir = a.dgh + (size_t)dir * B * T * 3 * H;
  const int Gp = a.G;
  const __amdgpu_buffer_rsrc_t rg_ = rsrc(a.xbuf + (size_t)dir * kHandoffSlots * Gp * 64 * 3 * H);   // [3][Gp][4][NKB][64][4]
  unsigned* myflags = dc_flags(a, dir, group, c, rb);
  const int slot_id = (lr & 7) + 8 * lq;
  float* mytp = tp + w * 512;
  // the wave's 48 k blocks: i -> gate i / 16, slice 16 kh + ((i + rot) mod 16), k block g * S + slice
  const int rot = slice & 15;
  auto kblock = [&](int i) { const int g = i >> 4; return g * S + 16 * kh + (((i & 15) + rot) & 15); };
  float dhz[4] = {0.f, 0.f, 0.f, 0.f};

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? T - 1 - step : step;
    const int tprev = dir == 0 ? t - 1 : t + 1;
    const bool edge = (step == T - 1);   // h_prev = 0 here
    stamp(a, step, 0);
    float g_r[4], g_z[4], g_n[4], g_h[4], dyv[4], hpv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {   // epilogue operands of the lane's cells (earlier launches)
      const int b = min(rbase + lq * 4 + r, b_last);
      const v4f gv = *reinterpret_cast<const v4f*>(a.gates + (((size_t)dir * T + t) * B + b) * 4 * H + 4 * j);
      g_r[r] = gv.x;
      g_z[r] = gv.y;
      g_n[r] = gv.z;
      g_h[r] = gv.w;
      dyv[r] = a.dy[((size_t)b * T + t) * 2 * H + dir * H + j];
      hpv[r] = edge ? 0.f : a.y_in[((size_t)b * T + tprev) * 2 * H + dir * H + j];
    }
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if (step > 0) {
      dc_wait(a, myflags + 32 * kh, step);
      stamp(a, step, 1);
      dc_stamp_chain1(a, step);
      const unsigned base =
          (unsigned)(((((size_t)((step - 1) % kHandoffSlots) * Gp + group) * 4 + 2 * c + rb) * NKB * 64 + lane) * 16);
      v4f dv[2][CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) dv[0][i] = ld4_sc1(rg_, base + kblock(i) * 1024);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int cur = ch & 1;
        if (ch + 1 < NCH) {
#pragma unroll
          for (int i = 0; i < CH; ++i) dv[cur ^ 1][i] = ld4_sc1(rg_, base + kblock((ch + 1) * CH + i) * 1024);
        }
        __builtin_amdgcn_sched_barrier(0);
        v4f wv[2];
        wv[0] = ld4(Wt + lr * WP + kblock(ch * CH) * 16 + 4 * lq);
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int cw = i & 1;
          if (i + 1 < CH) wv[cw ^ 1] = ld4(Wt + lr * WP + kblock(ch * CH + i + 1) * 16 + 4 * lq);
          __builtin_amdgcn_sched_barrier(0);
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[cur][i].x, wv[cw].x, acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[cur][i].y, wv[cw].y, acc[1], 0, 0, 0);
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[cur][i].z, wv[cw].z, acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[cur][i].w, wv[cw].w, acc[1], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (a.trace) {
        asm volatile("" ::"v"(acc[0][0]), "v"(acc[1][0]));
        stamp(a, step, 2);
      }
    }
    // k-half combine (p0 + p1) of the recurrent sum
    float dsum[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) dsum[r] = acc[0][r] + acc[1][r];
    {
      const int par = step & 1;
      float* out = xch + ((((c * 2 + rb) * 2 + par) * 2 + kh) * 32 + slot_id) * 4;
      const float* in = xch + ((((c * 2 + rb) * 2 + par) * 2 + (kh ^ 1)) * 32 + slot_id) * 4;
      if (!own) st4(out, v4f{dsum[0], dsum[1], dsum[2], dsum[3]});
      dc_pair_sync(a, pf, w, step);
      if (own) {
        const v4f o = ld4(in);
#pragma unroll
        for (int r = 0; r < 4; ++r) dsum[r] = kh == 0 ? dsum[r] + o[r] : o[r] + dsum[r];
      }
    }
    if (own) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float dh = dyv[r];
        if (step > 0) dh += dsum[r] + dhz[r];
        const float rg = g_r[r], zg = g_z[r], ng = g_n[r], ghn = g_h[r], hp = hpv[r];
        const float dn = dh * (1.0f - zg);
        const float daz = dh * (hp - ng) * zg * (1.0f - zg);
        const float dan = dn * (1.0f - ng * ng);
        const float dar = dan * ghn * rg * (1.0f - rg);
        dhz[r] = dh * zg;
        float* o = mytp + (4 * lq + r) * 32 + (lr & 7);
        o[0] = dar;
        o[8] = daz;
        o[16] = dan * rg;
        o[24] = dan;
      }
    }
    dc_wave_lds_fence();
    stamp(a, step, 3);
    // lane l < 32 = (q, row): units 8 kh + 4 q .. + 3 of its row, for each gate image
    const int prow = lane & 15, pq = (lane >> 4) & 1;
    const bool prow_ok = rbase + prow <= b_last;
    v4f val[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) val[g] = ld4(mytp + prow * 32 + 8 * g + 4 * pq);
    if (lane < 32 && !edge && prow_ok) {
#pragma unroll
      for (int g = 0; g < 3; ++g)
        st4_ho(rg_, (unsigned)((((((size_t)(step % kHandoffSlots) * Gp + group) * 4 + 2 * c + rb) * NKB + g * S + slice) * 64 +
                                32 * kh + lane) * 16), val[g], local);
    }
    dc_flag(a, myflags + 2 * slice + kh, step, local);
    stamp(a, step, 4);
    if (lane < 32 && prow_ok) {
      const int b = rbase + prow, u = j0 + 8 * kh + 4 * pq;
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        if (!edge) {
          st4(dgh_dir + ((size_t)b * T + t) * 3 * H + g * H + u, val[g]);
        } else {
          st4(a.dgh_edge + ((size_t)dir * B + b) * 3 * H + g * H + u, val[g]);
          st4(dgh_dir + ((size_t)b * T + t) * 3 * H + g * H + u, v4f{0.f, 0.f, 0.f, 0.f});
        }
        st4(a.dgi + ((size_t)b * T + t) * 6 * H + dir * 3 * H + g * H + u, g == 2 ? val[3] : val[g]);
      }
    }
  }
}

// ------------------------------------------------------------------ bf16 / fp16 operands
// The same two kernels with the recurrent matmul on v_mfma_f32_16x16x32_{bf16,f16} (16x the fp32
// MFMA rate; srk_set_option "matmul_precision" 1 / 2): the W_hh slice is held in LDS rounded to
// 16 bits (half the bytes), the hand-off carries h (fwd) / dg (bwd) rounded to 16 bits in
// fragment order — a 1 KB chunk per (16-row block, 32-wide k block): lane l holds the 8 k
// 32 kb + 8 (l >> 4) + j of row l & 15, one 16-B load per MFMA — and everything else (gates,
// cell update, the register carries, y, dgi, dgh) stays fp32.  A 16-unit slice s fills half of
// k block s / 2 (lane quarter-rows q = 2 (s & 1) + {0, 1}), 8 units per 16-B store.
template <bool F16>
struct RecOps;
template <>
struct RecOps<false> {
  typedef __bf16 e8 __attribute__((ext_vector_type(8)));
  __device__ static __forceinline__ f32x4 mma(e8 a, e8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct RecOps<true> {
  typedef _Float16 e8 __attribute__((ext_vector_type(8)));
  __device__ static __forceinline__ f32x4 mma(e8 a, e8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
typedef float v8f __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4_ __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));

template <bool F16>
__device__ __forceinline__ u32x4 pack8(v8f v) {
  return __builtin_bit_cast(u32x4, __builtin_convertvector(v, typename RecOps<F16>::e8));
}
__device__ __forceinline__ v8f cat8(v4f lo, v4f hi) { return v8f{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w}; }

// row pitches in 16-bit elements (+16: a ds_read_b128 B-fragment of 16 rows x 4 quarter-rows hits
// 16 distinct bank quads per lane group)
template <int H> constexpr int lp_fwd_wpe() { return H + 16; }
template <int H> constexpr int lp_bwd_wpe() { return 3 * H + 16; }

// LDS: W slice [48][H + 16] (16-bit; gate g, unit jj -> row g*16 + jj), then hT [64][20] fp32.
template <int H, bool F16>
__global__ __launch_bounds__(256, 1) void gru_fwd_persistent_lp_kernel(GruPArgs a) {
  using Ops = RecOps<F16>;
  using e8 = typename Ops::e8;
  constexpr int WPQ = lp_fwd_wpe<H>() / 8, HTP = kUnits + 4, NKB = H / 32;
  constexpr int RNDX = F16 ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  u32x4* Ws = reinterpret_cast<u32x4*>(smem);
  float* hT = smem + 3 * kUnits * WPQ * 4;
  float* Wx = hT + 64 * HTP;   // fused input projection: W_ih slice [48][kXP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
  int dir, group, slice;
  bool local;
  place(a, H / kUnits, dir, group, slice, local);
  trace_id(a, dir, group, slice);
  const int T = a.T, j0 = slice * kUnits, j = j0 + lr;
  const int b0 = a.b_begin + group * kRows;
  const int b_last = a.b_end - 1;
  unsigned* cnt = a.counters + pw_counter(dir, a.G, group);

  {  // this slice of W_hh[dir], rounded to 16 bits -> LDS (read once per layer)
    const float* W = a.w_hh + (size_t)dir * 3 * H * H;
    for (int v = tid; v < 3 * kUnits * (H / 8); v += 256) {
      const int c = v / (H / 8), kq = v % (H / 8), g = c / kUnits, jj = c % kUnits;
      const float* src = W + (size_t)(g * H + j0 + jj) * H + kq * 8;
      Ws[c * WPQ + kq] = pack8<F16>(cat8(ld4(src), ld4(src + 4)));
    }
  }
  const bool fused = a.x_in != nullptr;
  if (fused) stage_wih<RNDX>(a, Wx, dir, j0, H);
  float xnext[kFusedIn / 4];   // x of the next step (fused projection), loaded a step ahead
  if (fused) load_x(a, dir == 0 ? 0 : a.T - 1, min(a.b_begin + group * kRows + wave * 16 + lr, a.b_end - 1), lq, xnext);
  const float bir = fused ? a.b_ih[dir * 3 * H + j] : 0.f, biz = fused ? a.b_ih[dir * 3 * H + H + j] : 0.f,
              bin = fused ? a.b_ih[dir * 3 * H + 2 * H + j] : 0.f;
  const float bhr = a.b_hh[dir * 3 * H + j], bhz = a.b_hh[dir * 3 * H + H + j], bhn = a.b_hh[dir * 3 * H + 2 * H + j];
  __syncthreads();

  const int Gp = a.G;
  const __amdgpu_buffer_rsrc_t rx = rsrc(a.xbuf + (size_t)dir * 2 * Gp * 64 * H);   // 16-bit [2][Gp][4][H/32][64][8]
  float hreg[4] = {0.f, 0.f, 0.f, 0.f};
  float gsv[4][4];

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    stamp(a, step, 0);
    float gr[4], gz[4], gn[4];
    if (fused) {   // this step's input projection, before the wait (independent of h)
      fused_gi<RNDX>(a, Wx, xnext, lr, lq, bir, biz, bin, gr, gz, gn);
      if (step + 1 < T) load_x(a, dir == 0 ? t + 1 : t - 1, min(b0 + wave * 16 + lr, b_last), lq, xnext);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {   // input projections of the lane's cells (written by an earlier launch)
        const int b = min(b0 + wave * 16 + lq * 4 + r, b_last);
        const float* gi = a.gi + ((size_t)b * T + t) * 6 * H + dir * 3 * H;
        gr[r] = gi[j];
        gz[r] = gi[H + j];
        gn[r] = gi[2 * H + j];
      }
    }
    f32x4 acc[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (step > 0) {
      sync_wait(a, cnt, dir, group, H / kUnits, step, local);
      stamp(a, step, 1);
      const unsigned base = (unsigned)(((((size_t)((step - 1) & 1) * Gp + group) * 4 + wave) * NKB * 64 + lane) * 16);
      const int rot = slice % NKB;   // per-slice k rotation, see the fp32 kernel
      v4f hv[NKB];
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) hv[kb] = ld4_sc1(rx, base + ((kb + rot) & (NKB - 1)) * 1024);
      __builtin_amdgcn_sched_barrier(0);
      u32x4 wv[2][3];
#pragma unroll
      for (int g = 0; g < 3; ++g) wv[0][g] = Ws[(g * kUnits + lr) * WPQ + rot * 4 + lq];
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        const int c = kb & 1;
        if (kb + 1 < NKB) {
          const int kn = (kb + 1 + rot) & (NKB - 1);
#pragma unroll
          for (int g = 0; g < 3; ++g) wv[c ^ 1][g] = Ws[(g * kUnits + lr) * WPQ + kn * 4 + lq];
        }
        __builtin_amdgcn_sched_barrier(0);
        const e8 hf = __builtin_bit_cast(e8, hv[kb]);
#pragma unroll
        for (int g = 0; g < 3; ++g) acc[g] = Ops::mma(hf, __builtin_bit_cast(e8, wv[c][g]), acc[g]);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (a.trace) {
        asm volatile("" ::"v"(acc[0][0]), "v"(acc[1][0]), "v"(acc[2][0]));
        stamp(a, step, 2);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wave * 16 + lq * 4 + r, b = b0 + rl;
      const float ghn = acc[2][r] + bhn;
      const float rg = sigmoid_fast(gr[r] + (acc[0][r] + bhr));
      const float zg = sigmoid_fast(gz[r] + (acc[1][r] + bhz));
      const float ng = tanh_fast(gn[r] + rg * ghn);
      const float h = (1.0f - zg) * ng + zg * hreg[r];
      hreg[r] = h;
      hT[rl * HTP + lr] = h;
      gsv[r][0] = rg;
      gsv[r][1] = zg;
      gsv[r][2] = ng;
      gsv[r][3] = ghn;
    }
    __syncthreads();
    stamp(a, step, 3);
    const int yrl = tid >> 2, yuq = (tid & 3) * 4;   // y (fp32): thread = (row tid/4, units 4*(tid%4) .. +3)
    const v4f yv = ld4(hT + yrl * HTP + yuq);
    if (step + 1 < T && tid < 128) {   // hand-off (16-bit): thread = (row tid/2, units 8*(tid%2) .. +7)
      const int rl = tid >> 1, half = tid & 1;
      if (b0 + rl <= b_last) {
        const float* src = hT + rl * HTP + 8 * half;
        const int l = (2 * (slice & 1) + half) * 16 + (rl & 15);
        st4_ho(rx, (unsigned)(((((size_t)(step & 1) * Gp + group) * 4 + (rl >> 4)) * NKB + (slice >> 1)) * 64 + l) * 16,
                __builtin_bit_cast(v4f, pack8<F16>(cat8(ld4(src), ld4(src + 4)))), local);
      }
    }
    sync_arrive(a, cnt, dir, group, slice, step, local);   // the hand-off only: y and the gates go out after it
    stamp(a, step, 4);
    if (b0 + yrl <= b_last) {
      st4(a.y + ((size_t)(b0 + yrl) * T + t) * 2 * H + dir * H + j0 + yuq, yv);
      if (a.y16) {   // the layer's 16-bit copy of h for its weight-gradient GEMM (4 units = 8 B)
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        typedef __attribute__((ext_vector_type(4))) typename std::conditional<F16, _Float16, __bf16>::type e4;
        *reinterpret_cast<u32x2*>(a.y16 + ((size_t)(b0 + yrl) * T + t) * 2 * H + dir * H + j0 + yuq) =
            __builtin_bit_cast(u32x2, __builtin_convertvector(yv, e4));
      }
    }
    store_gates(a, gsv, dir, t, b0 + wave * 16 + lq * 4, b_last, j);
  }
}

// LDS: W^T slice [16][3H + 16] (16-bit; unit jj, gate row c), then the dg transpose tile [64][3][20].
template <int H, bool F16>
__global__ __launch_bounds__(256, 1) void gru_bwd_persistent_lp_kernel(GruPArgs a) {
  using Ops = RecOps<F16>;
  using e8 = typename Ops::e8;
  constexpr int WPQ = lp_bwd_wpe<H>() / 8, DTP = kUnits + 4, NKB = 3 * H / 32, CH = 16;
  static_assert(NKB % CH == 0, "chunking");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  u32x4* Wt = reinterpret_cast<u32x4*>(smem);
  float* dT = smem + kUnits * WPQ * 4;   // [64][3][DTP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
  int dir, group, slice;
  bool local;
  place(a, H / kUnits, dir, group, slice, local);
  trace_id(a, dir, group, slice);
  const int T = a.T, B = a.B, j0 = slice * kUnits, j = j0 + lr;
  const int b0 = a.b_begin + group * kRows;
  const int b_last = a.b_end - 1;
  unsigned* cnt = a.counters + pw_counter(dir, a.G, group);

  {  // W_hh[dir][c][j0 .. j0+15], all 3H rows c, transposed [jj][c] in 8-deep c packs
    const float* W = a.w_hh + (size_t)dir * 3 * H * H;
    for (int v = tid; v < (3 * H / 8) * (kUnits / 4); v += 256) {
      const int cb = v / (kUnits / 4), jq = (v % (kUnits / 4)) * 4;
      v4f w[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) w[e] = ld4(W + (size_t)(cb * 8 + e) * H + j0 + jq);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        Wt[(jq + u) * WPQ + cb] = pack8<F16>(v8f{w[0][u], w[1][u], w[2][u], w[3][u], w[4][u], w[5][u], w[6][u], w[7][u]});
    }
  }
  __syncthreads();

  float* dgh_dir = a.dgh + (size_t)dir * B * T * 3 * H;
  const int Gp = a.G;
  const __amdgpu_buffer_rsrc_t rg_ = rsrc(a.xbuf + (size_t)dir * 2 * Gp * 64 * 3 * H);   // 16-bit [2][Gp][4][3H/32][64][8]
  float dhz[4] = {0.f, 0.f, 0.f, 0.f};
  float dgv[4][3];
  const bool h16 = a.dgi16 != nullptr;   // 16-bit dgi / dgh outputs + in-kernel bias gradients
  float* dI = dT + 64 * 3 * DTP;         // [64][DTP]: dan (dgi's third gate; dT holds dan * r there)
  float sb[4] = {0.f, 0.f, 0.f, 0.f};    // sums of dar, daz, dan, dan * r over t and the lane's rows

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? T - 1 - step : step;
    const int tprev = dir == 0 ? t - 1 : t + 1;
    const bool edge = (step == T - 1);
    stamp(a, step, 0);
    float g_r[4], g_z[4], g_n[4], g_h[4], dyv[4], hpv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = min(b0 + wave * 16 + lq * 4 + r, b_last);
      const float* gs = a.gates + (((size_t)dir * T + t) * B + b) * 4 * H;
      g_r[r] = gs[j];
      g_z[r] = gs[H + j];
      g_n[r] = gs[2 * H + j];
      g_h[r] = gs[3 * H + j];
      dyv[r] = a.dy[((size_t)b * T + t) * 2 * H + dir * H + j];
      hpv[r] = edge ? 0.f : a.y_in[((size_t)b * T + tprev) * 2 * H + dir * H + j];
    }
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    if (step > 0) {
      sync_wait(a, cnt, dir, group, H / kUnits, step, local);
      stamp(a, step, 1);
      const unsigned base = (unsigned)(((((size_t)((step - 1) & 1) * Gp + group) * 4 + wave) * NKB * 64 + lane) * 16);
      const int rot = (slice * (NKB / (H / kUnits))) % NKB;
      auto kr = [&](int i) { const int v = i + rot; return v >= NKB ? v - NKB : v; };
      v4f dv[2][CH];
#pragma unroll
      for (int kb = 0; kb < CH; ++kb) dv[0][kb] = ld4_sc1(rg_, base + kr(kb) * 1024);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ch = 0; ch < NKB / CH; ++ch) {
        const int cur = ch & 1;
        if (ch + 1 < NKB / CH) {
#pragma unroll
          for (int kb = 0; kb < CH; ++kb) dv[cur ^ 1][kb] = ld4_sc1(rg_, base + kr((ch + 1) * CH + kb) * 1024);
        }
        __builtin_amdgcn_sched_barrier(0);
        u32x4 wv[2];
        wv[0] = Wt[lr * WPQ + kr(ch * CH) * 4 + lq];
#pragma unroll
        for (int kb = 0; kb < CH; ++kb) {
          const int c = kb & 1;
          if (kb + 1 < CH) wv[c ^ 1] = Wt[lr * WPQ + kr(ch * CH + kb + 1) * 4 + lq];
          __builtin_amdgcn_sched_barrier(0);
          acc[c] = Ops::mma(__builtin_bit_cast(e8, dv[cur][kb]), __builtin_bit_cast(e8, wv[c]), acc[c]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (a.trace) {
        asm volatile("" ::"v"(acc[0][0]), "v"(acc[1][0]));
        stamp(a, step, 2);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wave * 16 + lq * 4 + r, b = b0 + rl;
      float dh = dyv[r];
      if (step > 0) dh += (acc[0][r] + acc[1][r]) + dhz[r];
      const float rg = g_r[r], zg = g_z[r], ng = g_n[r], ghn = g_h[r], hp = hpv[r];
      const float dn = dh * (1.0f - zg);
      const float daz = dh * (hp - ng) * zg * (1.0f - zg);
      const float dan = dn * (1.0f - ng * ng);
      const float dar = dan * ghn * rg * (1.0f - rg);
      dhz[r] = dh * zg;
      dT[(rl * 3 + 0) * DTP + lr] = dar;
      dT[(rl * 3 + 1) * DTP + lr] = daz;
      dT[(rl * 3 + 2) * DTP + lr] = dan * rg;
      dgv[r][0] = dar;
      dgv[r][1] = daz;
      dgv[r][2] = dan;
      if (h16) {
        dI[rl * DTP + lr] = dan;
        if (b <= b_last) {
          sb[0] += dar;
          sb[1] += daz;
          sb[2] += dan;
          sb[3] += dan * rg;
        }
      }
    }
    __syncthreads();
    stamp(a, step, 3);
    v4f val[3];   // dgh (fp32, the dW_hh GEMM operand), stored after the arrival
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int v = tid + i * 256, rl = v / 12, g = (v % 12) / 4, uq = (v % 4) * 4;
      val[i] = ld4(dT + (rl * 3 + g) * DTP + uq);
    }
    if (!edge) {   // hand-off (16-bit): 64 rows x 3 gates x 2 halves of 8 units
      for (int v = tid; v < 64 * 3 * 2; v += 256) {
        const int rl = v / 6, g = (v % 6) >> 1, half = v & 1;
        if (b0 + rl > b_last) continue;
        const float* src = dT + (rl * 3 + g) * DTP + 8 * half;
        const int l = (2 * (slice & 1) + half) * 16 + (rl & 15);
        const int kb = g * (H / 32) + (slice >> 1);
        st4_ho(rg_, (unsigned)(((((size_t)(step & 1) * Gp + group) * 4 + (rl >> 4)) * NKB + kb) * 64 + l) * 16,
                __builtin_bit_cast(v4f, pack8<F16>(cat8(ld4(src), ld4(src + 4)))), local);
      }
    }
    sync_arrive(a, cnt, dir, group, slice, step, local);   // the hand-off only: dgh, dgh_edge and dgi go out after it
    stamp(a, step, 4);
    if (h16) {   // 16-bit dgh (edge rows zero) and dgi: (row, gate, 8 units) = one 16-B store each
      for (int v = tid; v < 64 * 3 * 2 * 2; v += 256) {
        const int which = v / 384, w = v % 384, rl = w / 6, g = (w % 6) >> 1, half = w & 1, b = b0 + rl;
        if (b > b_last) continue;
        const float* src = which == 0 || g < 2 ? dT + (rl * 3 + g) * DTP + 8 * half : dI + rl * DTP + 8 * half;
        v4f pk = __builtin_bit_cast(v4f, pack8<F16>(cat8(ld4(src), ld4(src + 4))));
        if (which == 0) {
          if (edge) pk = v4f{0.f, 0.f, 0.f, 0.f};
          *reinterpret_cast<v4f*>(a.dgh16 + (((size_t)dir * B + b) * T + t) * 3 * H + g * H + j0 + 8 * half) = pk;
        } else {
          *reinterpret_cast<v4f*>(a.dgi16 + ((size_t)b * T + t) * 6 * H + dir * 3 * H + g * H + j0 + 8 * half) = pk;
        }
      }
      continue;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int v = tid + i * 256, rl = v / 12, g = (v % 12) / 4, uq = (v % 4) * 4, b = b0 + rl;
      if (b > b_last) continue;
      if (!edge) {
        st4(dgh_dir + ((size_t)b * T + t) * 3 * H + g * H + j0 + uq, val[i]);
      } else {
        st4(a.dgh_edge + ((size_t)dir * B + b) * 3 * H + g * H + j0 + uq, val[i]);
        st4(dgh_dir + ((size_t)b * T + t) * 3 * H + g * H + j0 + uq, v4f{0.f, 0.f, 0.f, 0.f});
      }
    }
    store_dgi(a, dgv, dir, t, b0 + wave * 16 + lq * 4, b_last, j);
  }
  if (h16) {   // bias-gradient partials: lanes lr, lr + 16, lr + 32, lr + 48, then the 4 waves in order
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sb[q] += __shfl_xor(sb[q], 16);
      sb[q] += __shfl_xor(sb[q], 32);
    }
    __syncthreads();
    if (lq == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) dT[(wave * 4 + q) * 16 + lr] = sb[q];
    }
    __syncthreads();
    if (tid < 64) {
      const int q = tid >> 4, u = tid & 15;
      const float v = ((dT[(0 * 4 + q) * 16 + u] + dT[(1 * 4 + q) * 16 + u]) + dT[(2 * 4 + q) * 16 + u]) +
                      dT[(3 * 4 + q) * 16 + u];
      a.dbias[(((size_t)(a.chunk * 4 + group) * 2 + dir) * 4 + q) * H + j0 + u] = v;
    }
  }
}

// ------------------------------------------------------------------ 16-bit operands, 32 x 32 workgroups
// The bf16 / fp16 recurrence with workgroup = (direction, 32 batch rows, 32 hidden units) instead of
// (direction, 64 rows, 16 units): the same MFMA work per workgroup, but every consumer reads half the
// hand-off (32 rows x H instead of 64 x H: the L2 -> CU broadcast that sets the step time,
// profiles/r02*_gru_trace*) and each wave depends on 8 producers instead of 32.
//  * wave w = (row block rb = w & 1, k half kh = w >> 1): 16 rows x all 96 gate columns (fwd) or both
//    16-unit column blocks (bwd), over HALF of k — the k blocks of producers 8 kh .. 8 kh + 7 (slice s
//    owns units 32 s .. 32 s + 31 = k block s of h, blocks g * 16 + s of the 3H-wide dg);
//  * the two k halves are combined through LDS in a fixed order (kh = 0 part + kh = 1 part, IEEE
//    addition commutes), after which wave (rb, kh) owns units 32 s + 16 kh .. + 16 of its rows: the
//    cell epilogue is the 64 x 16 kernels' per-lane layout;
//  * a wave waits only for its 8 producers (per-wave polls of per-producer flags in the XCD-local /
//    flag protocols; the group counter otherwise), loads its 8 (fwd) or 24 (bwd) fragment chunks and
//    runs 48 MFMAs;
//  * hand-off chunks [buffer][group][rb][k block][lane][8 x 16-bit] (1 KB each): a producer writes 2
//    (fwd: k block s) or 6 (bwd: g * 16 + s); flags [2 dir][G][16] (<= 256 words).
// The backward kernel needs the 16-bit outputs (dgi16 / dgh16 / bias partials [chunk * 8 + group]).
constexpr int kRows2 = 32, kUnits2 = 32;

__device__ __forceinline__ void lp2_wait(const GruPArgs& a, int dir, int group, int first, int count, int step,
                                         bool per) {
  const int lane = threadIdx.x & 63;
  unsigned spins = 0;
  if (per) {   // per-producer flags, this wave's producers only
    unsigned* fl = a.counters + pw_flag_lp2(dir, a.G, group, first);
    while (true) {
      const unsigned v = lane < count ? __hip_atomic_load(fl + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : 0xffffffffu;
      if (__all(v >= (unsigned)step)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins >= a.spin_limit) {
        if (lane == 0) spin_gave_up(a);
        break;
      }
    }
  } else {     // the group's arrival counter (16 producers per step)
    unsigned* cnt = a.counters + pw_counter(dir, a.G, group);
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 16u * (unsigned)step) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins >= a.spin_limit) {
        if (lane == 0) spin_gave_up(a);
        break;
      }
    }
  }
}

__device__ __forceinline__ void lp2_arrive(const GruPArgs& a, int dir, int group, int slice, int step, bool per,
                                           bool local) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (per) {
      unsigned* f = a.counters + pw_flag_lp2(dir, a.G, group, slice);
      if (local)
        __builtin_amdgcn_raw_buffer_store_b32((unsigned)(step + 1), rsrc(reinterpret_cast<const float*>(f)), 0, 0, 0);
      else
        __hip_atomic_store(f, (unsigned)(step + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_fetch_add(a.counters + pw_counter(dir, a.G, group), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int H> constexpr int lp2_fwd_wpq() { return (H + 16) / 8; }
template <int H> constexpr int lp2_bwd_wpq() { return (3 * H + 16) / 8; }
constexpr int kXP2 = 20;   // pitch of the k-half exchange tiles (16 columns + 4: conflict-free b32 writes)

// OW (RB = 2, option gru_fwd_worker): the forward with 4 more waves (one more per SIMD) that take every
// global access off the recurrence waves except the hand-off: vmcnt retires in order, so the y / y16 /
// gate stores a recurrence wave issued after its publish, and (layer 1) its loads of the next step's gi,
// held the answer of its next flag poll back behind their own latency.  The recurrence
// waves now leave h in hT and the gates in an LDS tile; the workers store y, y16 and the gates after the
// publish barrier, and (no fused projection) fetch gi two steps ahead by LDS-DMA into a double buffer
// that reuses the fused projection's W_ih region.  Same arithmetic and outputs, bitwise.  The workers
// keep the recurrence waves' barriers (prologue, exchange, cell, publish).
template <int H, bool F16>
__device__ __forceinline__ void fwd_worker(const GruPArgs& a, const float* hT, const float* Gt, float* GI, int dir,
                                           int group, int j0, int b0, int b_last, int w, int lane) {
  constexpr int U = kUnits2, HTP = U + 4;
  const int T = a.T, tid = w * 64 + lane;   // 0 .. 255 over the 4 worker waves
  const bool fused = a.x_in != nullptr;
  auto bar = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
  auto rsrc_of = [](const void* p) {
    const uint64_t ad = (uint64_t)(uintptr_t)p;
    return u32x4s{(unsigned)__builtin_amdgcn_readfirstlane((unsigned)ad),
                  (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(ad >> 32)), 0x7ffffff0u, 0x00020000u};
  };
  const u32x4s rsG = rsrc_of(a.gi);   // the gi DMA (inline asm: a plain SGPR quad)
  const __amdgpu_buffer_rsrc_t rsY = rsrc(a.y), rsGt = rsrc(a.gates),
                               rsY16 = rsrc(a.y16 ? reinterpret_cast<const float*>(a.y16) : a.y);
  const unsigned zero = 0;
  // gi of step s (time t): [32 rows][3 gates][32 units] fp32 = 12 KB into buffer s & 1, i.e. [32 rows][24
  // 16-B units]; DMA instruction k (0 .. 11 over the 4 workers, 1 KB each, lane-linear at M0 + 16 lane)
  // fills units 64 k .. 64 k + 63 of that linear image
  auto dma_gi = [&](int s) {
    const int t = dir == 0 ? s : T - 1 - s;
    float* buf = GI + (s & 1) * 32 * 96;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int k = 3 * w + i, unit = 64 * k + lane, row = unit / 24, g = (unit % 24) >> 3, q = unit & 7;
      const unsigned v = b0 + row <= b_last
                             ? (unsigned)((((size_t)(b0 + row) * T + t) * 6 * H + dir * 3 * H + g * H + j0 + 4 * q) * 4)
                             : 0x80000000u;
      const unsigned ldsa = (unsigned)__builtin_amdgcn_readfirstlane(
          (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)(buf + 64 * k * 4));
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(v), "s"(rsG), "s"(ldsa), "s"(zero)
                   : "memory");
    }
  };
  // y / y16 / gates of step s from hT and the gate tile: 6 buffer stores per thread, always issued
  // (rows past the batch go past num_records and are dropped) so the vmcnt count per step is fixed
  auto store_out = [&](int s) {
    const int t = dir == 0 ? s : T - 1 - s;
    {
      const int row = tid >> 3, u4 = (tid & 7) * 4;
      const v4f yv = *reinterpret_cast<const v4f*>(hT + row * HTP + u4);
      const bool ok = b0 + row <= b_last;
      const size_t e = ((size_t)(b0 + row) * T + t) * 2 * H + dir * H + j0 + u4;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, yv), rsY, ok ? (int)(e * 4) : (int)0x80000000u, 0, 0);
      typedef __attribute__((ext_vector_type(4))) typename std::conditional<F16, _Float16, __bf16>::type e4;
      const u32x2_ y2 = __builtin_bit_cast(u32x2_, __builtin_convertvector(yv, e4));
      __builtin_amdgcn_raw_buffer_store_b64(y2, rsY16, (ok && a.y16) ? (int)(e * 2) : (int)0x80000000u, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // cells (row, unit) = (c / 32, c % 32), c = tid + 256 i: unit-interleaved gates
      const int c = tid + 256 * i, row = c >> 5, u = c & 31;
      const v4f gv = *reinterpret_cast<const v4f*>(Gt + (row * 32 + u) * 4);
      const bool ok = b0 + row <= b_last;
      const size_t e = ((((size_t)dir * T + t) * a.B + b0 + row) * H + j0 + u) * 4;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, gv), rsGt, ok ? (int)(e * 4) : (int)0x80000000u, 0, 0);
    }
  };
  if (!fused) {   // gi of step 0 before the prologue barrier (the recurrence waves' first cell follows it)
    dma_gi(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();   // = the prologue barrier
  if (!fused && T > 1) dma_gi(1);
  for (int step = 0; step < T; ++step) {
    if (step > 0) {
      // gi of this step landed (issued two steps ago): only the previous step's 6 stores and, when it
      // issued one, its gi DMA (3) may still be in flight
      if (!fused) {
        if (step + 1 < T) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      }
      bar();   // = the k-half exchange
    }
    bar();     // = the cell barrier: h and the gates of this step are in LDS
    bar();     // = the publish (lp2_arrive)
    store_out(step);
    if (!fused && step + 2 < T) dma_gi(step + 2);   // into the buffer this step's cell has consumed
  }
}

// RB row blocks of 16 per workgroup (2 x RB waves: wave = kh * RB + rb): RB = 2 is the 32 x 32
// workgroup; RB = 4 (64 rows, 8 waves, the same W slice in LDS) runs a 512-row batch in ONE launch
// where RB = 2 needs two chunks one after the other.  Per row the arithmetic is the same.
template <int RB> constexpr int lp2_fused_in() { return RB == 2 ? kFusedIn : 40; }   // RB = 4: LDS fits 40
// LDS: W slice [96][H + 16] 16-bit (row g * 32 + jj) | hT [16 RB][36] fp32 | W_ih slice [96][KF + 1] fp32 |
// exchange [2 RB waves][3][16][kXP2] fp32
template <int H, bool F16, int RB, bool OW = false>
__global__ __launch_bounds__(OW ? 512 : 128 * RB, 1) void gru_fwd_persistent_lp2_kernel(GruPArgs a) {
  using Ops = RecOps<F16>;
  using e8 = typename Ops::e8;
  constexpr int U = kUnits2, S = H / U, WPQ = lp2_fwd_wpq<H>(), HTP = U + 4, NKB = H / 32, KH = NKB / 2;
  constexpr int RNDX = F16 ? 2 : 1, NT = 128 * RB, ROWS = 16 * RB, KF = lp2_fused_in<RB>(), XP = KF + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  u32x4* Ws = reinterpret_cast<u32x4*>(smem);
  float* hT = smem + 3 * U * WPQ * 4;
  float* Wx = hT + ROWS * HTP;
  float* X = Wx + 3 * U * XP;
  float* Gt = X + 2 * RB * 3 * 16 * kXP2;   // OW: the step's gates [32 rows][32 units][4]
  float* GI = Wx;                           // OW without the fused projection: gi [2][32 rows][3][32]
  static_assert(!OW || (RB == 2 && 2 * 32 * 96 <= 3 * U * XP), "forward worker: 32-row workgroups");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
  const int rb = wave % RB, kh = wave / RB;
  int dir, group, slice;
  bool local;
  stamp(a, 0, 6);   // kernel entry (prologue = slot 0 - slot 6 of step 0)
  place(a, S, dir, group, slice, local);
  trace_id(a, dir, group, slice);
  const bool per = a.flags || local;
  const int T = a.T, j0 = slice * U, ju = kh * 16 + lr, j = j0 + ju;
  const int b0 = a.b_begin + group * ROWS, b_last = a.b_end - 1, rbase = b0 + rb * 16;
  if constexpr (OW) {
    if (wave >= 2 * RB) {   // the output / input worker waves
      fwd_worker<H, F16>(a, hT, Gt, GI, dir, group, j0, b0, b_last, wave - 2 * RB, lane);
      return;
    }
  }

  {  // this slice of W_hh[dir] (3 gates x 32 units), rounded to 16 bits -> LDS; loads issued 8 packs
     // at a time ahead of their stores (the prologue is a chain of L2 round trips otherwise)
    const float* W = a.w_hh + (size_t)dir * 3 * H * H;
    constexpr int NV = 3 * U * (H / 8), NB = 2048 / NT;
    static_assert(NV % (NT * NB) == 0, "prologue batches");
    for (int v0 = tid; v0 < NV; v0 += NT * NB) {
      v4f w[NB][2];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int v = v0 + NT * u, c = v / (H / 8), kq = v % (H / 8), g = c / U, jj = c % U;
        const float* src = W + (size_t)(g * H + j0 + jj) * H + kq * 8;
        w[u][0] = ld4(src);
        w[u][1] = ld4(src + 4);
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int v = v0 + NT * u, c = v / (H / 8), kq = v % (H / 8);
        Ws[c * WPQ + kq] = pack8<F16>(cat8(w[u][0], w[u][1]));
      }
    }
  }
  const bool fused = a.x_in != nullptr;
  if (fused) {   // W_ih slice (rows g * 32 + jj), rounded like the GEMM operands, 8 loads in flight
    const float* W = a.w_ih + (size_t)dir * 3 * H * a.in;
    constexpr int NV = 3 * U * KF, NB = 2048 / NT;   // the last batch is partial for RB = 4
    for (int v0 = tid; v0 < NV; v0 += NT * NB) {
      float w[NB];
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int v = min(v0 + NT * u, NV - 1), c = v / KF, k = v % KF, g = c / U, jj = c % U;
        w[u] = k < a.in ? W[(size_t)(g * H + j0 + jj) * a.in + k] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        const int v = v0 + NT * u, c = v / KF, k = v % KF;
        if (v < NV) Wx[c * XP + k] = rnd16<RNDX>(w[u]);
      }
    }
  }
  float xnext[kFusedIn / 4];
  if (fused) load_x(a, dir == 0 ? 0 : T - 1, min(rbase + lr, b_last), lq, xnext);
  const float bir = fused ? a.b_ih[dir * 3 * H + j] : 0.f, biz = fused ? a.b_ih[dir * 3 * H + H + j] : 0.f,
              bin = fused ? a.b_ih[dir * 3 * H + 2 * H + j] : 0.f;
  const float bhr = a.b_hh[dir * 3 * H + j], bhz = a.b_hh[dir * 3 * H + H + j], bhn = a.b_hh[dir * 3 * H + 2 * H + j];
  __syncthreads();

  const int Gp = a.G;
  const __amdgpu_buffer_rsrc_t rx = rsrc(a.xbuf + (size_t)dir * 2 * Gp * ROWS * H);   // 16-bit [2][Gp][RB][NKB][64][8]
  float hreg[4] = {0.f, 0.f, 0.f, 0.f};
  float gsv[4][4];

  // y (fp32 + the 16-bit copy) and the saved gates of a step, from hT / gsv, after its arrival.
  // (Issuing them one step later, behind the next step's hand-off loads, shortens that step's wait --
  // vmcnt retires in order, so stores ahead of a flag poll hold its answer back -- but their issue
  // then lands on the MFMA phase: measured slower, DESIGN.md.)
  auto flush_outputs = [&](int sstep) {
    const int ts = dir == 0 ? sstep : T - 1 - sstep;
    const int row = tid >> 3, u4 = (tid & 7) * 4;   // 32 rows x 32 units
    if (b0 + row <= b_last) {
      const v4f yv = ld4(hT + row * HTP + u4);
      st4(a.y + ((size_t)(b0 + row) * T + ts) * 2 * H + dir * H + j0 + u4, yv);
      if (a.y16) {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        typedef __attribute__((ext_vector_type(4))) typename std::conditional<F16, _Float16, __bf16>::type e4;
        *reinterpret_cast<u32x2*>(a.y16 + ((size_t)(b0 + row) * T + ts) * 2 * H + dir * H + j0 + u4) =
            __builtin_bit_cast(u32x2, __builtin_convertvector(yv, e4));
      }
    }
    if (a.y16) store_gates_il(a, gsv, dir, ts, rbase + lq * 4, b_last, j);   // read by the 16-bit bwd kernel
    else store_gates(a, gsv, dir, ts, rbase + lq * 4, b_last, j);
  };
  float gr[4], gz[4], gn[4];
  auto load_gi = [&](int t) {   // non-fused: this step's input projections from the gi GEMM
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = min(rbase + lq * 4 + r, b_last);
      const float* gi = a.gi + ((size_t)b * T + t) * 6 * H + dir * 3 * H;
      gr[r] = gi[j];
      gz[r] = gi[H + j];
      gn[r] = gi[2 * H + j];
    }
  };
  // this step's input-side loads (fused: the next step's x), ahead of the wait
  auto issue_inputs = [&](int step, int t) {
    if (fused) {
      if (step + 1 < T) load_x(a, dir == 0 ? t + 1 : t - 1, min(rbase + lr, b_last), lq, xnext);
    } else if (!OW) {
      load_gi(t);
    }
  };

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    stamp(a, step, 0);
    if (fused) {   // the lane's input projections (rows rbase + 4 lq + r, unit j), before the wait
      float xv[kFusedIn / 4];
#pragma unroll
      for (int m = 0; m < kFusedIn / 4; ++m) xv[m] = rnd16<RNDX>(xnext[m]);
      f32x4 ax[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int m = 0; m < KF / 4; ++m) {
        if (4 * m >= a.in) break;   // uniform
#pragma unroll
        for (int g = 0; g < 3; ++g)
          ax[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[m], Wx[(g * U + kh * 16 + lr) * XP + 4 * m + lq], ax[g], 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gr[r] = ax[0][r] + bir;
        gz[r] = ax[1][r] + biz;
        gn[r] = ax[2][r] + bin;
      }
    }
    issue_inputs(step, t);
    float full[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if (step > 0) {
      lp2_wait(a, dir, group, kh * KH, KH, step, per);
      stamp(a, step, 1);
      const unsigned base =
          (unsigned)((((((size_t)((step - 1) & 1) * Gp + group) * RB + rb) * NKB + kh * KH) * 64 + lane) * 16);
      v4f hv[KH];
#pragma unroll
      for (int i = 0; i < KH; ++i) hv[i] = ld4_sc1(rx, base + i * 1024);
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc[6];
#pragma unroll
      for (int cb = 0; cb < 6; ++cb) acc[cb] = f32x4{0.f, 0.f, 0.f, 0.f};
      u32x4 wv[2][6];
#pragma unroll
      for (int cb = 0; cb < 6; ++cb) wv[0][cb] = Ws[((cb >> 1) * U + (cb & 1) * 16 + lr) * WPQ + (kh * KH) * 4 + lq];
#pragma unroll
      for (int i = 0; i < KH; ++i) {
        const int c = i & 1;
        if (i + 1 < KH) {
#pragma unroll
          for (int cb = 0; cb < 6; ++cb)
            wv[c ^ 1][cb] = Ws[((cb >> 1) * U + (cb & 1) * 16 + lr) * WPQ + (kh * KH + i + 1) * 4 + lq];
        }
        __builtin_amdgcn_sched_barrier(0);
        const e8 hf = __builtin_bit_cast(e8, hv[i]);
#pragma unroll
        for (int cb = 0; cb < 6; ++cb) acc[cb] = Ops::mma(hf, __builtin_bit_cast(e8, wv[c][cb]), acc[cb]);
        __builtin_amdgcn_sched_barrier(0);
      }
      // k halves: hand the partner (same rows, other kh) the column blocks it owns, take ours.  kh is
      // wave-uniform: one static code path per value (an acc index computed from kh would make the
      // compiler select registers with compare / cndmask chains)
      float* Xw = X + wave * (3 * 16 * kXP2);
      const float* Xp = X + (wave ^ RB) * (3 * 16 * kXP2);
      auto exchange = [&](auto KH_) {
        constexpr int K = decltype(KH_)::value;
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r) Xw[(g * 16 + 4 * lq + r) * kXP2 + lr] = acc[2 * g + (1 - K)][r];
        __syncthreads();
#pragma unroll
        for (int g = 0; g < 3; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float o = acc[2 * g + K][r], p = Xp[(g * 16 + 4 * lq + r) * kXP2 + lr];
            full[g][r] = K == 0 ? o + p : p + o;   // always (kh 0 part) + (kh 1 part)
          }
      };
      if (__builtin_amdgcn_readfirstlane(kh) == 0) exchange(std::integral_constant<int, 0>{});
      else exchange(std::integral_constant<int, 1>{});
      if (a.trace) {
        asm volatile("" ::"v"(full[0][0]), "v"(full[1][0]), "v"(full[2][0]));
        stamp(a, step, 2);
      }
    }
    if (OW && !fused) {   // this step's gi, fetched into LDS by the workers (landed before the exchange barrier)
      const float* gib = GI + (step & 1) * 32 * 96;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = rb * 16 + lq * 4 + r;
        gr[r] = gib[rl * 96 + ju];
        gz[r] = gib[rl * 96 + 32 + ju];
        gn[r] = gib[rl * 96 + 64 + ju];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = rb * 16 + lq * 4 + r;
      const float ghn = full[2][r] + bhn;
      const float rg = sigmoid_fast(gr[r] + (full[0][r] + bhr));
      const float zg = sigmoid_fast(gz[r] + (full[1][r] + bhz));
      const float ng = tanh_fast(gn[r] + rg * ghn);
      const float h = (1.0f - zg) * ng + zg * hreg[r];
      hreg[r] = h;
      hT[rl * HTP + ju] = h;
      gsv[r][0] = rg;
      gsv[r][1] = zg;
      gsv[r][2] = ng;
      gsv[r][3] = ghn;
      if constexpr (OW) *reinterpret_cast<v4f*>(Gt + (rl * 32 + ju) * 4) = v4f{rg, zg, ng, ghn};
    }
    __syncthreads();
    stamp(a, step, 3);
    if (step + 1 < T && tid < 64 * RB) {   // hand-off (16-bit): chunk (rb', k block = slice), lane l: row l & 15, 8 units
      const int rbp = tid >> 6, l = tid & 63, row = rbp * 16 + (l & 15);
      if (b0 + row <= b_last) {
        const float* src = hT + row * HTP + 8 * (l >> 4);
        st4_ho(rx, (unsigned)((((((size_t)(step & 1) * Gp + group) * RB + rbp) * NKB + slice) * 64 + l) * 16),
               __builtin_bit_cast(v4f, pack8<F16>(cat8(ld4(src), ld4(src + 4)))), local);
      }
    }
    lp2_arrive(a, dir, group, slice, step, per, local);   // the hand-off only: y and the gates go out after it
    stamp(a, step, 4);
    if constexpr (!OW) flush_outputs(step);   // OW: the worker waves store them
  }
}

// LDS: W^T slice [32][3H + 16] 16-bit (unit jj, gate row c) | dT [16 RB][3][36] | dI [16 RB][36] |
// exchange [2 RB waves][16][kXP2] | bias partials [2 RB waves][4][16] | (DW) dg image [32 rows][96] 16-bit |
// (DW) h_prev images [4 worker waves][32 rows][128 columns] 16-bit
//
// DW (RB = 2, option gru_dwhh_fused): the recurrent weight gradient dW_hh = sum_t dg_t^T h_(t-1) is
// accumulated by this kernel instead of by a GEMM over the stored dgh16 / y16 afterwards.  The workgroup
// gets 4 more waves (one more per SIMD) that do only that: after each step's publish barrier, worker
// wave w multiplies the workgroup's 96 gate rows (3 gates x the slice's 32 units) of dg_t^T [96 x 32 rows]
// by h_prev [32 rows x columns 128 w .. + 127] on v_mfma_f32_16x16x32 (the 32 batch rows are the k of
// one MFMA), 6 x 8 accumulator tiles held for the whole sequence — the recurrence waves' matrix pipe is
// idle through their hand-off waits, and their registers are untouched.  Operands are [row][column]
// 16-bit LDS images read with ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group, delivered
// column-major: 8 consecutive rows of one column per lane = the operand fragment): the dg image is
// written by the cell (rounded exactly as the dgh16 the GEMM read); each worker fetches its own h_prev
// columns (the forward's y16 rows, zero past the batch) by LDS-DMA one step ahead into a private image,
// so its loads never sit in front of a recurrence wave's flag poll.  The workers keep the recurrence
// waves' barrier count (prologue, exchange, cell, publish, bias partials).  At the end each worker
// writes its partial [96][128] to dw_part[chunk * 8 + group][dir]; dwhh_reduce_kernel sums the
// partials in part order.
constexpr int kDgP = 96;   // dg image row pitch (16-bit elements)
// h_prev image of one worker: [32 rows][8 granules of 32 B]; granule g of row r at g ^ dw_swz(r): the
// 4 rows of a 16-lane transposed read and the two groups of a 32-lane half (8 rows apart) fall in 8
// distinct 32-B bank windows
__device__ __forceinline__ int dw_swz(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }

// The DW worker waves (wave 4 + w): see above.  Barrier sequence = the recurrence waves'.
template <int H, bool F16>
__device__ __forceinline__ void dw_worker(const GruPArgs& a, const unsigned short* Aimg, unsigned char* Bimg, int dir,
                                          int group, int j0, int b0, int b_last, int w, int lane) {
  const int T = a.T;
  unsigned char* img = Bimg + w * 32 * 256;   // this worker's [32][256 B]
  typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
  const uint64_t ya = (uint64_t)(uintptr_t)a.y16_in;
  const u32x4s rsY{(unsigned)__builtin_amdgcn_readfirstlane((unsigned)ya),
                   (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(ya >> 32)), 0x7ffffff0u, 0x00020000u};
  const unsigned zero = 0;
  // h_prev of step s: y16 rows (b, tprev), columns dir H + 128 w .. + 127; DMA instruction i fills rows
  // 4 i .. 4 i + 3 (1 KB, lane-linear at M0 + 16 lane), so lane l fetches the unit the swizzle puts there
  auto dma = [&](int s) {
    const int t = dir == 0 ? T - 1 - s : s, tprev = dir == 0 ? t - 1 : t + 1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = 4 * i + (lane >> 4), g = ((lane & 15) >> 1) ^ dw_swz(row);
      const int col = 128 * w + 16 * g + 8 * (lane & 1);
      const unsigned v = b0 + row <= b_last
                             ? (unsigned)(((((size_t)(b0 + row) * T + tprev) * 2 * H + dir * H) + col) * 2)
                             : 0x80000000u;
      const unsigned ldsa = (unsigned)__builtin_amdgcn_readfirstlane(
          (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)(img + i * 1024));
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(v), "s"(rsY), "s"(ldsa), "s"(zero)
                   : "memory");
    }
  };
  typedef __attribute__((address_space(3))) s16x4_ lds_s16x4;
  auto tr4 = [](const void* p) { return __builtin_bit_cast(u32x2_, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p)); };
  f32x4 acc[6][8];
#pragma unroll
  for (int m = 0; m < 6; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g4 = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3, r0 = 8 * g4 + q;
  // raw s_barrier: __syncthreads() would first drain this wave's LDS-DMA (vmcnt(0)) and hold the
  // recurrence waves' barrier behind the next step's h_prev fetch
  auto bar = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  const bool late = (a.dw_mode & 2) != 0;   // fetch step s's h_prev after step s's exchange barrier (the recurrence
                                            // waves are past their hand-off loads then), not right after step s-1's MFMAs
  bar();   // = the prologue barrier (W slice in LDS)
  if (T > 1) dma(0);
  for (int step = 0; step < T; ++step) {
    if (step > 0) {
      bar();   // = the k-half exchange
      if (late && step < T - 1) dma(step);
    }
    bar();                 // = the cell barrier: this step's dg image is complete
    bar();                 // = the publish (lp2_arrive)
    if (step == T - 1) continue;     // the edge step: h_prev = 0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this step's h_prev image (its DMA was issued a step ago)
    u32x4 af[6];
#pragma unroll
    for (int mb = 0; mb < 6; ++mb) {
      const u32x2_ lo = tr4(Aimg + r0 * kDgP + 16 * mb + 4 * p4);
      const u32x2_ hi = tr4(Aimg + (r0 + 4) * kDgP + 16 * mb + 4 * p4);
      af[mb] = u32x4{lo.x, lo.y, hi.x, hi.y};
    }
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const unsigned char* bb = img + r0 * 256 + 32 * (nb ^ dw_swz(r0)) + 8 * p4;   // row r0 + 4: the same swizzle
      const u32x2_ lo = tr4(bb);
      const u32x2_ hi = tr4(bb + 4 * 256);
      const u32x4 bf = u32x4{lo.x, lo.y, hi.x, hi.y};
#pragma unroll
      for (int mb = 0; mb < 6; ++mb)
        acc[mb][nb] = RecOps<F16>::mma(__builtin_bit_cast(typename RecOps<F16>::e8, af[mb]),
                                       __builtin_bit_cast(typename RecOps<F16>::e8, bf), acc[mb][nb]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // image reads done: the next DMA may overwrite
    if (!late && step + 1 < T - 1) dma(step + 1);
  }
  bar();   // = the bias-partials barrier
  float* dst = a.dw_part + ((size_t)(a.chunk * 8 + group) * 2 + dir) * 3 * H * H;
#pragma unroll
  for (int mb = 0; mb < 6; ++mb)
#pragma unroll
    for (int nb = 0; nb < 8; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = (mb >> 1) * H + j0 + 16 * (mb & 1) + 4 * (lane >> 4) + r, col = 128 * w + 16 * nb + (lane & 15);
        dst[(size_t)row * H + col] = acc[mb][nb][r];
      }
}

template <int H, bool F16, int RB, bool DW = false>
__global__ __launch_bounds__(DW ? 512 : 128 * RB, 1) void gru_bwd_persistent_lp2_kernel(GruPArgs a) {
  using Ops = RecOps<F16>;
  using e8 = typename Ops::e8;
  constexpr int U = kUnits2, S = H / U, WPQ = lp2_bwd_wpq<H>(), DTP = U + 4, NKB = 3 * H / 32, KS = S / 2;
  constexpr int NT = 128 * RB, ROWS = 16 * RB, NW = 2 * RB;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  u32x4* Wt = reinterpret_cast<u32x4*>(smem);
  float* dT = smem + U * WPQ * 4;              // [ROWS][3][DTP]
  float* dI = dT + ROWS * 3 * DTP;             // [ROWS][DTP]: dan (dgi's third gate; dT holds dan * r)
  float* X = dI + ROWS * DTP;                  // [NW][16][kXP2]
  float* red = X + NW * 16 * kXP2;             // [NW][4][16]
  unsigned short* Aimg = reinterpret_cast<unsigned short*>(red + NW * 4 * 16);   // DW: [32][kDgP]
  unsigned char* Bimg = reinterpret_cast<unsigned char*>(Aimg + 32 * kDgP);      // DW: [4 workers][32][256 B]
  static_assert(!DW || (RB == 2 && H == 512), "fused dW_hh: 32-row workgroups, H = 512");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lq = lane >> 4;
  const int rb = wave % RB, kh = wave / RB;
  int dir, group, slice;
  bool local;
  stamp(a, 0, 6);   // kernel entry
  place(a, S, dir, group, slice, local);
  trace_id(a, dir, group, slice);
  const bool per = a.flags || local;
  const int T = a.T, B = a.B, j0 = slice * U, ju = kh * 16 + lr, j = j0 + ju;
  const int b0 = a.b_begin + group * ROWS, b_last = a.b_end - 1, rbase = b0 + rb * 16;
  if constexpr (DW) {
    if (wave >= NW) {   // the dW worker waves
      dw_worker<H, F16>(a, Aimg, Bimg, dir, group, j0, b0, b_last, wave - NW, lane);
      return;
    }
    if (a.dw_mode & 4) __builtin_amdgcn_s_setprio(1);   // the recurrence waves ahead of the workers at issue
  }

  {  // W_hh[dir][c][j0 .. j0+31] for all 3H rows c, transposed [jj][c] in 8-deep c packs
    const float* W = a.w_hh + (size_t)dir * 3 * H * H;
    for (int v = tid; v < (3 * H / 8) * (U / 4); v += NT) {
      const int cb = v / (U / 4), jq = (v % (U / 4)) * 4;
      v4f w[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) w[e] = ld4(W + (size_t)(cb * 8 + e) * H + j0 + jq);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        Wt[(jq + u) * WPQ + cb] = pack8<F16>(v8f{w[0][u], w[1][u], w[2][u], w[3][u], w[4][u], w[5][u], w[6][u], w[7][u]});
    }
  }
  __syncthreads();

  const int Gp = a.G;
  const __amdgpu_buffer_rsrc_t rg_ = rsrc(a.xbuf + (size_t)dir * 2 * Gp * ROWS * 3 * H);   // 16-bit [2][Gp][RB][NKB][64][8]
  float dhz[4] = {0.f, 0.f, 0.f, 0.f};
  float sb[4] = {0.f, 0.f, 0.f, 0.f};   // sums of dar, daz, dan, dan * r over t and the lane's rows

  for (int step = 0; step < T; ++step) {
    const int t = dir == 0 ? T - 1 - step : step;
    const int tprev = dir == 0 ? t - 1 : t + 1;
    const bool edge = (step == T - 1);
    stamp(a, step, 0);
    float g_r[4], g_z[4], g_n[4], g_h[4], dyv[4], hpv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = min(rbase + lq * 4 + r, b_last);
      const float* gs = a.gates + (((size_t)dir * T + t) * B + b) * 4 * H;   // unit-interleaved (store_gates_il)
      const v4f gv = *reinterpret_cast<const v4f*>(gs + 4 * j);
      g_r[r] = gv.x;
      g_z[r] = gv.y;
      g_n[r] = gv.z;
      g_h[r] = gv.w;
      dyv[r] = a.dy[((size_t)b * T + t) * 2 * H + dir * H + j];
      hpv[r] = edge ? 0.f : a.y_in[((size_t)b * T + tprev) * 2 * H + dir * H + j];
    }
    float full[4] = {0.f, 0.f, 0.f, 0.f};
    if (step > 0) {
      lp2_wait(a, dir, group, kh * KS, KS, step, per);
      stamp(a, step, 1);
      const unsigned base = (unsigned)(((((size_t)((step - 1) & 1) * Gp + group) * RB + rb) * NKB * 64 + lane) * 16);
      v4f dv[3 * KS];   // dv[3 i + g] = k block g * 16 + kh * KS + i (gate g of producer kh * KS + i)
#pragma unroll
      for (int i = 0; i < KS; ++i)
#pragma unroll
        for (int g = 0; g < 3; ++g) dv[3 * i + g] = ld4_sc1(rg_, base + (g * 16 + kh * KS + i) * 1024);
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      auto blk = [&](int n) { return (n % 3) * 16 + kh * KS + n / 3; };
      u32x4 wv[2][2];
#pragma unroll
      for (int ub = 0; ub < 2; ++ub) wv[0][ub] = Wt[(ub * 16 + lr) * WPQ + blk(0) * 4 + lq];
#pragma unroll
      for (int n = 0; n < 3 * KS; ++n) {
        const int c = n & 1;
        if (n + 1 < 3 * KS) {
#pragma unroll
          for (int ub = 0; ub < 2; ++ub) wv[c ^ 1][ub] = Wt[(ub * 16 + lr) * WPQ + blk(n + 1) * 4 + lq];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ub = 0; ub < 2; ++ub) acc[ub] = Ops::mma(__builtin_bit_cast(e8, dv[n]), __builtin_bit_cast(e8, wv[c][ub]), acc[ub]);
        __builtin_amdgcn_sched_barrier(0);
      }
      float* Xw = X + wave * 16 * kXP2;   // the partner's unit block (static per kh, see the forward)
      const float* Xp = X + (wave ^ RB) * 16 * kXP2;
      auto exchange = [&](auto KH_) {
        constexpr int K = decltype(KH_)::value;
#pragma unroll
        for (int r = 0; r < 4; ++r) Xw[(4 * lq + r) * kXP2 + lr] = acc[1 - K][r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float o = acc[K][r], p = Xp[(4 * lq + r) * kXP2 + lr];
          full[r] = K == 0 ? o + p : p + o;
        }
      };
      if (__builtin_amdgcn_readfirstlane(kh) == 0) exchange(std::integral_constant<int, 0>{});
      else exchange(std::integral_constant<int, 1>{});
      if (a.trace) {
        asm volatile("" ::"v"(full[0]));
        stamp(a, step, 2);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = rb * 16 + lq * 4 + r, b = b0 + rl;
      float dh = dyv[r];
      if (step > 0) dh += full[r] + dhz[r];
      const float rg = g_r[r], zg = g_z[r], ng = g_n[r], ghn = g_h[r], hp = hpv[r];
      const float dn = dh * (1.0f - zg);
      const float daz = dh * (hp - ng) * zg * (1.0f - zg);
      const float dan = dn * (1.0f - ng * ng);
      const float dar = dan * ghn * rg * (1.0f - rg);
      dhz[r] = dh * zg;
      dT[(rl * 3 + 0) * DTP + ju] = dar;
      dT[(rl * 3 + 1) * DTP + ju] = daz;
      dT[(rl * 3 + 2) * DTP + ju] = dan * rg;
      dI[rl * DTP + ju] = dan;
      if constexpr (DW) {   // the dg image of the dW workers, rounded as the dgh16 the dW GEMM reads; rows past
                            // the batch are zeros (their hand-off input is never written: 0 x garbage = NaN)
        using E1 = typename std::conditional<F16, _Float16, __bf16>::type;
        const bool in_batch = b <= b_last;
        Aimg[rl * kDgP + ju] = in_batch ? __builtin_bit_cast(unsigned short, (E1)dar) : (unsigned short)0;
        Aimg[rl * kDgP + 32 + ju] = in_batch ? __builtin_bit_cast(unsigned short, (E1)daz) : (unsigned short)0;
        Aimg[rl * kDgP + 64 + ju] = in_batch ? __builtin_bit_cast(unsigned short, (E1)(dan * rg)) : (unsigned short)0;
      }
      if (b <= b_last) {
        sb[0] += dar;
        sb[1] += daz;
        sb[2] += dan;
        sb[3] += dan * rg;
      }
    }
    __syncthreads();
    stamp(a, step, 3);
    if (!edge) {   // hand-off (16-bit): chunks (rb', k block g * 16 + slice), lane l: row l & 15, 8 units
      for (int v = tid; v < 3 * RB * 64; v += NT) {
        const int c = v >> 6, rbp = c / 3, g = c % 3, l = v & 63, row = rbp * 16 + (l & 15);
        if (b0 + row > b_last) continue;
        const float* src = dT + (row * 3 + g) * DTP + 8 * (l >> 4);
        st4_ho(rg_, (unsigned)((((((size_t)(step & 1) * Gp + group) * RB + rbp) * NKB + g * 16 + slice) * 64 + l) * 16),
               __builtin_bit_cast(v4f, pack8<F16>(cat8(ld4(src), ld4(src + 4)))), local);
      }
    }
    lp2_arrive(a, dir, group, slice, step, per, local);   // the hand-off only: dgh16 / dgi16 go out after it
    stamp(a, step, 4);
    for (int v = tid; v < 2 * ROWS * 3 * 4; v += NT) {   // 16-bit dgh (edge rows zero) and dgi: (row, gate, 8 units)
      const int which = v / (ROWS * 12), w = v % (ROWS * 12), row = w / 12, g = (w % 12) >> 2, q8 = w & 3, b = b0 + row;
      if (b > b_last) continue;
      const float* src = which == 0 || g < 2 ? dT + (row * 3 + g) * DTP + 8 * q8 : dI + row * DTP + 8 * q8;
      v4f pk = __builtin_bit_cast(v4f, pack8<F16>(cat8(ld4(src), ld4(src + 4))));
      if (which == 0) {
        if (edge) pk = v4f{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<v4f*>(a.dgh16 + (((size_t)dir * B + b) * T + t) * 3 * H + g * H + j0 + 8 * q8) = pk;
      } else {
        *reinterpret_cast<v4f*>(a.dgi16 + ((size_t)b * T + t) * 6 * H + dir * 3 * H + g * H + j0 + 8 * q8) = pk;
      }
    }
  }
  // bias-gradient partials: lanes lr, lr + 16, lr + 32, lr + 48, then the RB row-block waves in order
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    sb[q] += __shfl_xor(sb[q], 16);
    sb[q] += __shfl_xor(sb[q], 32);
  }
  if (lq == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) red[(wave * 4 + q) * 16 + lr] = sb[q];
  }
  __syncthreads();
  if (tid < 128) {
    const int k2 = tid >> 6, q = (tid >> 4) & 3, u = tid & 15;   // waves (rb, k2) = RB k2 + rb
    float v = red[((RB * k2) * 4 + q) * 16 + u];
#pragma unroll
    for (int r = 1; r < RB; ++r) v += red[((RB * k2 + r) * 4 + q) * 16 + u];
    a.dbias[(((size_t)(a.chunk * 8 + group) * 2 + dir) * 4 + q) * H + j0 + k2 * 16 + u] = v;
  }
}

size_t lds_bytes(int H, bool backward, int prec) {
  if (prec == kPrecF32) return backward ? bwd_lds_bytes(H) : fwd_lds_bytes(H);
  const size_t need = backward ? (size_t)kUnits * (3 * H + 16) * 2 + 64 * 4 * (kUnits + 4) * 4
                               : (size_t)3 * kUnits * (H + 16) * 2 + 64 * (kUnits + 4) * 4 + 48 * kXP * 4;
  // the sc1 hand-off is the form measured at ONE workgroup per CU (MI355X_MICROARCH.md, "Valid
  // forms" row 1): reserve more than half of the 160 KB so a second workgroup never fits
  return std::max<size_t>(need, 96 * 1024);
}

size_t lp2_lds_bytes(int H, bool backward, int RB, bool dw = false, bool ow = false) {
  const size_t rows = 16 * RB, nw = 2 * RB, xp = (RB == 2 ? kFusedIn : 40) + 1;
  const size_t need = backward ? (size_t)kUnits2 * ((3 * H + 16) / 8) * 16 + rows * 3 * (kUnits2 + 4) * 4 +
                                     rows * (kUnits2 + 4) * 4 + nw * 16 * kXP2 * 4 + nw * 4 * 16 * 4 +
                                     (dw ? (size_t)32 * kDgP * 2 + (size_t)4 * 32 * 256 : 0)
                               : (size_t)3 * kUnits2 * ((H + 16) / 8) * 16 + rows * (kUnits2 + 4) * 4 +
                                     (size_t)3 * kUnits2 * xp * 4 + nw * 3 * 16 * kXP2 * 4 +
                                     (ow ? (size_t)32 * 32 * 4 * 4 : 0);
  return std::max<size_t>(need, 96 * 1024);   // one workgroup per CU (see lds_bytes)
}

template <int H>
const void* lp2_kernel_ptr(bool backward, int prec, int RB) {
  if (RB == 4) {
    if (prec == kPrecF16)
      return backward ? reinterpret_cast<const void*>(gru_bwd_persistent_lp2_kernel<H, true, 4>)
                      : reinterpret_cast<const void*>(gru_fwd_persistent_lp2_kernel<H, true, 4>);
    return backward ? reinterpret_cast<const void*>(gru_bwd_persistent_lp2_kernel<H, false, 4>)
                    : reinterpret_cast<const void*>(gru_fwd_persistent_lp2_kernel<H, false, 4>);
  }
  if (prec == kPrecF16)
    return backward ? reinterpret_cast<const void*>(gru_bwd_persistent_lp2_kernel<H, true, 2>)
                    : reinterpret_cast<const void*>(gru_fwd_persistent_lp2_kernel<H, true, 2>);
  return backward ? reinterpret_cast<const void*>(gru_bwd_persistent_lp2_kernel<H, false, 2>)
                  : reinterpret_cast<const void*>(gru_fwd_persistent_lp2_kernel<H, false, 2>);
}

template <int H>
const void* lp2_dw_kernel_ptr(int prec) {
  return prec == kPrecF16 ? reinterpret_cast<const void*>(gru_bwd_persistent_lp2_kernel<H, true, 2, true>)
                          : reinterpret_cast<const void*>(gru_bwd_persistent_lp2_kernel<H, false, 2, true>);
}

template <int H>
const void* lp2_ow_kernel_ptr(int prec) {
  return prec == kPrecF16 ? reinterpret_cast<const void*>(gru_fwd_persistent_lp2_kernel<H, true, 2, true>)
                          : reinterpret_cast<const void*>(gru_fwd_persistent_lp2_kernel<H, false, 2, true>);
}

template <int H>
int lp2_ow_occupancy_ok(int prec) {
  static std::mutex mu;
  static int occ[3] = {-1, -1, -1};
  std::lock_guard<std::mutex> lk(mu);
  int& o = occ[prec];
  if (o < 0) {
    const void* k = lp2_ow_kernel_ptr<H>(prec);
    const size_t lds = lp2_lds_bytes(H, false, 2, false, true);
    o = 0;
    if (lds <= 160 * 1024 && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess)
      SRK_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k, 512, lds));
    (void)hipGetLastError();
  }
  return o >= 1 ? 1 : 0;
}

template <int H>
int lp2_dw_occupancy_ok(int prec) {
  static std::mutex mu;
  static int occ[3] = {-1, -1, -1};
  std::lock_guard<std::mutex> lk(mu);
  int& o = occ[prec];
  if (o < 0) {
    const void* k = lp2_dw_kernel_ptr<H>(prec);
    const size_t lds = lp2_lds_bytes(H, true, 2, true);
    o = 0;
    if (lds <= 160 * 1024 && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess)
      SRK_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k, 512, lds));
    (void)hipGetLastError();
  }
  return o >= 1 ? 1 : 0;
}

template <int H>
int lp2_occupancy_ok(bool backward, int prec, int RB = 2) {
  static std::mutex mu;
  static int occ[2][2][3] = {{{-1, -1, -1}, {-1, -1, -1}}, {{-1, -1, -1}, {-1, -1, -1}}};
  std::lock_guard<std::mutex> lk(mu);
  int& o = occ[RB == 4 ? 1 : 0][backward ? 1 : 0][prec];
  if (o < 0) {
    const void* k = lp2_kernel_ptr<H>(backward, prec, RB);
    const size_t lds = lp2_lds_bytes(H, backward, RB);
    SRK_CHECK_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    SRK_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k, 128 * RB, lds));
  }
  return o >= 1 ? 1 : 0;
}

template <int H>
const void* kernel_ptr(bool backward, int prec) {
  if (prec == kPrecBF16)
    return backward ? reinterpret_cast<const void*>(gru_bwd_persistent_lp_kernel<H, false>)
                    : reinterpret_cast<const void*>(gru_fwd_persistent_lp_kernel<H, false>);
  if (prec == kPrecF16)
    return backward ? reinterpret_cast<const void*>(gru_bwd_persistent_lp_kernel<H, true>)
                    : reinterpret_cast<const void*>(gru_fwd_persistent_lp_kernel<H, true>);
  return backward ? reinterpret_cast<const void*>(gru_bwd_persistent_kernel<H>)
                  : reinterpret_cast<const void*>(gru_fwd_persistent_kernel<H>);
}

template <int H>
int dc_occupancy_ok() {
  static std::mutex mu;
  static int occ = -1;
  std::lock_guard<std::mutex> lk(mu);
  if (occ < 0) {
    int o2 = 0;
    const std::pair<const void*, size_t> ks[3] = {
        {reinterpret_cast<const void*>(gru_fwd_persistent_dc_kernel<H, false>), dc_fwd_lds_floats(H) * 4},
        {reinterpret_cast<const void*>(gru_fwd_persistent_dc_kernel<H, true>), dc_fwd_lds_floats(H) * 4},
        {reinterpret_cast<const void*>(gru_bwd_persistent_dc_kernel<H>), dc_bwd_lds_floats(H) * 4}};
    for (const auto& k : ks) {
      SRK_CHECK_HIP(hipFuncSetAttribute(k.first, hipFuncAttributeMaxDynamicSharedMemorySize, (int)k.second));
      SRK_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o2, k.first, 512, k.second));
      occ = occ < 0 ? o2 : std::min(occ, o2);
    }
  }
  return occ >= 1 ? 1 : 0;
}

template <int H>
int occupancy_ok(bool backward, int prec, int grid) {
  static std::mutex mu;
  static int cus = -1, occ[2][3] = {{-1, -1, -1}, {-1, -1, -1}};
  std::lock_guard<std::mutex> lk(mu);
  if (cus < 0) {
    int dev = 0;
    SRK_CHECK_HIP(hipGetDevice(&dev));
    hipDeviceProp_t p;
    SRK_CHECK_HIP(hipGetDeviceProperties(&p, dev));
    cus = p.multiProcessorCount;
  }
  int& o = occ[backward ? 1 : 0][prec];
  if (o < 0) {
    const void* k = kernel_ptr<H>(backward, prec);
    const size_t lds = lds_bytes(H, backward, prec);
    SRK_CHECK_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    SRK_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k, 256, lds));
  }
  return (o >= 1 && grid <= cus) ? 1 : 0;   // one workgroup per CU: the sc1 hand-off form measured
}

}  // namespace

size_t fwd_lds_bytes(int H) { return (size_t)(3 * 16 * (H + 4) + 64 * 20 + 48 * kXP) * 4; }
size_t bwd_lds_bytes(int H) { return (size_t)(16 * (3 * H + 4) + 64 * 4 * 20) * 4; }

int gru_persistent_groups(int64_t H) {
  if (H != 512) return 0;
  return 4;   // 2 dirs x 4 groups x 32 slices = 256 workgroups (one per CU)
}

int gru_persistent_supported(int64_t B, int64_t T, int64_t H, bool backward) {
  const int gmax = gru_persistent_groups(H);
  if (gmax == 0) return 0;
  // byte offsets of the buffer instructions are 32-bit
  if ((double)B * T * 3 * H * 4 >= 2147483647.0 || (double)B * T * 2 * H * 4 >= 2147483647.0) return 0;
  const int64_t G = std::min<int64_t>((B + kRows - 1) / kRows, gmax);
  const int grid = (int)(2 * G * (H / kUnits));
  const int prec = matmul_prec();
  int ok = occupancy_ok<512>(backward, prec, grid);
  if (ok > 0 && prec != kPrecF32 && g_opt_gru_lp2) ok = lp2_occupancy_ok<512>(backward, prec);
  return ok < 0 ? 0 : ok;
}

// 16-bit recurrence over more than 256 rows: the 64-row workgroups (RB = 4) run up to 512 rows per
// launch instead of 256-row chunks one after the other (a fused input projection needs in <= 40)
bool lp2_wide(int64_t B, int prec, bool backward, int in_fused) {
  return prec != kPrecF32 && g_opt_gru_lp2 && g_opt_gru_lp_wide && B > 256 && in_fused <= 40 &&
         lp2_occupancy_ok<512>(backward, prec, 4) > 0;
}

int gru_dwhh_fused_parts(int64_t B, int64_t T) {
  const int prec = matmul_prec();
  if (!g_opt_gru_dwhh_fused || prec == kPrecF32 || !g_opt_gru_lp2 || T < 2 || lp2_wide(B, prec, true, 0)) return 0;
  if (lp2_dw_occupancy_ok<512>(prec) <= 0) return 0;
  return (int)((B + 255) / 256) * 8;
}

int gru_bias_part_rows(int64_t B) {
  const int prec = matmul_prec();
  if (lp2_wide(B, prec, true, 0)) return 64;
  return (prec != kPrecF32 && g_opt_gru_lp2) ? kRows2 : kRows;
}

int gru_persistent_launch(GruPArgs a, bool backward, hipStream_t s) {
  const int gmax = gru_persistent_groups(a.H);
  SRK_REQUIRE(gmax > 0 && a.H == 512, SRK_ERR_INVALID, "gru persistent: unsupported H");
  const int prec = matmul_prec();
  const bool wide = lp2_wide(a.B, prec, backward, a.x_in ? a.in : 0) && (!backward || a.dgi16 != nullptr);
  const int rows_per_launch = wide ? 512 : gmax * kRows;
  // 16-bit operands: the 32 x 32 workgroup kernels (the backward one writes the 16-bit outputs only)
  const bool lp2 = prec != kPrecF32 && g_opt_gru_lp2 && (!backward || a.dgi16 != nullptr);
  const int rows_g = wide ? 64 : lp2 ? kRows2 : kRows, slices = lp2 ? a.H / kUnits2 : a.H / kUnits;
  if (lp2 && lp2_occupancy_ok<512>(backward, prec) <= 0)
    SRK_REQUIRE(false, SRK_ERR_INVALID, "gru persistent: the 32 x 32 kernels do not fit one workgroup per CU");
  // fp32 forward: the two-chain 8-wave kernel (same grid, W slice and outputs)
  const bool dc = prec == kPrecF32 && g_opt_gru_dc && dc_occupancy_ok<512>() > 0;
  // 16-bit forward on 32-row workgroups: the output / input worker waves (option gru_fwd_worker; the gate
  // store offsets are 32-bit buffer offsets)
  const bool ow = lp2 && !backward && !wide && g_opt_gru_fwd_worker && a.y16 &&
                  (double)2 * a.T * a.B * 4 * a.H * 4 < 2147483647.0 && lp2_ow_occupancy_ok<512>(prec) > 0;
  for (int c0 = 0; c0 < a.B; c0 += rows_per_launch) {
    GruPArgs ac = a;
    ac.trace = g_opt_gru_trace;
    unsigned* health_host = nullptr;
    if (int rc = health_word(&health_host, &ac.health)) return rc;
    ac.spin_limit = g_opt_gru_spin_limit ? g_opt_gru_spin_limit : kSpinLimit;
    static const int flags_env = [] { const char* v = getenv("SRK_GRU_FLAGS"); return v && *v ? atoi(v) : 0; }();
    ac.flags = flags_env;
    ac.xcd_local = g_opt_gru_xcd_local;
    ac.dc_offset = g_opt_gru_dc_offset;
    ac.fast_cell = g_opt_gru_fast_cell;
    ac.dc_prio = g_opt_gru_dc_prio;
    ac.dw_mode = g_opt_gru_dwhh_fused;
    ac.b_begin = c0;
    ac.b_end = std::min(a.B, c0 + rows_per_launch);
    ac.G = (ac.b_end - c0 + rows_g - 1) / rows_g;
    ac.chunk = c0 / rows_per_launch;
    SRK_CHECK_HIP(hipMemsetAsync(ac.counters, 0, (size_t)kCounterFloats * 4, s));
    const dim3 grid((unsigned)(2 * ac.G * slices));
    const double flops = 2.0 * 2.0 * (double)(ac.b_end - c0) * 3 * a.H * a.H * (a.T - 1);
    ProfScope prof(backward ? (prec == kPrecF32 ? "gru_bwd_seq" : "gru_bwd_seq_lp")
                            : (prec == kPrecF32 ? "gru_fwd_seq" : "gru_fwd_seq_lp"), s, flops);
    prof.detail("gru_%s_persistent%s_kernel B%d T%d chunk%d", backward ? "bwd" : "fwd",
                dc ? "_dc" : wide ? "_lp2w" : lp2 ? (backward && ac.dw_part ? "_lp2dw" : ow ? "_lp2ow" : "_lp2") : (prec == kPrecF32 ? "" : "_lp"),
                ac.b_end - c0, a.T, ac.chunk);
    if (dc && backward)
      hipLaunchKernelGGL((gru_bwd_persistent_dc_kernel<512>), grid, dim3(512), dc_bwd_lds_floats(512) * 4, s, ac);
    else if (dc && ac.x_in)
      hipLaunchKernelGGL((gru_fwd_persistent_dc_kernel<512, true>), grid, dim3(512), dc_fwd_lds_floats(512) * 4, s, ac);
    else if (dc)
      hipLaunchKernelGGL((gru_fwd_persistent_dc_kernel<512, false>), grid, dim3(512), dc_fwd_lds_floats(512) * 4, s, ac);
    else if (lp2 && backward && ac.dw_part) {   // with the fused recurrent weight gradient (gru_dwhh_fused_parts)
      SRK_REQUIRE(!wide && ac.y16_in, SRK_ERR_INTERNAL, "gru persistent: fused dW_hh needs the 32-row kernel and y16");
      hipLaunchKernelGGL(reinterpret_cast<void (*)(GruPArgs)>(const_cast<void*>(lp2_dw_kernel_ptr<512>(prec))), grid,
                         dim3(512), lp2_lds_bytes(512, true, 2, true), s, ac);
    } else if (lp2 && !backward && ow) {   // the forward with the output / input worker waves
      hipLaunchKernelGGL(reinterpret_cast<void (*)(GruPArgs)>(const_cast<void*>(lp2_ow_kernel_ptr<512>(prec))), grid,
                         dim3(512), lp2_lds_bytes(512, false, 2, false, true), s, ac);
    } else if (lp2)
      hipLaunchKernelGGL(reinterpret_cast<void (*)(GruPArgs)>(const_cast<void*>(lp2_kernel_ptr<512>(backward, prec, wide ? 4 : 2))),
                         grid, dim3(wide ? 512 : 256), lp2_lds_bytes(512, backward, wide ? 4 : 2), s, ac);
    else
      hipLaunchKernelGGL(reinterpret_cast<void (*)(GruPArgs)>(const_cast<void*>(kernel_ptr<512>(backward, prec))), grid,
                         dim3(256), lds_bytes(512, backward, prec), s, ac);
    SRK_CHECK_HIP(hipGetLastError());
  }
  return SRK_OK;
}

}  // namespace srk

namespace srk {
int health_word(unsigned** host, unsigned** dev) {
  static std::mutex mu;
  static unsigned* h = nullptr;
  static unsigned* d = nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (!h) {
    void* p = nullptr;
    SRK_CHECK_HIP(hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *static_cast<volatile unsigned*>(p) = 0;
    void* dp = nullptr;
    SRK_CHECK_HIP(hipHostGetDevicePointer(&dp, p, 0));
    h = static_cast<unsigned*>(p);
    d = static_cast<unsigned*>(dp);
  }
  *host = h;
  *dev = d;
  return SRK_OK;
}
}  // namespace srk

extern "C" int srk_health_check(int sync) {
  SRK_API_BEGIN
  if (sync) SRK_CHECK_HIP(hipDeviceSynchronize());
  unsigned *h = nullptr, *d = nullptr;
  if (int rc = srk::health_word(&h, &d)) return rc;
  const unsigned v = __atomic_load_n(h, __ATOMIC_ACQUIRE);
  SRK_REQUIRE(v == 0, SRK_ERR_TIMEOUT,
              "a persistent GRU kernel's spin-wait timed out (its workgroups were not all co-resident): "
              "the recurrence results since then are invalid");
  return SRK_OK;
  SRK_API_END
}

extern "C" int srk_health_reset(void) {
  SRK_API_BEGIN
  SRK_CHECK_HIP(hipDeviceSynchronize());
  unsigned *h = nullptr, *d = nullptr;
  if (int rc = srk::health_word(&h, &d)) return rc;
  __atomic_store_n(h, 0u, __ATOMIC_RELEASE);
  return SRK_OK;
  SRK_API_END
}

extern "C" int64_t srk_spin_timeouts(void) {
  unsigned long long v = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(srk::g_spin_timeouts), sizeof(v)) != hipSuccess) return -1;
  return (int64_t)v;
}

// Host-side audit of the step-ordering words (tests/test_gru_audit.py, no GPU needed): plans the
// launches of gru_persistent_launch for a batch of B rows (256-row chunks, the variant the current
// options and precision select) and walks every word each workgroup polls, stores or adds to with
// the kernels' own index helpers.  *max_word = the largest word touched (must stay below the census
// at kCensusOff), *chunks = launches, *census = kCensusOff.  A fault that depends on the chunk
// (b_begin > 0) would need a chunk-dependent word: none of these indices involves b_begin.
extern "C" int srk_gru_audit_words(int64_t B, int precision, int backward, int64_t* max_word, int64_t* chunks,
                                   int64_t* census) {
  SRK_API_BEGIN
  SRK_REQUIRE(B > 0 && max_word && chunks && census && precision >= 0 && precision <= 2, SRK_ERR_INVALID,
              "gru_audit_words: bad arguments");
  using namespace srk;
  const bool lp2 = precision != kPrecF32 && g_opt_gru_lp2;
  const bool wide = lp2 && g_opt_gru_lp_wide && B > 256;   // as lp2_wide (occupancy aside)
  const int rows_per_launch = wide ? 512 : gru_persistent_groups(512) * kRows;
  const bool dc = precision == kPrecF32 && g_opt_gru_dc;
  const int rows_g = wide ? 64 : lp2 ? kRows2 : kRows, S = lp2 ? 512 / kUnits2 : 512 / kUnits;
  int64_t mx = -1, n = 0;
  auto see = [&](int w) { mx = std::max<int64_t>(mx, w); };
  for (int64_t c0 = 0; c0 < B; c0 += rows_per_launch, ++n) {
    const int G = (int)((std::min<int64_t>(B, c0 + rows_per_launch) - c0 + rows_g - 1) / rows_g);
    for (int dir = 0; dir < 2; ++dir)
      for (int group = 0; group < G; ++group) {
        see(pw_counter(dir, G, group));
        if (dc) {
          for (int c = 0; c < 2; ++c)
            for (int rb = 0; rb < 2; ++rb)
              for (int kh = 0; kh < 2; ++kh) {
                for (int lane = 0; lane < 32; ++lane) see(pw_flag_dc(dir, G, group, c, rb, 32 * kh + lane));   // dc_wait
                for (int slice = 0; slice < S; ++slice) see(pw_flag_dc(dir, G, group, c, rb, 2 * slice + kh));   // dc_flag
              }
        } else if (lp2) {
          for (int first = 0; first < S; first += 8)
            for (int lane = 0; lane < 8; ++lane) see(pw_flag_lp2(dir, G, group, first + lane));   // lp2_wait
          for (int slice = 0; slice < S; ++slice) see(pw_flag_lp2(dir, G, group, slice));          // lp2_arrive
        } else {
          for (int lane = 0; lane < S; ++lane) see(pw_flag64(dir, G, group, lane));   // sync_wait
          for (int slice = 0; slice < S; ++slice) see(pw_flag64(dir, G, group, slice));   // sync_arrive
        }
      }
  }
  (void)backward;   // the backward kernels use the same words as their forward twins
  *max_word = mx;
  *chunks = n;
  *census = kCensusOff;
  return SRK_OK;
  SRK_API_END
}

