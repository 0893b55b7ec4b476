// Internal interface between gru.hip (entry points, per-step kernels) and gru_persistent.hip
// (one-launch-per-layer recurrence kernels).
#pragma once
#include <algorithm>

#include "srk_internal.h"

namespace srk {

// Arrival counters / per-producer flags of the persistent kernels ([2 directions][groups <= 4] at a
// 64-B stride, or [2][G][32] flags: words 0..255; the fp32 two-chain kernels' per-wave flags
// [2 dir][G][2 chains][2 row blocks][32 slices][2 k halves]: words 0..2047), the XCD census in
// words kCensusOff..+8; zeroed by a hipMemsetAsync of exactly this block before every launch.
constexpr int kCounterFloats = 4096;
constexpr int kCensusOff = 4080;
// Word indices of the step-ordering state inside that block — host + device, so the kernels and
// srk_gru_audit_words (a host-side check of every word a launch plan touches) share one arithmetic.
__host__ __device__ constexpr int pw_counter(int dir, int G, int group) { return (dir * G + group) * 16; }
__host__ __device__ constexpr int pw_flag64(int dir, int G, int group, int slot) { return (dir * G + group) * 32 + slot; }
__host__ __device__ constexpr int pw_flag_lp2(int dir, int G, int group, int slot) { return (dir * G + group) * 16 + slot; }
__host__ __device__ constexpr int pw_flag_dc(int dir, int G, int group, int c, int rb, int slot) {
  return (((dir * G + group) * 2 + c) * 2 + rb) * 64 + slot;
}
// Hand-off ring depth of the persistent kernels (slots per direction in the workspace): the fp32
// two-chain kernels need 3 (a wave waits only for the producers of its k half, see gru_persistent.hip)
constexpr int kHandoffSlots = 3;
constexpr int kFusedIn = 64;   // widest layer input whose projection the forward kernels fuse

struct GruPArgs {
  int B, T, H;
  int G;                 // 64-row groups in this launch
  int b_begin, b_end;    // batch rows [b_begin, b_end) of this launch
  const float* gi;       // fwd: [B*T][6H]
  const float* w_hh;     // [2][3H][H]
  const float* b_hh;     // [2][3H]
  float* y;              // fwd output [B][T][2H] (also the h hand-off buffer)
  const float* y_in;     // bwd: the forward output
  float* gates;          // [2][T][B][4H]
  const float* dy;       // bwd: [B][T][2H]
  float* dgi;            // bwd: [B*T][6H]
  float* dgh;            // bwd: [2][B][T][3H] (also the dg hand-off buffer)
  float* dgh_edge;       // bwd: [2][B][3H]
  float* xbuf;           // hand-off ping-pong: fwd h [2 dir][2][B][H], bwd dg [2 dir][2][B][3H]
  unsigned* counters;    // kCounterFloats words
  int flags;             // 1: per-producer step flags [2][G][32] (sc1 stores) instead of arrival counters
  int xcd_local;         // 1: try the XCD-local hand-off (census at launch; plain stores kept in the XCD's L2)
  // 16-bit operand outputs of the bf16 / fp16 kernels (nullptr = off), for the GEMMs of the layer:
  uint16_t* y16;         // fwd: h [B][T][2H] rounded to 16 bit
  uint16_t* dgi16;       // bwd: dgi [B*T][6H] (replaces the fp32 dgi)
  uint16_t* dgh16;       // bwd: dgh [2][B][T][3H], edge rows zero (replaces dgh / dgh_edge)
  float* dbias;          // bwd with dgi16: bias-gradient partials [chunk * (256 / rows per group) + group][2 dir][4][H]
                         //   (sum over t and the group's rows of dar, daz, dan, dan * r)
  int chunk;             // index of this launch's 64*G-row batch chunk
  // fused small input projection (in <= kFusedIn, the 39 MFCC features of model_mfcc_bgru.py:25):
  // with x_in set the forward kernels compute gi_t = x_t W_ih^T + b_ih themselves (gi unused)
  const float* x_in;     // [B][T][in]
  const float* w_ih;     // [2][3H][in]
  const float* b_ih;     // [2][3H]
  int in;
  unsigned long long* trace;   // optional per-(workgroup, step) timestamps (tools/gru_trace.py)
  unsigned* health;      // host-pinned, device-mapped word: set when a spin-wait gives up (srk_health_check)
  unsigned spin_limit;   // s_sleep polls before a wait gives up (~2 s by default)
  unsigned dc_offset;    // fp32 two-chain kernels: chain 1 starts this many s_memrealtime ticks (10 ns) late
  int fast_cell;         // fp32 two-chain forward: hardware exp / rcp in the cell (v_exp_f32, v_rcp_f32)
  int dc_prio;           // fp32 two-chain kernels: 0 = equal priority, 1 / 2 = chain 0 / 1 at s_setprio 1
  // 16-bit backward with the recurrent weight gradient fused in (gru_dwhh_fused_parts): h_prev in 16 bit
  // (the forward's y16) and the per-(chunk, row group) partial dW_hh [part][2 dir][3H][H], summed by
  // dwhh_reduce_kernel
  const uint16_t* y16_in;
  float* dw_part;
  int dw_mode;           // option gru_dwhh_fused bits: 2 = h_prev fetched after the exchange barrier, 4 = recurrence waves at prio 1
};

size_t fwd_lds_bytes(int H);
size_t bwd_lds_bytes(int H);
// 1 if the persistent kernels can run this layer (H, co-residency, 32-bit buffer offsets).
int gru_persistent_supported(int64_t B, int64_t T, int64_t H, bool backward);
// Enqueue the whole recurrence (all T steps; batch split into co-resident chunks).
int gru_persistent_launch(GruPArgs a, bool backward, hipStream_t s);

// Runtime options (srk_set_option): persistent GRU recurrence on/off (default on).
extern int g_opt_gru_persistent;
extern unsigned long long* g_opt_gru_trace;   // device buffer or nullptr
extern unsigned g_opt_gru_spin_limit;          // 0 = default (~2 s); test hook "gru_spin_limit"
extern int g_opt_gru_xcd_local;                // XCD-local hand-off when the census allows (default 1)
extern int g_opt_gru_lp_wide;                 // 16-bit recurrence over > 256 rows: 64-row workgroups, one launch (default 1)
extern int g_opt_gru_lp2;                      // 16-bit recurrence on 32 x 32 workgroups (default 1)
extern int g_opt_gru_dc;                       // fp32 recurrence: two independent row chains per workgroup (default 1)
extern unsigned g_opt_gru_dc_offset;            // chain-1 start delay (ticks of 10 ns), default 200 (2 us)
extern int g_opt_gru_fast_cell;                 // fp32 two-chain forward: hardware exp / rcp cell math (default 1)
extern int g_opt_gru_dc_prio;                   // fp32 two-chain kernels: static priority of one chain (0, 1, 2)
// Batch rows per bias-gradient partial of the 16-bit backward kernel (32 or 64; 256-row launch chunks).
int gru_bias_part_rows(int64_t B);
// Partials of dW_hh the 16-bit backward kernel would write with the fused recurrent weight gradient
// (option gru_dwhh_fused; 32 x 32 workgroups, 256-row chunks): chunks x 8, or 0 when it does not apply
// (fp32, the 64-row workgroups of B > 256, the kernel not fitting one workgroup per CU, T < 2).
int gru_dwhh_fused_parts(int64_t B, int64_t T);
extern int g_opt_gru_dwhh_fused;               // fused recurrent weight gradient in the 16-bit backward (default 1)
extern int g_opt_gru_fwd_worker;               // 16-bit forward: output / input worker waves (default 0 until measured)
// Host-pinned health word (device-mapped pointer in *dev): non-zero once any persistent-kernel
// spin-wait has given up; read without a device synchronization by srk_health_check.
int health_word(unsigned** host, unsigned** dev);

}  // namespace srk
