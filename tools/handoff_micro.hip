// Hand-off latency floor of the persistent GRU recurrence (VERDICT r04 "next" #4): two workgroups
// pass a 1 KB payload (64 lanes x 16 B, the MFMA-fragment chunk of csrc/gru_persistent.hip) and a
// step flag back and forth; the time per round trip / 2 is one producer -> consumer hop with the
// kernel's own protocol (flag store after the payload stores drained, consumer polls the flag with an
// sc1 load, then loads the payload with sc1 loads).
//
//   hipcc -O3 --offload-arch=gfx950 tools/handoff_micro.hip -o tools/_exp/handoff_micro
//   tools/_exp/handoff_micro            -> one line per variant: ns per hop (median of 5 launches)
//
// Variants (bit mask):
//   1  payload + flag stored write-through (sc1; the placement-independent protocol) instead of plain
//      stores that stay in the XCD's L2 (the XCD-local protocol)
//   2  no s_sleep between polls (the kernels sleep 64 clk between flag polls)
//   4  flag only (no payload)
//   8  4 waves per workgroup: wave 0 polls, a workgroup barrier releases the others, every wave loads
//      its 1 KB and stores its own, barrier, one lane publishes (the recurrence kernels' step shape)
//  16  partner on another XCD (blocks 0 and 1) instead of the same XCD (blocks 0 and 8)
//  32  pipelined polls: four flag loads in flight (issued ~64 clk apart), each checked as it returns
//      (vmcnt retires in order), instead of one load -> wait -> check -> sleep at a time
//  64  tagged payload (round 6, VERDICT r05 "next" #3): the step number rides in the last dword of every
//      lane's 16-B chunk, written by the chunk's one 16-B store; every lane polls its own chunk with an sc1
//      16-B load until the tag says `need` (__all over the wave), so the poll IS the payload load — no flag
//      store, no vmcnt(0) drain before it, no second L2 round trip.  The floor a tagged hand-off would have.
// Every spin is bounded (a hop that waits > ~1 s gives up and the run reports it), and every
// workgroup of the grid reaches the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int kSc1 = 16;
constexpr unsigned kSpin = 1u << 22;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

template <int V>
__global__ __launch_bounds__(256) void pingpong(unsigned* flags, float* payload, unsigned long long* out, int iters,
                                                unsigned* failed) {
  constexpr bool WT = V & 1, NOSLEEP = V & 2, NOPAY = V & 4, FOURW = V & 8, CROSS = V & 16, PIPE = V & 32, TAG = V & 64;
  const int partner = CROSS ? 1 : 8;
  const int role = blockIdx.x == 0 ? 0 : blockIdx.x == partner ? 1 : -1;
  if (role < 0) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned* my_flag = flags + 64 * role;          // separate 256-B lines
  unsigned* other_flag = flags + 64 * (1 - role);
  float* my_pay = payload + (size_t)role * 4 * 256 * 4;   // [wave][lane][4] floats
  float* other_pay = payload + (size_t)(1 - role) * 4 * 256 * 4;
  const auto rmy = rs(my_pay), rother = rs(other_pay), rflag = rs(my_flag);
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  __shared__ int bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    // wait: role 0 waits for the partner's step i (none at i = 0), role 1 for step i + 1
    const unsigned need = role == 0 ? (unsigned)i : (unsigned)(i + 1);
    if constexpr (TAG) {   // every wave polls its own chunks: the load that sees the tag carries the payload
      const unsigned off = (unsigned)((wave * 64 + lane) * 16);
      v4f x = {0.f, 0.f, 0.f, 0.f};
      if (need > 0) {
        unsigned spins = 0;
        while (true) {
          // the memory clobber re-issues the load every spin (the same sc1 load as the payload reads; it is not
          // hoisted as loop-invariant)
          asm volatile("" ::: "memory");
          x = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rother, (int)off, 0, kSc1));
          if (__all(__float_as_uint(x.w) >= need)) break;
          if (!NOSLEEP) __builtin_amdgcn_s_sleep(1);
          if (++spins >= kSpin) {
            if (lane == 0) bad = 1;
            break;
          }
        }
      }
      if (bad) break;
      acc += v4f{x.x, x.y, x.z, 0.f};
      const v4f v = {(float)i, acc.x, acc.y, __uint_as_float((unsigned)(i + 1))};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rmy, (int)off, 0, WT ? kSc1 : 0);
      continue;
    }
    if (need > 0) {
      if (wave == 0 && PIPE) {
        unsigned spins = 0;
        unsigned q0 = __hip_atomic_load(other_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_sleep(1);
        unsigned q1 = __hip_atomic_load(other_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_sleep(1);
        unsigned q2 = __hip_atomic_load(other_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_sleep(1);
        unsigned q3 = __hip_atomic_load(other_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (true) {
          if (q0 >= need) break;
          q0 = __hip_atomic_load(other_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (q1 >= need) break;
          q1 = __hip_atomic_load(other_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (q2 >= need) break;
          q2 = __hip_atomic_load(other_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (q3 >= need) break;
          q3 = __hip_atomic_load(other_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (++spins >= kSpin / 4) {
            if (lane == 0) bad = 1;
            break;
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (wave == 0) {
        unsigned spins = 0;
        while (true) {
          const unsigned v = __hip_atomic_load(other_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (v >= need) break;
          if (!NOSLEEP) __builtin_amdgcn_s_sleep(1);
          if (++spins >= kSpin) {
            if (lane == 0) bad = 1;
            break;
          }
        }
      }
      if (FOURW) __syncthreads();
    }
    if (bad) break;
    if (!NOPAY) {
      const unsigned off = (unsigned)((wave * 64 + lane) * 16);
      acc += __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rother, (int)off, 0, kSc1));
      const v4f v = {(float)i, acc.x, acc.y, (float)lane};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rmy, (int)off, 0, WT ? kSc1 : 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (FOURW) __syncthreads();
    if (threadIdx.x == 0) {
      if (WT) __hip_atomic_store(my_flag, (unsigned)(i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else __builtin_amdgcn_raw_buffer_store_b32((unsigned)(i + 1), rflag, 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    out[role * 4 + 0] = t1 - t0;
    out[role * 4 + 1] = xcc;
    out[role * 4 + 2] = (unsigned long long)(acc.x != acc.x);   // keep the loads live
    if (bad) atomicAdd(failed, 1u);
  }
}

template <int V>
double run(unsigned* flags, float* pay, unsigned long long* out, unsigned* failed, int iters, unsigned* xcc) {
  std::vector<double> ns;
  for (int rep = 0; rep < 5; ++rep) {
    hipMemset(flags, 0, 4096);
    hipMemset(pay, 0, 2 * 4 * 256 * 16);
    hipMemset(failed, 0, 4);
    hipLaunchKernelGGL(pingpong<V>, dim3(16), dim3((V & 8) ? 256 : 64), 0, 0, flags, pay, out, iters, failed);
    if (hipDeviceSynchronize() != hipSuccess) return -1.0;
    unsigned long long h[8];
    unsigned f = 0;
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    hipMemcpy(&f, failed, 4, hipMemcpyDeviceToHost);
    if (f) return -2.0;
    xcc[0] = (unsigned)h[1];
    xcc[1] = (unsigned)h[5];
    ns.push_back((double)h[0] * 10.0 / (2.0 * iters));   // 100 MHz ticks; a round trip is two hops
  }
  std::sort(ns.begin(), ns.end());
  return ns[2];
}

int main() {
  std::setvbuf(stdout, nullptr, _IOLBF, 0);   // a line per variant as it finishes (stdout may be a file)
  unsigned *flags, *failed;
  float* pay;
  unsigned long long* out;
  if (hipMalloc(&flags, 4096) || hipMalloc(&pay, 2 * 4 * 256 * 16) || hipMalloc(&out, 64) || hipMalloc(&failed, 4)) {
    std::printf("alloc failed\n");
    return 1;
  }
  const int iters = 4000;
  struct { int v; const char* what; } vs[] = {
      {0, "plain payload+flag (XCD-local), sleep 1 between polls"},
      {2, "plain payload+flag (XCD-local), no sleep"},
      {4, "flag only (XCD-local), sleep"},
      {6, "flag only (XCD-local), no sleep"},
      {8, "4 waves + barriers, plain (XCD-local), sleep"},
      {10, "4 waves + barriers, plain (XCD-local), no sleep"},
      {1, "write-through payload+flag, same XCD, sleep"},
      {17, "write-through payload+flag, other XCD, sleep"},
      {19, "write-through payload+flag, other XCD, no sleep"},
      {25, "4 waves + barriers, write-through, other XCD, sleep"},
      {32, "pipelined polls, plain payload+flag (XCD-local)"},
      {40, "pipelined polls, 4 waves + barriers, plain (XCD-local)"},
      {49, "pipelined polls, write-through, other XCD"},
      {64, "tagged payload (poll = load), XCD-local, sleep"},
      {66, "tagged payload (poll = load), XCD-local, no sleep"},
      {72, "tagged payload, 4 waves, XCD-local, sleep"},
      {81, "tagged payload, write-through, other XCD, sleep"},
  };
  for (auto& e : vs) {
    unsigned xcc[2] = {99, 99};
    double ns = -3;
    switch (e.v) {
      case 0: ns = run<0>(flags, pay, out, failed, iters, xcc); break;
      case 2: ns = run<2>(flags, pay, out, failed, iters, xcc); break;
      case 4: ns = run<4>(flags, pay, out, failed, iters, xcc); break;
      case 6: ns = run<6>(flags, pay, out, failed, iters, xcc); break;
      case 8: ns = run<8>(flags, pay, out, failed, iters, xcc); break;
      case 10: ns = run<10>(flags, pay, out, failed, iters, xcc); break;
      case 1: ns = run<1>(flags, pay, out, failed, iters, xcc); break;
      case 17: ns = run<17>(flags, pay, out, failed, iters, xcc); break;
      case 19: ns = run<19>(flags, pay, out, failed, iters, xcc); break;
      case 25: ns = run<25>(flags, pay, out, failed, iters, xcc); break;
      case 32: ns = run<32>(flags, pay, out, failed, iters, xcc); break;
      case 40: ns = run<40>(flags, pay, out, failed, iters, xcc); break;
      case 49: ns = run<49>(flags, pay, out, failed, iters, xcc); break;
      case 64: ns = run<64>(flags, pay, out, failed, iters, xcc); break;
      case 66: ns = run<66>(flags, pay, out, failed, iters, xcc); break;
      case 72: ns = run<72>(flags, pay, out, failed, iters, xcc); break;
      case 81: ns = run<81>(flags, pay, out, failed, iters, xcc); break;
    }
    std::printf("variant %2d  %-55s  %8.1f ns/hop  (xcc %u / %u)\n", e.v, e.what, ns, xcc[0], xcc[1]);
  }
  return 0;
}
