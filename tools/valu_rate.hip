// Microbenchmark: issue cost of packed vs scalar fp32 VALU ops and of ds_bpermute on gfx950, at 1 and
// 2 waves per SIMD (shader cycles per wave-instruction from s_memtime).  Sizes the K1 MFCC arithmetic.
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rate.hip -o tools/_exp/valu_rate && tools/_exp/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int kIters = 2048;

template <int MODE>
__global__ __launch_bounds__(256) void rate_kernel(float* out, unsigned long long* cyc, float s) {
  float a[16];
  v2f p[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    a[i] = s * (threadIdx.x + i);
    p[i] = v2f{a[i], a[i] + 1.0f};
  }
  const v2f m2 = v2f{s, s * 0.5f};
  const float m = s * 0.25f;
  const int addr = ((threadIdx.x + 1) & 63) * 4;
  __builtin_amdgcn_s_barrier();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (MODE == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(m), "v"(a[(i + 1) & 15]));
      if (MODE == 1) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[i]) : "v"(m2), "v"(p[(i + 1) & 15]));
      if (MODE == 2) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(p[i]) : "v"(m2));
      if (MODE == 3) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[i]) : "v"(m));
      if (MODE == 4) a[i] = __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(a[i])));
      if (MODE == 5) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(p[i]) : "v"(m2));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += a[i] + p[i].x + p[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE>
double run(int blocks) {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, blocks * 256 * sizeof(float));
  hipMalloc(&cyc, blocks * 4 * sizeof(unsigned long long));
  hipLaunchKernelGGL(rate_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0001f);
  hipLaunchKernelGGL(rate_kernel<MODE>, dim3(blocks), dim3(256), 0, 0, out, cyc, 1.0001f);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), cyc, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  hipFree(out);
  hipFree(cyc);
  double s = 0;
  for (auto v : h) s += (double)v;
  return s / h.size() / (16.0 * kIters);
}

int main() {
  const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_add_f32", "ds_bpermute_b32", "v_pk_mul_f32"};
  for (int wps = 1; wps <= 3; ++wps) {
    const int blocks = 256 * wps;   // 4 waves per block, one per SIMD: wps waves per SIMD
    double r[6] = {run<0>(blocks), run<1>(blocks), run<2>(blocks), run<3>(blocks), run<4>(blocks), run<5>(blocks)};
    for (int m = 0; m < 6; ++m)
      printf("%d wave(s)/SIMD  %-16s %6.2f cycles per wave-instruction (SIMD: %5.2f)\n", wps, names[m], r[m], r[m] / wps);
  }
  return 0;
}
