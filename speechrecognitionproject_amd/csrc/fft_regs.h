// Register-resident FFT building blocks for the feature kernels (features.hip), gfx950.
// Complex values are 2-float ext vectors so the compiler emits packed v_pk_{add,mul,fma}_f32.
#pragma once
#include "srk_internal.h"

namespace srk {
namespace fftr {

// N = 640 real = 320 complex, factored 320 = 16 (j) x 20 (i): n = j + 16 i, k = k1 + 20 k2.
//   pass A (lane per (frame, j), 16 lanes / frame): 20-point DFT over i in registers,
//                                                   then twiddle W320^(j k1)
//   LDS transpose (row pitch 17 complex: conflict-free ds_read_b64 / ds_write_b64)
//   pass B (lane per (frame, k1), 20 lanes / frame): 16-point DFT over j in registers
// A wave processes 3 frames at a time (48 lanes in pass A, 60 in pass B); no workgroup barrier
// is needed inside the frame loop (each wave owns its LDS slices).
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v2f cm2(v2f a, v2f b) { return v2f{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ v2f mi2(v2f a) { return v2f{a.y, -a.x}; }   // -i * a

__device__ constexpr float kW16[4][4][2] = {
  {{1.f, 0.f}, {1.f, 0.f}, {1.f, 0.f}, {1.f, 0.f}},
  {{1.f, 0.f}, {9.238795325e-01f, -3.826834324e-01f}, {7.071067812e-01f, -7.071067812e-01f},
   {3.826834324e-01f, -9.238795325e-01f}},
  {{1.f, 0.f}, {7.071067812e-01f, -7.071067812e-01f}, {0.f, -1.f}, {-7.071067812e-01f, -7.071067812e-01f}},
  {{1.f, 0.f}, {3.826834324e-01f, -9.238795325e-01f}, {-7.071067812e-01f, -7.071067812e-01f},
   {-9.238795325e-01f, 3.826834324e-01f}}};

// a + (-i) b = (a.x + b.y, a.y - b.x) and a - (-i) b = (a.x - b.y, a.y + b.x): one VOP3P add each, the swap and
// the sign in its op_sel / neg modifiers (the compiler's form of mi2 then an add spends moves and sign-bit xors)
__device__ __forceinline__ v2f padd_mi(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ v2f psub_mi(v2f a, v2f b) {
  v2f r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a * w for a twiddle w held in registers: (a.x w.x, a.y w.x), then + (-a.y w.y, a.x w.y) by one fma
__device__ __forceinline__ v2f pcmul(v2f a, v2f w) {
  v2f t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(w));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]" : "=v"(r) : "v"(a), "v"(w), "v"(t));
  return r;
}

// radix-4 butterfly from the even pair's sum / difference (a0 + a2, a0 - a2) and the odd inputs a1, a3
__device__ __forceinline__ void dft4v_sd(v2f s02, v2f d02, v2f& a0, v2f& a1, v2f& a2, v2f& a3) {
  const v2f s13 = a1 + a3, v = a1 - a3;
  a0 = s02 + s13;
  a2 = s02 - s13;
  a1 = padd_mi(d02, v);
  a3 = psub_mi(d02, v);
}
__device__ __forceinline__ void dft4v(v2f& a0, v2f& a1, v2f& a2, v2f& a3) { dft4v_sd(a0 + a2, a0 - a2, a0, a1, a2, a3); }

__device__ __forceinline__ void dft5v(v2f& a0, v2f& a1, v2f& a2, v2f& a3, v2f& a4) {
  constexpr float c1 = 0.30901699437494745f, c2 = -0.8090169943749473f;
  constexpr float s1 = 0.9510565162951535f, s2 = 0.5877852522924732f;
  const v2f t1 = a1 + a4, t2 = a2 + a3, t3 = a1 - a4, t4 = a2 - a3;
  const v2f b1 = a0 + c1 * t1 + c2 * t2, b2 = a0 + c2 * t1 + c1 * t2;
  const v2f q1 = s1 * t3 + s2 * t4, q2 = s2 * t3 - s1 * t4;
  a0 = a0 + t1 + t2;
  a1 = padd_mi(b1, q1);
  a4 = psub_mi(b1, q1);
  a2 = padd_mi(b2, q2);
  a3 = psub_mi(b2, q2);
}

// in-place 20-point forward DFT, natural order in and out.  Good-Thomas prime-factor form (20 = 4 x 5,
// coprime): input n = (5 n1 + 4 n2) mod 20, output k = (5 k1 + 16 k2) mod 20, so that
// W20^(n k) = W4^(n1 k1) W5^(n2 k2) and no twiddles sit between the 4- and the 5-point stages.
__device__ __forceinline__ void dft20v(v2f (&a)[20]) {
  v2f y[5][4];
#pragma unroll
  for (int n2 = 0; n2 < 5; ++n2) {
    v2f t0 = a[(4 * n2) % 20], t1 = a[(5 + 4 * n2) % 20], t2 = a[(10 + 4 * n2) % 20], t3 = a[(15 + 4 * n2) % 20];
    dft4v(t0, t1, t2, t3);
    y[n2][0] = t0; y[n2][1] = t1; y[n2][2] = t2; y[n2][3] = t3;
  }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    v2f u0 = y[0][k1], u1 = y[1][k1], u2 = y[2][k1], u3 = y[3][k1], u4 = y[4][k1];
    dft5v(u0, u1, u2, u3, u4);
    a[(5 * k1) % 20] = u0; a[(5 * k1 + 16) % 20] = u1; a[(5 * k1 + 32) % 20] = u2;
    a[(5 * k1 + 48) % 20] = u3; a[(5 * k1 + 64) % 20] = u4;
  }
}

// a * W16^(q k1) for compile-time q, k1: W16^4 = -i and W16^{2,6} = (+-1 - i) / sqrt(2) take adds and
// one packed multiply instead of a complex product
__device__ __forceinline__ v2f tw16(v2f a, int q, int k1) {
  constexpr float c = 7.071067812e-01f;
  const int m = q * k1;
  if (m == 4) return mi2(a);
  if (m == 2) return c * v2f{a.x + a.y, a.y - a.x};
  if (m == 6) return c * v2f{a.y - a.x, -(a.x + a.y)};
  return cm2(a, v2f{kW16[q][k1][0], kW16[q][k1][1]});
}

// in-place 16-point forward DFT (j = 4p + q, k = k1 + 4 k2).  The -i twiddle of (q, k1) = (2, 2) is folded into
// the second stage's adds (padd_mi / psub_mi) instead of a swap and a sign flip of its own.
__device__ __forceinline__ void dft16v(v2f (&a)[16]) {
  v2f b[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v2f t0 = a[q], t1 = a[4 + q], t2 = a[8 + q], t3 = a[12 + q];
    dft4v(t0, t1, t2, t3);
    b[q][0] = t0; b[q][1] = t1; b[q][2] = t2; b[q][3] = t3;
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1)
      if (q > 0 && q * k1 != 4) b[q][k1] = tw16(b[q][k1], q, k1);
  }
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    v2f u0 = b[0][k1], u1 = b[1][k1], u2 = b[2][k1], u3 = b[3][k1];
    if (k1 == 2) dft4v_sd(padd_mi(u0, u2), psub_mi(u0, u2), u0, u1, u2, u3);   // u2 = -i b[2][2]
    else dft4v(u0, u1, u2, u3);
    a[k1] = u0; a[k1 + 4] = u1; a[k1 + 8] = u2; a[k1 + 12] = u3;
  }
}

// The packed-real untangle of one (A = Z[k], B = Z[N/2 - k]) pair on the packed fp32 pipe, with W = W_N^k:
// S = (A.x + B.x, A.y - B.y), U = (A.y + B.y, B.x - A.x), 2 X[k] = S + W U, 2 X[N/2 - k] = (S - W U)*; returns
// (|2 X[k]|^2, |2 X[N/2 - k]|^2).  Eight VOP3P instructions whose op_sel / neg modifiers do the component swaps and
// sign flips (the scalar form takes sixteen, and the compiler's packed form adds moves and sign-bit xors).
__device__ __forceinline__ v2f untangle_pk(v2f A, v2f B, v2f W) {
  v2f S, U, T, V, R, I, P;
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(S) : "v"(A), "v"(B));                                   // (ax + bx, ay - by)
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]" : "=v"(U) : "v"(A), "v"(B));      // (ay + by, bx - ax)
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(T) : "v"(W), "v"(U));                                 // (wx ux, wy ux)
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[1,0,0]"
      : "=v"(V) : "v"(W), "v"(U), "v"(T));                                                                  // W U
  asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,0] neg_hi:[0,1]" : "=v"(R) : "v"(S), "v"(V));                    // (sx + vr, sx - vr)
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] neg_hi:[0,1]" : "=v"(I) : "v"(S), "v"(V));                       // (sy + vi, sy - vi)
  asm("v_pk_mul_f32 %0, %1, %1" : "=v"(P) : "v"(R));
  asm("v_pk_fma_f32 %0, %1, %1, %2" : "=v"(P) : "v"(I), "v"(P));
  return P;
}

__device__ __forceinline__ void wave_lds_fence() {
  // orders this wave's LDS writes before its later LDS reads (no workgroup barrier needed)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace fftr
}  // namespace srk
