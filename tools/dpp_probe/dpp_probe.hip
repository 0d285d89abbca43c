// Root-cause probe for the hand-written v_cndmask_b32_dpp quad transpose that
// round 1 tried and dropped (wrong results).  Diagnostic only, not part of the
// engine.  One wave; every lane holds f4 {4·lane + q}; the engine's
// quad_transpose (C++: DPP movs + selects, hazards handled by the compiler) is
// the reference, and the first transpose round (xor-1 exchange) is redone in
// inline asm with the fused select, in the two forms that differ only in the
// DPP read-after-VALU-write wait states:
//   variant 0: t = select(...) then immediately v_cndmask_b32_dpp reading t;
//   variant 1: the same with s_nop 1 between them (the ISA asks for 2 wait
//              states between a VALU write of a VGPR and a DPP read of it).
// The inline asm declares vcc clobbered in both (an undeclared vcc write is the
// other candidate cause: the compiler keeps live masks in vcc).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int CTRL> __device__ __forceinline__ float dpp_quad(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// round 1 of the engine's quad_transpose (nerfhip.hip), C++ form
__device__ f4 round1_cpp(f4 v, int c) {
  const bool o1 = c & 1;
  float r0 = dpp_quad<0xB1>(o1 ? v[0] : v[1]), r1 = dpp_quad<0xB1>(o1 ? v[2] : v[3]);
  v[0] = o1 ? r0 : v[0];
  v[1] = o1 ? v[1] : r0;
  v[2] = o1 ? r1 : v[2];
  v[3] = o1 ? v[3] : r1;
  return v;
}

// fused form: t = o1 ? v0 : v1 ; v1' = o1 ? v1 : dpp(t) ; v0' = !o1 ? v0 : dpp(t)
template <int NOP>
__device__ f4 round1_asm(f4 v, int c) {
  const uint64_t odd = __builtin_amdgcn_ballot_w64((c & 1) != 0);
  float t0, t1, n0, n1, n2, n3;
  if (NOP) {
    asm volatile(
        "s_mov_b64 vcc, %[m]\n\t"
        "v_cndmask_b32 %[t0], %[v1], %[v0], vcc\n\t"     // t0 = odd ? v0 : v1
        "v_cndmask_b32 %[t1], %[v3], %[v2], vcc\n\t"     // t1 = odd ? v2 : v3
        "s_nop 1\n\t"
        "v_cndmask_b32_dpp %[n1], %[t0], %[v1], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %[n3], %[t1], %[v3], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_not_b64 vcc, %[m]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_dpp %[n0], %[t0], %[v0], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %[n2], %[t1], %[v2], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        : [t0] "=&v"(t0), [t1] "=&v"(t1), [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2),
          [n3] "=&v"(n3)
        : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [m] "s"(odd)
        : "vcc");
  } else {
    asm volatile(
        "s_mov_b64 vcc, %[m]\n\t"
        "v_cndmask_b32 %[t0], %[v1], %[v0], vcc\n\t"
        "v_cndmask_b32 %[t1], %[v3], %[v2], vcc\n\t"
        "v_cndmask_b32_dpp %[n1], %[t0], %[v1], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %[n3], %[t1], %[v3], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_not_b64 vcc, %[m]\n\t"
        "v_cndmask_b32_dpp %[n0], %[t0], %[v0], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_cndmask_b32_dpp %[n2], %[t1], %[v2], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        : [t0] "=&v"(t0), [t1] "=&v"(t1), [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2),
          [n3] "=&v"(n3)
        : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [m] "s"(odd)
        : "vcc");
  }
  f4 o = {n0, n1, n2, n3};
  return o;
}

// variant 2: variant 1's asm WITHOUT declaring vcc, placed between two uses of
// the same lane mask by compiler-generated selects (the compiler keeps that
// mask in vcc across the asm block)
__device__ f4 round1_asm_undeclared(f4 v, int c, f4& after) {
  const bool o1 = c & 1;
  const float keep0 = o1 ? v[0] : v[1], keep1 = o1 ? v[2] : v[3];
  const uint64_t odd = __builtin_amdgcn_ballot_w64((c & 1) != 0);
  float t0, t1, n0, n1, n2, n3;
  asm volatile(
      "s_mov_b64 vcc, %[m]\n\t"
      "v_cndmask_b32 %[t0], %[v1], %[v0], vcc\n\t"
      "v_cndmask_b32 %[t1], %[v3], %[v2], vcc\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_dpp %[n1], %[t0], %[v1], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %[n3], %[t1], %[v3], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_not_b64 vcc, %[m]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32_dpp %[n0], %[t0], %[v0], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "v_cndmask_b32_dpp %[n2], %[t1], %[v2], vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      : [t0] "=&v"(t0), [t1] "=&v"(t1), [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2),
        [n3] "=&v"(n3)
      : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [m] "s"(odd));
  // the same mask again after the asm
  after[0] = o1 ? keep1 : keep0;
  after[1] = o1 ? v[3] : v[1];
  after[2] = o1 ? n0 : n1;
  after[3] = o1 ? n2 : n3;
  f4 o = {n0, n1, n2, n3};
  return o;
}

__global__ void probe(float* out) {
  const int lane = threadIdx.x;
  const int c = lane & 15;
  f4 v = {4.f * lane + 0, 4.f * lane + 1, 4.f * lane + 2, 4.f * lane + 3};
  f4 r = round1_cpp(v, c);
  f4 a0 = round1_asm<0>(v, c);
  f4 a1 = round1_asm<1>(v, c);
  f4 after;
  f4 a2 = round1_asm_undeclared(v, c, after);
  const bool o1 = c & 1;
  f4 want_after = {o1 ? (o1 ? v[2] : v[3]) : (o1 ? v[0] : v[1]), o1 ? v[3] : v[1],
                   o1 ? r[0] : r[1], o1 ? r[2] : r[3]};
  for (int q = 0; q < 4; ++q) {
    out[(0 * 64 + lane) * 4 + q] = r[q];
    out[(1 * 64 + lane) * 4 + q] = a0[q];
    out[(2 * 64 + lane) * 4 + q] = a1[q];
    out[(3 * 64 + lane) * 4 + q] = a2[q];
    out[(4 * 64 + lane) * 4 + q] = after[q];
    out[(5 * 64 + lane) * 4 + q] = want_after[q];
  }
}

int main() {
  float* d;
  float h[6 * 64 * 4];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* name[4] = {"", "no s_nop before the DPP reads", "s_nop 1 before the DPP reads",
                         "vcc written but not declared clobbered"};
  for (int v = 1; v <= 3; ++v) {
    int bad = 0, first = -1;
    for (int i = 0; i < 256; ++i)
      if (h[v * 256 + i] != h[i]) { ++bad; if (first < 0) first = i; }
    printf("variant %d (%s): %d / 256 elements differ from the C++ transpose", v - 1, name[v],
           bad);
    if (first >= 0)
      printf("; first at lane %d q %d: got %.0f want %.0f", first / 4, first % 4,
             h[v * 256 + first], h[first]);
    printf("\n");
  }
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += h[4 * 256 + i] != h[5 * 256 + i];
  printf("variant 2: compiler-generated selects after the asm (same lane mask): %d / 256 wrong\n",
         bad);
  hipFree(d);
  return 0;
}
