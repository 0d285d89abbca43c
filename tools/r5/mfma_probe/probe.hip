// Microbenchmark (development tool): cycles per k-step of the rows32 MFMA
// pattern — six v_mfma_f32_32x32x16_bf16 per k-step (five into a correction
// accumulator, one into the main one) at one wave per SIMD — with the B
// operand in AGPRs or VGPRs, with or without three ds_read_b128 A-fragment
// reads per k-step (pinned ahead of the MFMAs, waited for at the end).
// Output: one line per variant, median cycles per k-step over the waves.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
typedef float f16v __attribute__((ext_vector_type(16)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
struct S8 { u4 h, m, l; };
__device__ __forceinline__ f16v mf(u4 a, u4 b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ void x3(const S8& a, const S8& b, f16v& hi, f16v& lo) {
  lo = mf(a.h, b.l, lo); lo = mf(a.l, b.h, lo); lo = mf(a.m, b.m, lo);
  lo = mf(a.h, b.m, lo); lo = mf(a.m, b.h, lo); hi = mf(a.h, b.h, hi);
}
__device__ __forceinline__ S8 to_agpr(const S8& v) {
  S8 r;
  asm("" : "=a"(r.h) : "0"(v.h));
  asm("" : "=a"(r.m) : "0"(v.m));
  asm("" : "=a"(r.l) : "0"(v.l));
  return r;
}
template <int OFF> __device__ __forceinline__ u4 dsr(uint32_t base) {
  u4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base), "n"(OFF));
  return r;
}
template <int AG, int LDS, int NV = 0, int ST = 0, int DMA = 0, int SG = 0>
__global__ void __launch_bounds__(256, 1) k(const u4* in, float* out, unsigned long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) u4 sm[3 * 1024];
  const int t = threadIdx.x;
  for (int i = t; i < 3 * 1024; i += 256) sm[i] = in[i % 512];
  __syncthreads();
  S8 b[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    S8 v = {in[t + i], in[t + i + 1], in[t + i + 2]};
    b[i] = AG ? to_agpr(v) : v;
  }
  S8 a = {in[t], in[t + 3], in[t + 7]};
  f16v hi = {}, lo = {};
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)sm + 16 * (t & 63);
  float vv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) vv[q] = (float)(t + q);
  typedef __attribute__((address_space(3))) void lds_void;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, 0x7fffffff, 0x00020000);
  float* st_base = out + 65536 + blockIdx.x * 4096 * 4 + (t >> 6) * 4096 + (t & 63) * 4;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      if (DMA && (kk & 7) < 6) {   // six 1 KB LDS-DMA pieces per 8 k-steps per wave
        int v = 16 * (t + 256 * (kk & 7));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(sm + 2048 + 64 * (t >> 6)), 16, v, 0, 0, 0);
      }
      if (ST && (kk & 1) == 0) {   // one 16-B-per-lane non-temporal store per 2 k-steps
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 x = {vv[0], vv[1], vv[2], vv[3]};
        __builtin_nontemporal_store(x, reinterpret_cast<f4*>(st_base + 256 * (kk >> 1)));
      }
#pragma unroll
      for (int q = 0; q < NV; ++q) vv[q & 7] = fmaf(vv[q & 7], 1.0001f, 0.5f);
      S8 an = a;
      if (LDS) {
        an.h = dsr<0>(base + 1024 * (kk & 1));
        an.m = dsr<4096>(base + 1024 * (kk & 1));
        an.l = dsr<8192>(base + 1024 * (kk & 1));
        __builtin_amdgcn_sched_barrier(0);
      }
      x3(a, b[kk], hi, lo);
      if (SG) {   // interleave: MFMA, then NV/6 VALU, six times
#pragma unroll
        for (int m = 0; m < 6; ++m) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, (NV + 5) / 6, 0);
        }
      }
      if (LDS) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(an.h), "+v"(an.m), "+v"(an.l));
        __builtin_amdgcn_sched_barrier(0);
        a = an;
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((t & 63) == 0) cyc[blockIdx.x * 4 + (t >> 6)] = t1 - t0;
  if (DMA) asm volatile("s_waitcnt vmcnt(0)");
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) s += hi[q] + lo[q];
#pragma unroll
  for (int q = 0; q < 8; ++q) s += vv[q];
  out[blockIdx.x * 256 + t] = s;
}
template <int AG, int LDS, int NV = 0, int ST = 0, int DMA = 0, int SG = 0>
void run(const char* name, u4* in, float* out, unsigned long long* cyc, int iters) {
  hipLaunchKernelGGL((k<AG, LDS, NV, ST, DMA, SG>), dim3(256), dim3(256), 0, 0, in, out, cyc, iters);   // warm
  hipLaunchKernelGGL((k<AG, LDS, NV, ST, DMA, SG>), dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(1024);
  hipMemcpy(h.data(), cyc, 1024 * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("{\"variant\": \"%s\", \"cycles_per_kstep\": %.1f, \"mfma_floor\": 192}\n", name,
         (double)h[512] / (iters * 16.0));
}
int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  u4* in; float* out; unsigned long long* cyc;
  hipMalloc(&in, 8192 * 16);
  hipMalloc(&out, (65536 + 256 * 4096 * 4) * 4);
  hipMalloc(&cyc, 1024 * 8);
  std::vector<unsigned> hin(8192 * 4);
  for (size_t i = 0; i < hin.size(); ++i) hin[i] = 0x3f803f80u ^ (unsigned)(i * 2654435761u & 0x007f007fu);
  hipMemcpy(in, hin.data(), hin.size() * 4, hipMemcpyHostToDevice);
  run<1, 0>("B in AGPR, A in regs", in, out, cyc, iters);
  run<0, 0>("B in VGPR, A in regs", in, out, cyc, iters);
  run<1, 1>("B in AGPR, A from LDS (3 ds_read_b128 per k-step)", in, out, cyc, iters);
  run<0, 1>("B in VGPR, A from LDS", in, out, cyc, iters);
  run<1, 1, 10>("AGPR B, LDS A, +10 VALU per k-step", in, out, cyc, iters);
  run<1, 1, 20>("AGPR B, LDS A, +20 VALU per k-step", in, out, cyc, iters);
  run<1, 1, 30>("AGPR B, LDS A, +30 VALU per k-step", in, out, cyc, iters);
  run<1, 1, 40>("AGPR B, LDS A, +40 VALU per k-step", in, out, cyc, iters);
  run<1, 1, 0, 1>("AGPR B, LDS A, +1 store per 2 k-steps", in, out, cyc, iters);
  run<1, 1, 0, 0, 1>("AGPR B, LDS A, +6 LDS-DMA per 8 k-steps", in, out, cyc, iters);
  run<1, 1, 10, 1, 1>("AGPR B, LDS A, +10 VALU, stores, DMA", in, out, cyc, iters);
  run<1, 1, 30, 1, 1>("AGPR B, LDS A, +30 VALU, stores, DMA", in, out, cyc, iters);
  run<1, 1, 10, 0, 0, 1>("interleaved: +10 VALU", in, out, cyc, iters);
  run<1, 1, 20, 0, 0, 1>("interleaved: +20 VALU", in, out, cyc, iters);
  run<1, 1, 30, 0, 0, 1>("interleaved: +30 VALU", in, out, cyc, iters);
  run<1, 1, 40, 0, 0, 1>("interleaved: +40 VALU", in, out, cyc, iters);
  run<1, 1, 30, 1, 1, 1>("interleaved: +30 VALU, stores, DMA", in, out, cyc, iters);
  return 0;
}
