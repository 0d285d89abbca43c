// nerfhip.hip — MI355X (gfx950 / CDNA4) SIREN KV-fit engine.
//
// Replaces the per-epoch eager-PyTorch sequence of the reference training loop
// (nerf_attention/siren.py:98-105: zero_grad → SIREN.forward → F.mse_loss →
// backward → Adam.step → CosineAnnealingLR.step) with two hand-written kernels
// per epoch, for a whole GROUP of independent fits at once:
//
//   k_step_rows<W,D>    row-parallel: forward (sin(ω·(xWᵀ+b)), siren.py:33-34),
//                       MSE + dL/dŷ, backward dX chain; writes the activations
//                       Hᵢᵀ and pre-activation grads dZᵢᵀ (feature-major) that
//                       the weight gradients need.  One workgroup = 64 rows of
//                       one fit; one wave = 16 rows; every GEMM on the f32 MFMA
//                       v_mfma_f32_16x16x4_f32 in the "transposed" orientation
//                       (Zᵀ = W·Hᵀ) so each layer's accumulator IS the next
//                       layer's B operand (no LDS round trip, no shuffles).
//   k_step_params<W,D>  parameter-parallel: one workgroup per 64×64 tile of
//                       dWᵢ = dZᵢᵀ·Hᵢ₋₁ (K = seq_len, v_mfma_f32_32x32x2_f32),
//                       bias sums, then the Adam update of that tile
//                       (torch single-tensor Adam order, TORCH/optim/adam.py
//                       :457-547) writing both the canonical [out][in] weights
//                       and the transposed [in][out] copy the backward reads.
//
// The reduction over seq_len therefore happens inside one workgroup: no
// partial-gradient slabs, no atomics, fully deterministic.
//
// Scratch layout per fit (fp32, n_pad = seq_len rounded up to 64), all
// row-block-major: 16-row blocks, inside a block feature-major with the 16
// rows contiguous (64 B per feature):
//   H_i    [L_max+1][n_pad/16][W][16]  activations (input of linear layer i+1)
//   dZ_i   [L_max+1][n_pad/16][W][16]  grad at the pre-activation of layer i
//   G      [n_pad/16][D][16]           grad at the output (2(ŷ−y)/(N·D))
//   cos_i  [L_max+1][n_pad/16][W/16][64][4]  cos(ω z), MFMA-fragment order
//                                      (cos_0 is never stored: recomputed)
//
// Numerics: all fp32, inline ≈1-ulp sincos, f32-input MFMA = exact k-ordered
// fmaf chain.  Parity target: per-fit final cosine within 1e-3 of the
// reference PyTorch CPU path (BASELINE.json north_star).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <atomic>
#include <stdlib.h>
#include <math.h>
#include <type_traits>

#include "nerfhip.h"
#include "nerfhip_layout.h"

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Build split: the library is compiled as NERFHIP_PART = 0 (host ABI + small
// kernels) and one part per (hidden width, precision) (1..8 = W 64, 128, 256,
// 512 × fp32, bf16x3: those step kernels, both head dims), in parallel, and
// linked; without NERFHIP_PART the file is one translation unit.  Only KArgs
// and the launch templates have external linkage (nerfhip_detail).
#ifndef NERFHIP_PART
#define NERFHIP_PART (-1)
#endif

namespace nerfhip_detail {
struct KArgs {
  int32_t W, D, N, n_pad, n_fits, L_max, epochs, epoch, mode;
  int64_t p_stride, pt_stride, s_stride, t_stride, lp_stride, y_stride;
  const int32_t* fit_layers;
  const float* fit_omega;
  const float* pos;
  const float* target;
  float* tnorm;
  float* mean;
  float* stdv;
  float* params;
  float* params_t;
  float* m;
  float* v;
  float* scratch;
  const float* sched;
  float* loss_partial;
  float* y_out;
  float grad_scale;
  // split-K gradient reduction of small groups (nerfhip.h grad_partial):
  // n_split row slices write partial slabs gpart[fit][split][param]
  int32_t n_split;
  int64_t gp_stride;
  float* gpart;
  // 1 = the last-arriving slice of each parameter tile sums the slabs and
  // runs Adam itself (no k_adam_split launch); arrival counters, one int32
  // per tile, live at gpart + fit·gp_stride + ctr_off
  int32_t split_fused;
  int64_t ctr_off;
  // bf16x3 precision (NERFHIP_PRECISION_BF16X3): every MFMA weight operand as
  // exact 3-way bf16 split planes, forward and transposed (xoff layout)
  int32_t x3;
  int64_t ws_stride;
  uint16_t* wsplit;
  // row-step variant: 1 = the K-split kernel for small groups (k_step_rows_ks)
  int32_t rows_ks;
  // 1 = the 32-row kernel (k_step_rows32; bf16x3, W = 256, D = 128)
  int32_t rows32;
  // split-K parameter step on 64 × 64 tiles (ParamsCfg SMALL; split_for)
  int32_t small_tiles;
  // diagnostic builds only (NERFHIP_STAMPS): per-wave s_memrealtime stamps of
  // the parameter kernel, [blocks][4 waves][8] (NERFHIP_PSTAMPS = device address)
  unsigned long long* pstamps;
  // dynamic LDS (bytes) the regular row / parameter kernels launch with: an
  // occupancy knob (a padded row workgroup cannot share its CU with a second
  // row workgroup, only with a parameter one); 0 = none (make_args)
  uint32_t rows_dyn_lds, params_dyn_lds;
  // diagnostic builds only (NERFHIP_DIAG_FLIGHT): the launch's sequence number,
  // its group, a hash of the arguments the host sent, and the host-mapped
  // flight-recorder ring every workgroup marks on entry and exit
  uint32_t seq, group;
  uint64_t hash;
  unsigned char* flight;
};
template <int W, int D, bool X3> int launch_rows(const KArgs& a, hipStream_t st);
template <int W, int D, bool X3> int launch_params(const KArgs& a, hipStream_t st);
template <int W, int D> int launch_rows32(const KArgs& a, hipStream_t st);

// ---------------------------------------------------------------------------
// Flight recorder (NERFHIP_DIAG_FLIGHT builds only; tools/r6/flight.py).
// Every launch takes a slot of a host-mapped ring: the host writes what it
// launched (sequence number, kernel, epoch, group, grid, argument hash); every
// workgroup's thread 0 marks one byte on entry and one on exit, and checks the
// arguments it received against the hash and the fit's depth against L_max
// (a failed check is recorded and the workgroup returns without touching
// memory).  After a device fault the ring names the launches in flight.
// ---------------------------------------------------------------------------
constexpr int kFlightRing = 4096, kFlightHdr = 128, kFlightMaxB = 2048;
constexpr size_t kFlightSlot = kFlightHdr + 2 * (size_t)kFlightMaxB;
__host__ __device__ inline uint64_t flight_mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  return h;
}
__host__ __device__ inline uint64_t kargs_hash(const KArgs& a) {
  uint64_t h = 0x243f6a8885a308d3ull;
  const uint64_t v[] = {
      (uint64_t)a.W, (uint64_t)a.D, (uint64_t)a.N, (uint64_t)a.n_pad, (uint64_t)a.n_fits,
      (uint64_t)a.L_max, (uint64_t)a.epochs, (uint64_t)a.epoch, (uint64_t)a.mode,
      (uint64_t)a.p_stride, (uint64_t)a.pt_stride, (uint64_t)a.s_stride, (uint64_t)a.t_stride,
      (uint64_t)a.lp_stride, (uint64_t)a.y_stride, (uint64_t)(uintptr_t)a.fit_layers,
      (uint64_t)(uintptr_t)a.fit_omega, (uint64_t)(uintptr_t)a.pos, (uint64_t)(uintptr_t)a.target,
      (uint64_t)(uintptr_t)a.tnorm, (uint64_t)(uintptr_t)a.params, (uint64_t)(uintptr_t)a.params_t,
      (uint64_t)(uintptr_t)a.m, (uint64_t)(uintptr_t)a.v, (uint64_t)(uintptr_t)a.scratch,
      (uint64_t)(uintptr_t)a.sched, (uint64_t)(uintptr_t)a.loss_partial, (uint64_t)(uintptr_t)a.y_out,
      (uint64_t)a.n_split, (uint64_t)a.gp_stride, (uint64_t)(uintptr_t)a.gpart, (uint64_t)a.x3,
      (uint64_t)a.ws_stride, (uint64_t)(uintptr_t)a.wsplit, (uint64_t)a.rows_ks,
      (uint64_t)a.small_tiles, (uint64_t)a.seq, (uint64_t)a.group};
  for (uint64_t x : v) h = flight_mix(h, x);
  return h;
}
#ifdef NERFHIP_DIAG_FLIGHT
KArgs flight_stamp(const KArgs& a, int kid, unsigned grid);   // host: assign seq, hash, header
#define NERFHIP_KA(a, kid, grid) nerfhip_detail::flight_stamp((a), (kid), (unsigned)(grid))
#else
#define NERFHIP_KA(a, kid, grid) (a)
#endif
}  // namespace nerfhip_detail

namespace {
using nerfhip_detail::KArgs;

#ifdef NERFHIP_DIAG_FLIGHT
struct Flight {
  unsigned char* s = nullptr;
  unsigned b = 0;
  __device__ explicit Flight(const KArgs& a) {
    if (!a.flight) return;
    s = a.flight + (size_t)(a.seq % nerfhip_detail::kFlightRing) * nerfhip_detail::kFlightSlot;
    b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    if (threadIdx.x == 0 && b < nerfhip_detail::kFlightMaxB)
      __hip_atomic_store(s + nerfhip_detail::kFlightHdr + b, (unsigned char)1, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __device__ ~Flight() {
    if (s && threadIdx.x == 0 && b < nerfhip_detail::kFlightMaxB)
      __hip_atomic_store(s + nerfhip_detail::kFlightHdr + nerfhip_detail::kFlightMaxB + b,
                         (unsigned char)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // header words 8.. (device side): 8 seq seen by workgroup 0, 9 its argument
  // hash, 10 workgroups whose arguments failed the hash (flag), 11 depth out
  // of range (flag)
  __device__ void flag(int word, uint64_t v) {
    if (s && threadIdx.x == 0)
      __hip_atomic_store(reinterpret_cast<uint64_t*>(s) + word, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __device__ bool args_ok(const KArgs& a) {
    if (!s) return true;
    KArgs c = a;
    c.hash = 0;
    const uint64_t h = nerfhip_detail::kargs_hash(c);
    if (b == 0) { flag(8, a.seq); flag(9, h); }
    if (h != a.hash) { flag(10, 1ull + b); return false; }
    return true;
  }
  __device__ bool depth_ok(const KArgs& a, int L, int fit) {
    if (!s) return true;
    if (L >= 1 && L <= a.L_max && fit >= 0 && fit < a.n_fits) return true;
    flag(11, ((uint64_t)(uint32_t)L << 32) | (uint32_t)fit);
    return false;
  }
};
#define FLIGHT_ENTER()            \
  Flight flight_(a);              \
  if (!flight_.args_ok(a)) return;
#define FLIGHT_DEPTH(L, fit) \
  if (!flight_.depth_ok(a, (L), (fit))) return;
#else
#define FLIGHT_ENTER()
#define FLIGHT_DEPTH(L, fit)
#endif




#ifdef NERFHIP_STAMPS
// Diagnostic build only (tools/stamps.py): per-wave s_memtime stamps at the
// phase boundaries of the row kernel, written to a buffer nothing else reads.
__device__ unsigned long long* g_stamps = nullptr;
// The phase stamps go to a.pstamps + kRowStampsOff ([blocks][waves][16]): the
// kernel arguments reach every translation unit, g_stamps only part 0's.
constexpr size_t kRowStampsOff = 1u << 20;
#define STAMP(k)                                                                       \
  do {                                                                                 \
    if (a.pstamps && a.mode == 0 && (threadIdx.x & 63) == 0)                           \
      a.pstamps[kRowStampsOff +                                                        \
                ((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16 + (k)] = \
          __builtin_amdgcn_s_memtime();                                                \
  } while (0)
// accumulate cycles into g_stamps slot k (8..11) of this wave (part 0's
// kernels only, nerfhip_debug_set_stamps; a global
// read-modify-write: it waits for the vector-memory ops in flight, so
// NERFHIP_STAMPS_NOADD drops it where the phase totals and the clock matter)
#ifndef NERFHIP_STAMPS_NOADD
#define STAMP_ADD(k, v)                                                                \
  do {                                                                                 \
    if (g_stamps && (threadIdx.x & 63) == 0)                                           \
      g_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16 + (k)] += (v); \
  } while (0)
#else
#define STAMP_ADD(k, v) \
  do {                  \
  } while (0)
#endif
// s_memrealtime (100 MHz) into slot k (12, 13): the in-kernel clock is
// Δs_memtime / Δs_memrealtime × 100 MHz
#define STAMP_RT(k)                                                                    \
  do {                                                                                 \
    if (a.pstamps && a.mode == 0 && (threadIdx.x & 63) == 0)                           \
      a.pstamps[kRowStampsOff +                                                        \
                ((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16 + (k)] = \
          __builtin_amdgcn_s_memrealtime();                                            \
  } while (0)
#define MEMTIME() __builtin_amdgcn_s_memtime()
// the 32-row kernel's stamps: [blocks][4 waves][32] from a.pstamps + 262144
// (after the parameter and K-split kernels' regions), through a pointer the
// kernel hands to its phases (g_stamps is per translation unit)
// R32STAMP_ADD accumulates in registers (a read-modify-write of global
// memory would wait for every vector-memory op in flight and distort exactly
// the waits it measures); the kernel stores the sums at its end
#define R32STAMP_ADD(acc, k, v) \
  do {                          \
    (acc)[(k)] += (v);          \
  } while (0)
#define R32STAMP(p, k)                                                                 \
  do {                                                                                 \
    if ((p) && (threadIdx.x & 63) == 0)                                                \
      (p)[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define PSTAMP(k)                                                                      \
  do {                                                                                 \
    if (a.pstamps && (threadIdx.x & 63) == 0)                                          \
      a.pstamps[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (k)] =             \
          __builtin_amdgcn_s_memrealtime();                                            \
  } while (0)
// slots 5, 6 of the parameter kernel's wave record: HW_ID (CU / SIMD / SE)
// and XCC_ID, read once at entry
#define PSTAMP_HW()                                                                    \
  do {                                                                                 \
    if (a.pstamps && (threadIdx.x & 63) == 0) {                                        \
      const size_t o_ = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8;            \
      a.pstamps[o_ + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);                   \
      a.pstamps[o_ + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 20);                  \
    }                                                                                  \
  } while (0)
// the K-split row kernel's stamps, after the parameter kernel's 4096 x 4 x 8
#define KSTAMP(k)                                                                      \
  do {                                                                                 \
    if (a.pstamps && a.mode == 0 && (threadIdx.x & 63) == 0)                           \
      a.pstamps[131072 + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (k)] =    \
          __builtin_amdgcn_s_memrealtime();                                            \
  } while (0)
#else
#define R32STAMP_ADD(acc, k, v) \
  do {                          \
  } while (0)
#define R32STAMP(p, k) \
  do {                 \
  } while (0)
#define STAMP_RT(k) \
  do {             \
  } while (0)
#define PSTAMP(k) \
  do {            \
  } while (0)
#define PSTAMP_HW() \
  do {              \
  } while (0)
#define KSTAMP(k) \
  do {            \
  } while (0)
#define STAMP(k) \
  do {           \
  } while (0)
#define STAMP_ADD(k, v) \
  do {                  \
  } while (0)
#define MEMTIME() 0ull
#endif

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }
// scratch stores of the row kernel (activations / gradients for the parameter
// kernel and the backward): non-temporal, so ≈3 GB of once-written lines per
// launch do not evict the weight planes the LDS-DMA staging re-reads from L2
// (measured −5 % row-kernel time at W = 256 and 512; non-temporal loads of the
// scratch, in both kernels, measured 1.6 % slower on the sweep)
__device__ __forceinline__ void sst(float* p, float v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void sst4(float* p, f4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p));
}
// the row kernel's private cos(ωz) tiles (stored in the forward, re-read by
// the same workgroup's backward): NERFHIP_COS_NT=0 stores them L2-allocating
#ifndef NERFHIP_COS_NT
#define NERFHIP_COS_NT 1
#endif
__device__ __forceinline__ void cst4(float* p, f4 v) {
  if constexpr (NERFHIP_COS_NT) sst4(p, v); else st4(p, v);
}

template <int CTRL> __device__ __forceinline__ float dpp_quad(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// 4×4 transpose inside lane quads (two DPP quad_perm exchange rounds, xor 1
// then xor 2): lane b of a quad ends up with element b of every quad lane,
// v[k] = (lane k's v[b]).  The row kernel's accumulator lane (row c, group g)
// holds features 4g+q of one row; after the transpose lane 4a+b holds feature
// 4g+b of rows 4a..4a+3, which are adjacent in the row-block-major scratch —
// one 16-B store per lane writes a 16-feature × 16-row tile as one contiguous
// 1 KB run (whole 128-B lines) instead of four dword stores of 64-B pieces.
__device__ __forceinline__ f4 quad_transpose(f4 v, int c) {
  const bool o1 = c & 1, o2 = c & 2;
  float r0 = dpp_quad<0xB1>(o1 ? v[0] : v[1]), r1 = dpp_quad<0xB1>(o1 ? v[2] : v[3]);
  v[0] = o1 ? r0 : v[0];
  v[1] = o1 ? v[1] : r0;
  v[2] = o1 ? r1 : v[2];
  v[3] = o1 ? v[3] : r1;
  r0 = dpp_quad<0x4E>(o2 ? v[0] : v[2]);
  r1 = dpp_quad<0x4E>(o2 ? v[1] : v[3]);
  v[0] = o2 ? r0 : v[0];
  v[1] = o2 ? r1 : v[1];
  v[2] = o2 ? v[2] : r0;
  v[3] = o2 ? v[3] : r1;
  return v;
}

__device__ __forceinline__ f4 mfma16(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16v mfma32(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// sin and cos of one fp32 argument (torch.sin in the forward, its derivative
// cos in the backward, siren.py:34).  Cody–Waite reduction by π/2 with a
// 3-term fma split (exact quotient for |x| < 2^17, far beyond the |ω·z| ≲ 10²
// a SIREN sees), then minimax polynomials on [−π/4, π/4] (≈1 ulp, the same
// class as the SLEEF kernels ATen uses on CPU).  Kept branch-free and short:
// the OCML sincosf carries a Payne–Hanek path whose registers spill the
// W ≥ 256 step kernels.
#ifndef NERFHIP_SINCOS
#define NERFHIP_SINCOS 0
#endif
__device__ __forceinline__ void sincos_fast(float x, float* s_out, float* c_out) {
#if NERFHIP_SINCOS == 1
  // Cody–Waite by π (C1, C2 with 12 trailing zero bits: n·C exact for
  // |n| < 2^12), u = r/(2π) ∈ [−1/4, 1/4] revolutions, the hardware
  // v_sin_f32 / v_cos_f32, and the sign (−1)^n as a sign-bit xor
  {
    const float n = __builtin_rintf(x * 0.318309873342514038086f);
    float r = fmaf(n, -3.14062500000000000000e+00f, x);
    r = fmaf(n, -9.67502593994140625000e-04f, r);
    r = fmaf(n, -1.50995802528086642269e-07f, r);
    const float u = r * 0.159154936671257019043f;
    const uint32_t sg = (uint32_t)(int)n << 31;
    *s_out = __uint_as_float(__float_as_uint(__builtin_amdgcn_sinf(u)) ^ sg);
    *c_out = __uint_as_float(__float_as_uint(__builtin_amdgcn_cosf(u)) ^ sg);
    return;
  }
#elif NERFHIP_SINCOS == 2
  // reduction in revolutions (1/2π = hi + lo), the hardware v_sin / v_cos
  {
    const float n = __builtin_rintf(x * 0.159154936671257019043f);
    float u = fmaf(x, 0.159154936671257019043f, -n);
    u = fmaf(x, 6.42063824329852650408e-09f, u);
    *s_out = __builtin_amdgcn_sinf(u);
    *c_out = __builtin_amdgcn_cosf(u);
    return;
  }
#endif
  const float n = __builtin_rintf(x * 0.636619772367581343f);
  float r = fmaf(n, -1.57079601287841796875f, x);
  r = fmaf(n, -3.13916912752797361463e-07f, r);
  r = fmaf(n, -5.39030252995776476554e-15f, r);
  const int q = (int)n;
  const float r2 = r * r;
  float ps = fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
  ps = fmaf(r2, ps, -1.6666654611e-1f);
  ps = fmaf(r2 * r, ps, r);
  float pc = fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = fmaf(r2, pc, 4.166664568298827e-2f);
  pc = fmaf(r2 * r2, pc, fmaf(r2, -0.5f, 1.0f));
  // (the same selects as bit operations — a bit-field insert for the swap, a
  // sign xor from bits of q — compiled to fewer VALU but more live registers:
  // 33 → 139 spilled VGPRs at W = 256, −7 % on the sweep, ab_perm_sincos_bits.log)
  const bool swp = q & 1;
  float s = swp ? pc : ps;
  float c = swp ? ps : pc;
  s = (q & 2) ? -s : s;
  c = ((q + 1) & 2) ? -c : c;
  *s_out = s;
  *c_out = c;
}

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// ---------------------------------------------------------------------------
// bf16x3 precision: fp32 GEMMs on the bf16 matrix cores.
//
// x = h + m + l EXACTLY, each part a bf16: h keeps the top 8 significant bits
// of x (truncation), m the next 8 of the remainder, l the last ≤ 8 — both
// subtractions are exact in fp32.  A product is taken as
//   x·y ≈ h·h' + (h·l' + l·h' + m·m' + h·m' + m·h')
// and the dropped terms m·l', l·m', l·l' are < 2^-23·|x·y|: the class of
// fp32's own product rounding (2^-24), i.e. fp32 accuracy, not bf16.  The
// five correction products accumulate in their own fp32 accumulator
// (smallest first), so the h·h' chain takes as many roundings as an f32 MFMA
// chain.  Per 32-deep k-slice of a 16×16 tile: six v_mfma_f32_16x16x32_bf16
// (16 cycles each) instead of eight v_mfma_f32_16x16x4_f32 (32 cycles each).
// ---------------------------------------------------------------------------
struct S8 {            // one lane's 8 k-values of an MFMA operand, three planes
  u4 h, m, l;
};

#ifndef NERFHIP_EXP_X2PROXY   // diagnostic timing builds only, see mfma16x3
#define NERFHIP_X2P(bit) 0
#else
#define NERFHIP_X2P(bit) ((NERFHIP_EXP_X2PROXY) & (bit))
#endif
__device__ __forceinline__ void split3(float x, uint32_t& h, uint32_t& m, uint32_t& l) {
  const uint32_t u = __float_as_uint(x);
  const float r1 = x - __uint_as_float(u & 0xffff0000u);
  const uint32_t u1 = __float_as_uint(r1);
#if NERFHIP_X2P(8)
  h = u;
  m = u1;
  l = u1;
#else
  const float r2 = r1 - __uint_as_float(u1 & 0xffff0000u);
  h = u;
  m = u1;
  l = __float_as_uint(r2);   // ≤ 8 significant bits: its top half is exact
#endif
}
// low half ← bf16 of a, high half ← bf16 of b (the top 16 bits of each): one
// v_perm_b32 (bytes 2,3 of a then bytes 2,3 of b; {S0,S1} = {b,a}) instead of
// the shift / and / or the compiler otherwise emits.  Bitwise-equal results;
// medium 40-fit row kernel −4 %, sweep unchanged (ab_perm_sincos_bits.log)
__device__ __forceinline__ uint32_t pk_top(uint32_t a, uint32_t b) {
  return __builtin_amdgcn_perm(b, a, 0x07060302u);
}
__device__ __forceinline__ S8 split8(const float (&x)[8]) {
  uint32_t h[8], m[8], l[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) split3(x[s], h[s], m[s], l[s]);
  S8 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o.h[i] = pk_top(h[2 * i], h[2 * i + 1]);
    o.m[i] = pk_top(m[2 * i], m[2 * i + 1]);
    o.l[i] = pk_top(l[2 * i], l[2 * i + 1]);
  }
  return o;
}
// the lane's two accumulator tiles t0, t1 (4 features each) as one k-slice
__device__ __forceinline__ S8 split_pair(const float (&t0)[4], const float (&t1)[4]) {
  const float x[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  return split8(x);
}

__device__ __forceinline__ f4 mfma16b(u4 a, u4 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
__device__ __forceinline__ f16v mfma32b(u4 a, u4 b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
// NERFHIP_EXP_X2PROXY (diagnostic timing build, WRONG numerics): the cost of
// a two-plane operand split with three products (hi·hi', hi·lo', lo·hi', as
// an fp16 hi/lo split with power-of-two scaling would need): the m plane
// stands in for lo, the l plane is neither split, staged, read nor multiplied.
// Bit flags: 1 three products, 2 row-kernel weight DMA of two planes, 4 its
// A-fragment LDS reads of two planes, 8 no l in split3, 16 the parameter
// kernel's staging and reads of two planes (31 = all, 30 = data movement only).
#if NERFHIP_X2P(1)
__device__ __forceinline__ void mfma16x3(const S8& a, const S8& b, f4& hi, f4& lo) {
  lo = mfma16b(a.h, b.m, lo);
  lo = mfma16b(a.m, b.h, lo);
  hi = mfma16b(a.h, b.h, hi);
}
__device__ __forceinline__ void mfma32x3(const S8& a, const S8& b, f16v& hi, f16v& lo) {
  lo = mfma32b(a.h, b.m, lo);
  lo = mfma32b(a.m, b.h, lo);
  hi = mfma32b(a.h, b.h, hi);
}
#else
__device__ __forceinline__ void mfma16x3(const S8& a, const S8& b, f4& hi, f4& lo) {
  lo = mfma16b(a.h, b.l, lo);
  lo = mfma16b(a.l, b.h, lo);
  lo = mfma16b(a.m, b.m, lo);
  lo = mfma16b(a.h, b.m, lo);
  lo = mfma16b(a.m, b.h, lo);
  hi = mfma16b(a.h, b.h, hi);
}
__device__ __forceinline__ void mfma32x3(const S8& a, const S8& b, f16v& hi, f16v& lo) {
  lo = mfma32b(a.h, b.l, lo);
  lo = mfma32b(a.l, b.h, lo);
  lo = mfma32b(a.m, b.m, lo);
  lo = mfma32b(a.h, b.m, lo);
  lo = mfma32b(a.m, b.h, lo);
  hi = mfma32b(a.h, b.h, hi);
}
#endif

// weight element M_i[j][k] = p into both split copies (prologue / split-K)
__device__ __forceinline__ void put_w(uint16_t* XS, int ks, int W, int D, int L, int i, int j,
                                      int k, float p) {
  const int R = i <= L ? W : D;
  uint32_t h, m, l;
  split3(p, h, m, l);
  const uint32_t part[3] = {h >> 16, m >> 16, l >> 16};
  const int64_t f = xs_mat(W, D, L, false, i), b = xs_mat(W, D, L, true, i);
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
    XS[f + xoff_any(ks, R, W, j, k, pl)] = (uint16_t)part[pl];
    XS[b + xoff_any(ks, W, R, k, j, pl)] = (uint16_t)part[pl];
  }
}

// hidden_layers of a group's fit: a one-fit group's is L_max (nerfhip.h), a
// kernel argument — no dependent load of fit_layers in front of the tile
// decode of a lone fit's kernels (config 2's launches are latency-bound)
__device__ __forceinline__ int fit_layers_of(const KArgs& a, int fit) {
  return a.n_fits == 1 ? a.L_max : a.fit_layers[fit];
}
// the weight-plane layout the group's row kernel reads
__host__ __device__ inline int wlayout(const KArgs& a) {
  return a.rows_ks ? kLayKs : a.rows32 ? kLay32 : kLayX;
}

// Buffer-resource helpers (k_adam_split's masked stores, the parameter
// kernels' Adam epilogues).
constexpr uint32_t kOob = 0x80000000u;   // a byte offset past every resource below
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_over(const void* p, int64_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)nbytes, 0x00020000);
}
// an offset computed by every lane, then replaced by kOob where `keep` is
// false: the volatile empty asm pins the computation ahead of the select (left
// free, the compiler sank it into a branch per store, EXEC-masked)
__device__ __forceinline__ uint32_t lane_off(bool keep, uint32_t off) {
  asm volatile("" : "+v"(off));
  return keep ? off : kOob;
}
// buffer resources held in their SGPRs up to this point (after a vmcnt(0)
// drain: no store can still be waiting to read them)
__device__ __forceinline__ void keep_live(__amdgpu_buffer_rsrc_t a, __amdgpu_buffer_rsrc_t b,
                                          __amdgpu_buffer_rsrc_t c) {
  asm volatile("" ::"s"(a), "s"(b), "s"(c));
}
__device__ __forceinline__ void bstore_f32(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)off, 0, 0);
}
__device__ __forceinline__ void bstore_u16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint16_t v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, r, (int)off, 0, 0);
}
__device__ __forceinline__ float bload_f32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}

// A split-K partial-slab element.  For the fused reduction (split_finish)
// the store is write-through (sc1: agent-scope relaxed), so the slices need no
// L2 write-back (release fence) before their arrival — the fence costs each
// arriving workgroup a write-back of its XCD's whole dirty L2
// (cdna_hip_programming.md, in-launch split-K); k_adam_split's slabs cross a
// kernel boundary and stay plain.
// (WT: compile-time, the fused instantiation only — a run-time select put
// exec-masked branches around the slab stores of every split-K launch)
template <bool WT>
__device__ __forceinline__ void slab_store(float* p, float v) {
  if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// torch.optim.Adam, single-tensor path (the reference runs on CPU, where the
// foreach/fused paths are unavailable): TORCH/optim/adam.py:457,476,531-547.
__device__ __forceinline__ void adam_update(float& p, float& m, float& v, float g,
                                            float step_size, float bc2_sqrt) {
  // The roundings are spelled out (explicit fma, no contraction): the same
  // update is inlined into several kernels (the parameter tiles' epilogues,
  // k_adam_split, the fused split-K reducer), and left to the contraction
  // pass each copy could fuse differently — 1-ulp differences between paths
  // that must agree bitwise (test_split_fused_equals_separate_pass).
#pragma clang fp contract(off)
  m = fmaf(0.1f, g - m, m);                      // exp_avg.lerp_(grad, 1-β1)
  v = fmaf(0.001f * g, g, v * 0.999f);           // exp_avg_sq.mul_(β2).addcmul_(grad, grad, 1-β2)
  const float denom = sqrtf(v) / bc2_sqrt + 1e-8f;  // (√v / √bc2).add_(eps)
  p = fmaf(-step_size, m / denom, p);            // addcdiv_(m, denom, -lr/bc1)
}

// ---------------------------------------------------------------------------
// Row-parallel step: forward + loss + backward dX chain for 64 rows of a fit.
// mode 0 = train step; mode 1 = forward only (writes ŷ to y_out).
//
// Each GEMM phase streams its weight matrix through LDS in 16-row chunks,
// double-buffered: the whole workgroup loads chunk j+1 (coalesced 16-B global
// loads into registers) while its four waves run chunk j's MFMAs from LDS, so
// the L2 latency of the weights hides behind ≈2K cycles of MFMA per chunk and
// the four waves (64 rows) share one copy of every weight.  Per-lane epilogue
// operands (targets, cos) are issued at the top of the chunk for the same
// reason.  Rows of the LDS chunk are padded by 32 B so the lanes of one
// ds_read_b128 (16 rows × 4 k) hit distinct banks.
// ---------------------------------------------------------------------------

// LDS chunk buffers per GEMM phase: a 3-deep ring where it fits (so the next
// chunk is already visible while the current one computes), else 2.
template <int K> constexpr int phase_nbuf() { return K >= 512 ? 2 : 3; }
template <int K> constexpr int phase_lds_floats() { return phase_nbuf<K>() * 16 * (K + 8); }

// Stream rows [0, 16·JT) of `src` (row-major, row length K) through LDS and
// compute, for every 16-row chunk J, acc = src[16J..16J+15][:] · B where the
// B operand is the register tile b[K/16][4] (lane (c, g) holds B[16kt+4g+s][c]).
//
// Per chunk J, in issue order:
//   flush(J−2)        global stores of tile J−2 (J−1 with a 2-buffer ring): an
//                     old store, because vmcnt counts loads and stores together
//                     in issue order, so stores issued after the staging loads
//                     would be waited for at this chunk's barrier
//   staging loads of chunk J+NBUF−1, pre(J) per-lane loads
//   K/16 k-steps of 4 MFMAs; A fragments read two steps ahead — across the
//   chunk boundary when the ring has 3 buffers — and elem(J−1, q, acc, pre)
//   for q = 0..3 spread over four k-steps: the epilogue VALU (sincos, loss,
//   dZ) fills MFMA gaps instead of stalling the pipe between chunks (3-buffer
//   ring only; with 2 buffers — one wave per SIMD at K = 512 — elem(J) runs
//   right after chunk J's MFMAs, which measured faster there)
//   LDS ← staging registers, one barrier.
// Row stride K+8 floats: every start bank of a ds_read_b128 lane group is
// distinct (K+4 collides lanes with equal c+g).
template <int K, int JT, int NTH, class Pre, class Elem, class Flush>
__device__ __forceinline__ void gemm_phase(const float* __restrict__ src, float* lds,
                                           const float (&b)[K / 16][4], int tid, int c, int g,
                                           Pre&& pre, Elem&& elem, Flush&& flush) {
  constexpr int NB = phase_nbuf<K>();
  constexpr int LD = K + 8, CH = 16 * LD, C4 = K / 4, KT = K / 16;
  constexpr int NF4 = 16 * C4, NPT = (NF4 + NTH - 1) / NTH;   // f4 slots per chunk
  constexpr int QSTEP = (KT - 1) / 4 > 0 ? (KT - 1) / 4 : 1;
  f4 st[NPT];
  auto gload = [&](int chunk) {
    const float* cs = src + chunk * 16 * K;
#pragma unroll
    for (int m = 0; m < NPT; ++m) {
      const int i = tid + NTH * m;
      if (NF4 % NTH == 0 || i < NF4) st[m] = ld4(cs + (i / C4) * K + (i % C4) * 4);
    }
  };
  auto lput = [&](int chunk) {
    float* buf = lds + (chunk % NB) * CH;
#pragma unroll
    for (int m = 0; m < NPT; ++m) {
      const int i = tid + NTH * m;
      if (NF4 % NTH == 0 || i < NF4) st4(buf + (i / C4) * LD + (i % C4) * 4, st[m]);
    }
  };
#pragma unroll
  for (int j = 0; j < NB - 1 && j < JT; ++j) {
    gload(j);
    lput(j);
  }
  __syncthreads();
  const float* lane_off = lds + c * LD + 4 * g;
  f4 a_cur = ld4(lane_off), a_nxt = ld4(lane_off + 16);
  f4 acc_prev = {0.f, 0.f, 0.f, 0.f}, pv_prev = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int J = 0; J < JT; ++J) {
    // pending epilogue results are single-buffered: flush(J') must run before
    // elem(J'+1), i.e. two chunks late when elem lags a chunk (NB == 3), one
    // chunk late otherwise
    if (NB == 3 && J >= 2) flush(J - 2);
    if (NB == 2 && J >= 1) flush(J - 1);
    if (J + NB - 1 < JT) gload(J + NB - 1);
    const f4 pv = pre(J);
    const float* buf = lane_off + (J % NB) * CH;
    const float* nbuf = lane_off + ((J + 1) % NB) * CH;
    f4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      f4 a_n2;
      if (kt + 2 < KT) a_n2 = ld4(buf + 16 * (kt + 2));
      else if (NB == 3 && J + 1 < JT) a_n2 = ld4(nbuf + 16 * (kt + 2 - KT));
      else a_n2 = a_nxt;
      f4& ac = acc[kt & 1];
      ac = mfma16(a_cur[0], b[kt][0], ac);
      ac = mfma16(a_cur[1], b[kt][1], ac);
      ac = mfma16(a_cur[2], b[kt][2], ac);
      ac = mfma16(a_cur[3], b[kt][3], ac);
      if (NB == 3 && J > 0) {   // (measured: a net loss at one wave/SIMD, NB == 2)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kq = 1 + q * QSTEP < KT ? 1 + q * QSTEP : KT - 1;
          if (kt == kq) elem(J - 1, q, acc_prev[q], pv_prev[q]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      a_cur = a_nxt;
      a_nxt = a_n2;
    }
    acc_prev = acc[0] + acc[1];
    pv_prev = pv;
    if (NB == 2) {
#pragma unroll
      for (int q = 0; q < 4; ++q) elem(J, q, acc_prev[q], pv_prev[q]);
    }
    if (J + NB - 1 < JT) lput(J + NB - 1);
    __syncthreads();
    if (NB == 2 && J + 1 < JT) {  // 2-buffer ring: the next chunk is readable only now
      a_cur = ld4(nbuf);
      a_nxt = ld4(nbuf + 16);
    }
  }
  if (NB == 3) {
    if (JT >= 2) flush(JT - 2);
#pragma unroll
    for (int q = 0; q < 4; ++q) elem(JT - 1, q, acc_prev[q], pv_prev[q]);
  }
  flush(JT - 1);
  __syncthreads();   // the epilogue read LDS (bias): the next phase may overwrite it
}

// bf16x3 form of gemm_phase (same contract, same pre/elem/flush schedule):
// the weight rows arrive as split planes in the xoff layout, one sub-chunk
// u = J·NH + hh per (output tile J, k-slice hh of NH = K/KC), and each 32-deep
// k-step is six bf16 MFMAs against the B operand b[K/32] (split k-slices).
//
// Staging is LDS-DMA (global_load_lds_dwordx4) into a 3-deep ring of its own
// __shared__ object: sub-chunk u+2 is issued at the top of sub-chunk u and
// only retired (counted vmcnt, then the barrier) at the END of u+1, so every
// fill has two sub-chunks of MFMA time to land and costs no VGPRs.  The DMA
// image is lane-linear, so the bank swizzle lives on the source address:
// 16-B slot s of row r sits at physical slot s ^ (r mod min(16, slots/row)),
// which makes every 16-lane ds_read_b128 group of the A-fragment read hit the
// 16 slots of a bank row once.  The A fragments are read by inline-asm
// ds_read_b128 (hipcc would otherwise put a vmcnt(0) drain of the in-flight
// DMA in front of them) and retired by an lgkmcnt wait that also redefines
// the fragment registers, so no use can be scheduled before the data lands.
template <int K> constexpr int x3_ring_halfs() { return 3 * 3 * 16 * kc_of(K); }

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int N> constexpr std::integral_constant<int, N> ic{};

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// ds_read_b128 at base + OFF bytes; OFF must fit the 16-bit offset field
template <int OFF>
__device__ __forceinline__ u4 ds_read16(uint32_t base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  u4 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base), "n"(OFF));
  return r;
}

template <int K, int JT, int NTH, int NST, int NLD, bool PIN, class Pre, class Elem, class Flush>
__device__ __forceinline__ void gemm_phase_x3(const uint16_t* __restrict__ src, uint16_t* ring,
                                              const S8 (&b)[K / 32], int tid, int c, int g,
                                              Pre&& pre, Elem&& elem, Flush&& flush) {
  constexpr int KC = kc_of(K), NH = K / KC, U = JT * NH, KT = KC / 32;
  constexpr int SR = KC / 8;                                // 16-B slots per row
  constexpr int SWM = (SR < 16 ? SR : 16) - 1;              // swizzle mask
  constexpr int CH = 3 * 16 * KC;                           // bf16 per ring buffer
  constexpr int PLB = 32 * KC;                              // bytes per plane
#if NERFHIP_X2P(2)
  constexpr int SL = 2 * 16 * SR, NPT = (SL + NTH - 1) / NTH;   // planes 0, 1 only
#else
  constexpr int SL = 3 * 16 * SR, NPT = (SL + NTH - 1) / NTH;   // slots per sub-chunk
#endif
  constexpr int NDMA = SL / NTH;                                // DMAs every wave issues
  constexpr int QSTEP = (KT - 1) / 4 > 0 ? (KT - 1) / 4 : 1;
  typedef __attribute__((address_space(3))) void lds_void;
  // the wave index as an SGPR: every DMA's LDS destination (M0) is then SALU
  // arithmetic instead of a per-instruction v_readfirstlane of a VGPR address
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // This lane's source offset (bf16) inside a sub-chunk for DMA round m.  With
  // NTH = 256 the rounds step s = NTH/SR source rows; the swizzled offset of
  // round m is that of round m % P plus (m / P)·P·s·KC, P = max(1, 16/s)
  // (s = 8: rows r0 and r0 + 8 alternate, each pair of rounds is one plane),
  // so only P per-lane offsets stay live and the rest is a compile-time
  // addend on the SGPR sub-chunk offset.
  constexpr int S_ROWS = NTH / SR, P = S_ROWS >= 16 ? 1 : 16 / S_ROWS;
  static_assert(NTH % SR == 0 && 16 % (S_ROWS < 16 ? S_ROWS : 16) == 0, "DMA round layout");
  int soff[P];
#pragma unroll
  for (int m = 0; m < P; ++m) {
    const int i = tid + NTH * m;
    const int row = (i / SR) & 15, pl = i / (16 * SR), ps = i % SR;
    soff[m] = (pl * 16 + row) * KC + 8 * (ps ^ (row & SWM));
  }
  // buffer-resource form: SGPR base + per-lane 32-bit offset + SGPR sub-chunk offset
  // (a flat-pointer global_load_lds makes hipcc materialise a 64-bit address per
  // sub-chunk and round)
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7fffffff, 0x00020000);
  auto dma_round = [&](int u, int m) {
    uint16_t* buf = ring + (u % 3) * CH;
    if (SL % NTH == 0 || NTH * m + 64 * wave < SL)   // wave-uniform
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc, (lds_void*)(buf + 8 * (NTH * m + 64 * wave)), 16, 2 * soff[m % P],
          u * 96 * KC + 2 * (m / P) * P * S_ROWS * KC, 0, 0);
  };
  auto dma = [&](int u) {
#pragma unroll
    for (int m = 0; m < NPT; ++m) dma_round(u, m);
  };
  // lane (row c, group g): k-step kt reads logical slot 4kt + g of row c in
  // plane p of buffer u%3 = abase[kt] + (u%3)·2CH + p·PLB bytes
  uint32_t abase[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
    abase[kt] = lds_addr(ring) + 2 * (c * KC + 8 * ((4 * kt + g) ^ (c & SWM)));
  auto aread = [&](auto uc, auto ktc) {
    constexpr int OFF = (decltype(uc)::value % 3) * 2 * CH;
    constexpr int kt = decltype(ktc)::value;
    S8 r;
    r.h = ds_read16<OFF>(abase[kt]);
    r.m = ds_read16<OFF + PLB>(abase[kt]);
#if NERFHIP_X2P(4)
    r.l = r.m;
#else
    if constexpr (OFF + 2 * PLB < 65536) r.l = ds_read16<OFF + 2 * PLB>(abase[kt]);
    else r.l = ds_read16<OFF + PLB>(abase[kt] + PLB);
#endif
    return r;
  };
  auto lgkm_wait = [](S8& r) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r.h), "+v"(r.m), "+v"(r.l));
  };
  // Retire sub-chunk u+1's DMA, which is older than every vm op issued in
  // iteration u: [flush stores][pre loads][DMA(u+2)].  Those may stay in flight,
  // so the wait leaves exactly their count outstanding (NST / NLD are the exact
  // store / load instructions of flush / pre, or fewer: fewer only over-waits).
  // Stores thereby get two iterations to be acknowledged instead of one.
  auto vm_wait_barrier = [&](auto nc) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(nc)::value));
    asm volatile("s_waitcnt lgkmcnt(0)");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  dma(0);
  if (U > 1) dma(1);
  vm_wait_barrier(std::integral_constant<int, (U > 1 ? NDMA : 0)>{});
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  S8 a_cur = aread(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
  lgkm_wait(a_cur);
  f4 acc_prev = zero4, pv_prev = zero4, pv = zero4, hi = zero4, lo = zero4;
  static_for<0, U>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    constexpr int J = u / NH, hh = u % NH;
    if constexpr (hh == 0) {
#ifndef NERFHIP_EXP_NOFLUSH
      if constexpr (J >= 2) flush(J - 2);
#endif
      hi = zero4;
      lo = zero4;
      pv = pre(J);
    }
    __builtin_amdgcn_sched_barrier(0);   // flush / pre before the DMA: vmcnt counts in order
    const unsigned long long t_d0 = MEMTIME();
    // (one DMA round per k-step instead measured slower: the issue stall
    // moved into the k-steps and the end-of-sub-chunk wait grew)
#ifndef NERFHIP_EXP_NOSTAGE
    if constexpr (u + 2 < U) dma(u + 2);
#endif
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t_d1 = MEMTIME();
    static_for<0, KT>([&](auto ktc) {
      constexpr int kt = decltype(ktc)::value;
      S8 a_nxt = a_cur;
      if constexpr (kt + 1 < KT) a_nxt = aread(uc, std::integral_constant<int, kt + 1>{});
      mfma16x3(a_cur, b[hh * KT + kt], hi, lo);
      if constexpr (hh == 0 && J > 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kq = 1 + q * QSTEP < KT ? 1 + q * QSTEP : KT - 1;
          if (kt == kq) elem(J - 1, q, acc_prev[q], pv_prev[q]);
        }
      }
      // PIN (one wave per SIMD, W = 512): keep this k-step's MFMAs (and the
      // epilogue VALU beside them) ahead of the wait for the next fragments.
      // Left free, the scheduler sinks most MFMAs below the wait and the LDS
      // read latency is exposed every k-step; at two waves per SIMD the other
      // wave covers it and the free schedule measured 2 % faster (W = 256),
      // at one wave per SIMD pinning measured 2.5 % faster (W = 512,
      // profiles/r02/ab_pin_lgkm.log).
      if constexpr (PIN) __builtin_amdgcn_sched_barrier(0);
      if constexpr (kt + 1 < KT) lgkm_wait(a_nxt);
      __builtin_amdgcn_sched_barrier(0);
      a_cur = a_nxt;
    });
    if constexpr (hh == NH - 1) {
      acc_prev = hi + lo;
      pv_prev = pv;
    }
    const unsigned long long t_w0 = MEMTIME();
#ifndef NERFHIP_EXP_NOBARRIER
    constexpr int n_out = (u + 2 < U ? NDMA : 0) + (hh == 0 ? NLD : 0) +
                          (hh == 0 && J >= 2 ? NST : 0);
    vm_wait_barrier(std::integral_constant<int, n_out>{});   // sub-chunk u+1 landed everywhere
#endif
#if defined(NERFHIP_STAMPS) && !defined(NERFHIP_STAMPS_NOADD)
    asm volatile("s_waitcnt vmcnt(0)");
    const unsigned long long t_w1 = MEMTIME();
    STAMP_ADD(8, t_d1 - t_d0);     // DMA issue
    STAMP_ADD(9, t_w0 - t_d1);     // k-steps (MFMA + epilogue VALU + LDS reads)
    STAMP_ADD(10, t_w1 - t_w0);    // vm wait + barrier (+ drain, diagnostic only)
    STAMP_ADD(11, 1);              // sub-chunks
#else
    (void)t_d0; (void)t_d1; (void)t_w0;
#endif
    if constexpr (u + 1 < U) {           // its first fragment, only now readable
      a_cur = aread(std::integral_constant<int, u + 1>{}, std::integral_constant<int, 0>{});
      lgkm_wait(a_cur);
    }
  });
  if (JT >= 2) flush(JT - 2);
#pragma unroll
  for (int q = 0; q < 4; ++q) elem(JT - 1, q, acc_prev[q], pv_prev[q]);
  flush(JT - 1);
  __syncthreads();   // the epilogue read LDS (bias): the next phase may overwrite it
}

// one GEMM phase in the kernel's precision (B: float[K/16][4] or S8[K/32])
template <bool X3, int K, int JT, int NTH, int NST, int NLD, bool PIN, class B, class Pre,
          class Elem, class Flush>
__device__ __forceinline__ void gemm_any(const void* src, float* lds, uint16_t* ring, const B& b,
                                         int tid, int c, int g, Pre&& pre, Elem&& elem,
                                         Flush&& flush) {
  if constexpr (X3)
    gemm_phase_x3<K, JT, NTH, NST, NLD, PIN>(static_cast<const uint16_t*>(src), ring, b, tid, c, g,
                                             pre, elem, flush);
  else
    gemm_phase<K, JT, NTH>(static_cast<const float*>(src), lds, b, tid, c, g, pre, elem, flush);
}

template <bool C, class A, class B>
__device__ __forceinline__ auto& pick_ref(A& a, B& b) {
  if constexpr (C) return a;
  else return b;
}

// copy n floats (n % 4 == 0, n ≤ 1024) global → LDS, cooperatively
__device__ __forceinline__ void stage_vec(float* dst, const float* src, int n, int tid) {
  if (4 * tid < n) st4(dst + 4 * tid, ld4(src + 4 * tid));
}

// Output width split: a W-wide layer output is produced in NSPLIT passes of
// W/NSPLIT features; all passes but the last park their fragments in a
// per-wave LDS stash.  Live output registers drop from W/4 to W/(4·NSPLIT),
// which is what lets W = 512 fit the 256 VALU-addressable VGPRs.
// Rows per workgroup: 16 per wave.  (8 waves = 128 rows per workgroup at W = 256
// halves the weight staging per row but measured no faster: 1.98 vs 2.03 ms
// bf16x3, 2.88 vs 2.70 ms fp32 for the 160-fit medium group.)
#ifdef NERFHIP_EXP_DWORD_STORES
constexpr bool kQuadStores = false;   // diagnostic: the pre-transpose dword stores
#else
constexpr bool kQuadStores = true;
#endif

template <int W> struct RowsCfg {
  static constexpr int NSPLIT = W >= 512 ? 2 : 1;
  // (W = 256 at one wave per SIMD — no VGPR spills, 512 registers — measured
  // 25 % slower: the second wave's MFMAs are what fill the epilogue gaps)
  static constexpr int WAVES_PER_SIMD = W >= 512 ? 1 : 2;
// experiment knob: waves (16 rows each) per W = 256 workgroup.  8 (with
// NERFHIP_ROWPAD=128): isolated 40-fit launch 8 % slower, 200-epoch sweep
// +1.2 %, results equal only to rounding (profiles/r03/rows_w256_8waves.log)
#ifndef NERFHIP_ROWS_NWAVES_256
#define NERFHIP_ROWS_NWAVES_256 4
#endif
  static constexpr int NWAVES = W == 256 ? NERFHIP_ROWS_NWAVES_256 : 4;
  static constexpr int THREADS = 64 * NWAVES, ROWS = 16 * NWAVES;
};

template <int W, int D, bool X3, bool TRAIN>
__global__ void __launch_bounds__(RowsCfg<W>::THREADS, RowsCfg<W>::WAVES_PER_SIMD)
    k_step_rows(KArgs a) {
  FLIGHT_ENTER();
  constexpr int NWV = RowsCfg<W>::NWAVES, NTH = RowsCfg<W>::THREADS;
  constexpr int JW = W / 16, JD = D / 16, KMAX = (W > D ? W : D);
  constexpr int NS = RowsCfg<W>::NSPLIT, JP = JW / NS;     // J tiles per pass
  constexpr bool PIN = RowsCfg<W>::WAVES_PER_SIMD == 1;     // see gemm_phase_x3
  constexpr int WBUF_F = phase_lds_floats<W>() > phase_lds_floats<D>()
                             ? phase_lds_floats<W>() : phase_lds_floats<D>();
  constexpr int WBUF = X3 ? 0 : WBUF_F;   // fp32 weight ring, in floats (bf16x3: xring)
  constexpr int STASH = (NS - 1) * JP * 256;                // per wave
  __shared__ __attribute__((aligned(16))) float lds[WBUF + 2 * KMAX + NWV * STASH];
  __shared__ __attribute__((aligned(16))) uint16_t xring[X3 ? x3_ring_halfs<KMAX>() : 8];
  float* bias = lds + WBUF;   // a phase's bias, or w0 ‖ b0 in the layer-0 backward
  int fit, tile;
  if (!map_block(blockIdx.x, a.n_fits, a.n_pad / RowsCfg<W>::ROWS, fit, tile)) return;
  STAMP_RT(12);
  STAMP(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  float* stash = lds + WBUF + 2 * KMAX + wave * STASH + lane * 4;
  const int L = fit_layers_of(a, fit);
  FLIGHT_DEPTH(L, fit);
  const float om = a.fit_omega[fit];
  const int n_pad = a.n_pad;
  const int rblk = tile * NWV + wave;         // 16-row block
  const int r = rblk * 16 + c;                // this lane's row (B/D column)
  const bool valid = r < a.N;
  constexpr bool train = TRAIN;   // a.mode == 0

  const float* P = a.params + fit * a.p_stride;
  const float* PT = a.params_t + fit * a.pt_stride;
  float* S = a.scratch + fit * a.s_stride;
  const int64_t WN = (int64_t)W * n_pad;
  float* SH = S;
  float* SZ = S + (int64_t)(a.L_max + 1) * WN;
  float* SG = S + 2 * (int64_t)(a.L_max + 1) * WN;
  float* SC = SG + (int64_t)D * n_pad;
  // per-lane bases into the row-block-major [n_pad/16][F][16] scratch: the
  // element (feature 16J+4g+q, row r) sits at +(16J+q)·16 (compile-time)
  float* SHb = SH + (int64_t)rblk * W * 16 + g * 64 + c;
  float* SZb = SZ + (int64_t)rblk * W * 16 + g * 64 + c;
  float* SGb = SG + (int64_t)rblk * D * 16 + g * 64 + c;
  // after quad_transpose the lane writes feature 4g+(c&3) of rows 4(c>>2)..+3
  const int tq = g * 64 + (c & 3) * 16 + (c >> 2) * 4;
  float* SHt = SH + (int64_t)rblk * W * 16 + tq;
  float* SZt = SZ + (int64_t)rblk * W * 16 + tq;
  float* SGt = SG + (int64_t)rblk * D * 16 + tq;
  // one transposed 16-B store per accumulator tile (kQuadStores), or four dword stores
  auto tile_store = [&](float* base_t, float* base_d, int J, const float (&v)[4]) {
    if constexpr (kQuadStores) {
      const f4 t = {v[0], v[1], v[2], v[3]};
      sst4(base_t + J * 256, quad_transpose(t, c));
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) sst(base_d + (16 * J + q) * 16, v[q]);
    }
  };
  constexpr int kTS = kQuadStores ? 1 : 4;   // vm stores per tile_store
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  auto no_pre = [&](int) { return zero4; };

  float hp[JW][4];      // fp32: the layer input (B operand), all W features
  S8 hs[JW / 2];        // bf16x3: the same, as split k-slices
  float ho[JP][4];      // one pass of the layer output
  auto& hb = pick_ref<X3>(hs, hp);    // the B operand of this precision
  const uint16_t* XS = X3 ? a.wsplit + fit * a.ws_stride : nullptr;
  // weight operand of layer i (1..L hidden, L+1 final), forward or transposed
  auto wsrc = [&](bool bwd, int i) -> const void* {
    if (X3) return XS + xs_mat(W, D, L, bwd, i);
    if (bwd) return PT + (int64_t)(i - 1) * W * W;
    return i <= L ? P + off_hidden_w(W, i) : P + off_final_w(W, L);
  };

  // Run a W-wide output layer as NS passes over src rows; out(Jg, q, acc, pv)
  // writes element q of feature tile Jg into ho[Jg % JP], flush(Jg) stores
  // the tile; afterwards hb ← output.
  // nst / nld: the exact vm store / load counts of flush / pre (bf16x3 waits)
  auto wide_layer = [&](auto nst, auto nld, const void* src, auto& bop, auto&& pre, auto&& out,
                        auto&& flush) {
    constexpr int K = (sizeof(bop) / sizeof(bop[0])) * (X3 ? 32 : 16);
#pragma unroll
    for (int p = 0; p < NS; ++p) {
      gemm_any<X3, K, JP, NTH, decltype(nst)::value, decltype(nld)::value, PIN>(
          static_cast<const char*>(src) + (int64_t)p * JP * K * (X3 ? 96 : 64), lds, xring, bop, tid,
          c, g, [&](int J) { return pre(p * JP + J); },
          [&](int J, int q, float acc, float pv) { out(p * JP + J, q, acc, pv); },
          [&](int J) { flush(p * JP + J); });
      if (p + 1 < NS) {
#pragma unroll
        for (int J = 0; J < JP; ++J) {
          const f4 v = {ho[J][0], ho[J][1], ho[J][2], ho[J][3]};
          st4(stash + (p * JP + J) * 256, v);
        }
      }
    }
    // all passes done (gemm_phase ended with a barrier): assemble the operand
    auto tile = [&](int Jg, float (&t)[4]) {
      if (Jg < (NS - 1) * JP) {
        const f4 v = ld4(stash + Jg * 256);
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] = v[q];
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) t[q] = ho[Jg - (NS - 1) * JP][q];
      }
    };
    if constexpr (X3) {
#pragma unroll
      for (int J2 = 0; J2 < JW / 2; ++J2) {
        float t0[4], t1[4];
        tile(2 * J2, t0);
        tile(2 * J2 + 1, t1);
        hs[J2] = split_pair(t0, t1);
      }
    } else {
#pragma unroll
      for (int Jg = 0; Jg < JW; ++Jg) tile(Jg, hp[Jg]);
    }
  };

  // ---- layer 0: SineLayer(1, W, is_first) — K = 1, an outer product (VALU).
  // cos(ωz0) is not stored: it is a function of (x, w0, b0) and the layer-0
  // backward recomputes it bit-identically (half this layer's HBM writes).
  // (Regenerating H0 inside k_step_params as well was measured slower: the
  // sincos lands on its staging path.)
  stage_vec(lds, P, 2 * W, tid);              // w0 ‖ b0
  __syncthreads();
  const float x = a.pos[r];
#pragma unroll
  for (int J = 0; J < JW; ++J) {
    const f4 w = ld4(lds + 16 * J + 4 * g), b = ld4(lds + W + 16 * J + 4 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float z = __fadd_rn(__fmul_rn(x, w[q]), b[q]);
      float s, co;
      sincos_fast(__fmul_rn(om, z), &s, &co);
      hp[J][q] = s;
    }
    if (train) {
      tile_store(SHt, SHb, J, hp[J]);
    }
  }
  if constexpr (X3) {
#pragma unroll
    for (int J2 = 0; J2 < JW / 2; ++J2) hs[J2] = split_pair(hp[2 * J2], hp[2 * J2 + 1]);
  }
  __syncthreads();

  STAMP(1);
  // ---- hidden SineLayers 1..L: Zᵀ = Wᵢ·Hᵀ (+b), H = sin(ω Z)
  for (int i = 1; i <= L; ++i) {
    const float* Wi = P + off_hidden_w(W, i);
    stage_vec(bias, Wi + W * W, W, tid);
    float* SHi = SHb + (int64_t)i * WN;
    float* SHti = SHt + (int64_t)i * WN;
    float* SCi = SC + (int64_t)i * WN + (int64_t)rblk * JW * 256 + lane * 4;
    f4 cs_pend;
    wide_layer(
        ic<TRAIN ? 1 + kTS : 0>, ic<0>, wsrc(false, i), hb, no_pre,
        [&](int J, int q, float acc, float) {
          const float z = __fadd_rn(acc, bias[16 * J + 4 * g + q]);
          float s, co;
          sincos_fast(__fmul_rn(om, z), &s, &co);
          ho[J % JP][q] = s;
          cs_pend[q] = co;
        },
        [&](int J) {
          if (train) {
            cst4(SCi + J * 256, cs_pend);
            tile_store(SHti, SHi, J, ho[J % JP]);
          }
        });
  }

  STAMP(2);
  // ---- final nn.Linear(W, D): ŷᵀ = W_f·H_Lᵀ + b_f ; MSE ; dL/dŷ
  const float* Wf = P + off_final_w(W, L);
  stage_vec(bias, Wf + W * D, D, tid);
  const float* T = a.tnorm + fit * a.t_stride + (int64_t)r * D + 4 * g;
  // wave-uniform scalar test (no EXEC write right after the tile stores: a
  // store still waiting for the memory pipeline can read EXEC late on gfx950,
  // DESIGN.md §11)
  const bool has_y = a.y_out != nullptr;
  float* yo = has_y ? a.y_out + fit * a.y_stride + (int64_t)r * D + 4 * g : nullptr;
  float y[JD][4];
  S8 ys[JD / 2];
  float sq = 0.f;
  f4 y_pend;
  gemm_any<X3, W, JD, NTH, TRAIN ? kTS : 0, TRAIN ? 1 : 0, PIN>(
      wsrc(false, L + 1), lds, xring, hb, tid, c, g,
      [&](int J) { return train ? ld4(T + 16 * J) : zero4; },
      [&](int J, int q, float acc, float t) {
        y_pend[q] = __fadd_rn(acc, bias[16 * J + 4 * g + q]);
        if (train) {
          const float diff = y_pend[q] - t;
          sq = valid ? fmaf(diff, diff, sq) : sq;
          y[J][q] = valid ? a.grad_scale * diff : 0.f;
        }
      },
      [&](int J) {
        if (has_y) st4(yo + 16 * J, y_pend);       // lane holds ŷ[r][16J+4g+q]
        if (train) tile_store(SGt, SGb, J, y[J]);
      });
  STAMP(3);
  if (!train) return;
  sq = wave_sum(sq);
  if (lane == 0)
    a.loss_partial[fit * a.lp_stride + (int64_t)a.epoch * (n_pad / 16) + rblk] = sq;

  // ---- backward.  Each epilogue turns its dH tile into dZ = (dH ⊙ cos(ωz))·ω
  // right away (the next phase's B operand) and stores it for the weight grads.
  auto dz_out = [&](int K, int q, float acc, float cs) {
    ho[K % JP][q] = __fmul_rn(__fmul_rn(acc, cs), om);
  };
  auto dz_store = [&](int layer) {
    float* SZl = SZb + (int64_t)layer * WN;
    float* SZtl = SZt + (int64_t)layer * WN;
    return [&, SZl, SZtl](int K) { tile_store(SZtl, SZl, K, ho[K % JP]); };
  };
  auto cos_pre = [&](int layer) {
    const float* SCl = SC + (int64_t)layer * WN + (int64_t)rblk * JW * 256 + lane * 4;
    return [SCl](int K) { return ld4(SCl + K * 256); };
  };
  if constexpr (X3) {
#pragma unroll
    for (int J2 = 0; J2 < JD / 2; ++J2) ys[J2] = split_pair(y[2 * J2], y[2 * J2 + 1]);
  }
  auto& yb = pick_ref<X3>(ys, y);
  wide_layer(ic<kTS>, ic<1>, wsrc(true, L + 1), yb, cos_pre(L), dz_out,
             dz_store(L));   // W_fᵀ [W][D]
  STAMP(4);
  for (int i = L; i >= 2; --i)
    wide_layer(ic<kTS>, ic<1>, wsrc(true, i), hb, cos_pre(i - 1), dz_out, dz_store(i - 1));
  // layer 0: cos(ω(x·w0 + b0)) recomputed with the forward's exact op sequence
  stage_vec(bias, P, 2 * W, tid);   // visible after gemm_phase's prologue barrier
  auto dz0_out = [&](int K, int q, float acc, float) {
    const int f = 16 * K + 4 * g + q;
    const float z = __fadd_rn(__fmul_rn(x, bias[f]), bias[W + f]);
    float s, co;
    sincos_fast(__fmul_rn(om, z), &s, &co);
    ho[K % JP][q] = __fmul_rn(__fmul_rn(acc, co), om);
  };
  // dZ0 is only ever reduced (dw0 = Σ_r dZ0[r]·x_r, db0 = Σ_r dZ0[r]), so the
  // wave reduces its 16 rows here and stores 2W partial sums per 16-row block
  // ([n_pad/16][2][W] in dZ0's scratch slot: 1/8 of the bytes) instead of
  // dZ0 itself.  Reduce-scatter over the 16 lanes c of a lane group g: after
  // the xor-8/4/2/1 steps lanes c, c^1 hold value 4·c3 + 2·c2 + c1 of
  // {Σ dz·x for q = 0..3, Σ dz for q = 0..3}.
  float* PZ = SZ + (int64_t)rblk * 2 * W;
  auto dz0_reduce = [&, PZ](int K) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = __fmul_rn(ho[K % JP][q], x);
      v[4 + q] = ho[K % JP][q];
    }
    const bool b8 = c & 8, b4 = c & 4, b2 = c & 2;
    float w[4], y[2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (b8 ? v[i + 4] : v[i]) + __shfl_xor(b8 ? v[i] : v[i + 4], 8, 64);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      y[i] = (b4 ? w[i + 2] : w[i]) + __shfl_xor(b4 ? w[i] : w[i + 2], 4, 64);
    float t = (b2 ? y[1] : y[0]) + __shfl_xor(b2 ? y[0] : y[1], 2, 64);
    t += __shfl_xor(t, 1, 64);
    if (!(c & 1)) {
      const int idx = (c >> 1);                 // 4·c3 + 2·c2 + c1
      sst(PZ + (idx >> 2) * W + 16 * K + 4 * g + (idx & 3), t);
    }
  };
  wide_layer(ic<1>, ic<0>, wsrc(true, 1), hb, no_pre, dz0_out, dz0_reduce);
  STAMP(5);
  STAMP_RT(13);
}

// ---------------------------------------------------------------------------
// K-split row step for small groups (bf16x3, W >= 128, D = 128).
//
// k_step_rows gives one fit n_pad/64 workgroups, and each wave runs the whole
// GEMM chain of its 16 rows: a lone fit (BASELINE config 2) keeps 32 CUs busy
// and its epoch is that one serial chain.  Here the four waves of a workgroup
// share ONE 16-row block and split every GEMM's reduction (k) dimension:
// wave w owns the k-slices s ≡ w (mod 4) (32 features each) of every layer's
// input, so it holds a quarter of the B operand and loads a quarter of each
// weight tile straight from L2 into registers (PD items in flight, no LDS
// staging, each weight element read once per workgroup).  Per output tile J:
//   every wave: partial Zᵀ tile over its k-slices (6 bf16 MFMAs per slice)
//               → LDS part[slot][wave][q][lane]; one barrier per tile pair;
//   finalize:   wave w sums the four partials of element q = w of every lane
//               in wave order (deterministic) and runs the epilogue (bias,
//               sincos, MSE/dL/dŷ, dZ = dH·cos·ω) on that element only — the
//               epilogue VALU is split four ways too — then stores it to the
//               scratch and to LDS out[slot][q][lane];
//   owner:      wave (J/2) mod 4, whose k-slice of the next phase contains
//               tile J, reads the four elements back as its B-operand tile.
// The scratch layout (H, dZ, G, dZ0 partials) is k_step_rows' own, so the
// parameter kernel is shared; the cos map is private ([rblk][J][q][64 lanes]).
// The k sums are grouped differently from k_step_rows (four partial chains),
// so a fit's result depends on the row variant at the rounding level.
// ---------------------------------------------------------------------------
// Dynamic LDS of every K-split workgroup: with its static LDS (≤ 24 592 B
// at W = 512: partials, finalised tiles, bias) it takes the CU's whole
// 160 KB, so a K-split workgroup never shares a CU with any workgroup that
// uses LDS — its own kind or another kernel's.  Containment kept from the
// co-residency fault: a compile-time forward-only
// instantiation gave wrong blocks when two workgroups shared a CU; the cause
// was the SGPR-soffset rewrite right after a buffer load (KsPhase), which the
// source no longer produces, and the LDS protocol carries no cross-wave race
// (tools/r5/ks_lds_hb.py).  launch_rows also caps the pad at what the
// kernel's actual static LDS leaves.
#ifdef NERFHIP_EXP_KS_TRACE
constexpr unsigned kKsTraceLds = 64u;   // the trace build's ks_tr_* state (below)
#else
constexpr unsigned kKsTraceLds = 0u;
#endif
constexpr unsigned kKsDynLds = 163840u - 24592u - kKsTraceLds;
template <int W> struct KsCfg {
  // A-fragment items (S8) in flight per wave.  (W = 256: 10 and 12 items
  // measured 3.5 % and 7 % slower than 6 on one medium fit: not load-latency
  // bound, profiles/r02/ab_ks_prefetch_depth.log)
#ifndef NERFHIP_KS_PD256
#define NERFHIP_KS_PD256 6
#endif
#ifndef NERFHIP_KS_PD512
#define NERFHIP_KS_PD512 8
#endif
  static constexpr int PD = W >= 512 ? NERFHIP_KS_PD512 : NERFHIP_KS_PD256;
};
__host__ __device__ constexpr int ks_owner(int J) { return (J >> 1) & 3; }
__host__ __device__ constexpr int ks_local(int J) { return 2 * (J >> 3) + (J & 1); }

#ifdef NERFHIP_EXP_KS_TRACE
// Diagnostic build: every LDS access of the K-split kernel traced per lane —
// (barrier count, read/write, LDS byte address) — for two workgroups of each
// mode's launch; tools/r5/ks_lds_hb.py checks that every cross-wave
// write→read and read→overwrite pair of an address is separated by a barrier.
constexpr int kKsTrMax = 4096;   // events per wave
__shared__ uint32_t* ks_tr_buf;
__shared__ int ks_tr_n[4], ks_tr_bc[4];
__device__ __forceinline__ void ks_tr(const void* p, int rw) {
  uint32_t* b = ks_tr_buf;
  if (!b) return;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = ks_tr_n[w];
  if (n < kKsTrMax)
    b[((int64_t)w * kKsTrMax + n) * 64 + lane] =
        ((uint32_t)ks_tr_bc[w] << 18) | ((uint32_t)rw << 17) | ((uint32_t)(uintptr_t)p & 0x1ffffu);
  ks_tr_n[w] = n + 1;
}
__device__ __forceinline__ void ks_tr_barrier() { ks_tr_bc[threadIdx.x >> 6] += 1; }
#define KS_TR(p, rw) ks_tr((p), (rw))
#else
#define KS_TR(p, rw) ((void)0)
__device__ __forceinline__ void ks_tr_barrier() {}
#endif

__device__ __forceinline__ void ks_barrier() {
#ifdef NERFHIP_EXP_KS_VMWAIT   // diagnostic: also drain vector memory
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ks_tr_barrier();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void ks_sync() {
  ks_tr_barrier();
  __syncthreads();
}

// A phase's bias vector (N floats, N compile-time) global → LDS with no
// change of the EXEC mask: every lane of the waves that take part copies N/64
// consecutive floats (N >= 256: all four waves; N = 128: waves 0 and 1, a
// wave-uniform scalar branch).  A divergent `if (4·tid < n)` here narrowed
// EXEC a few instructions after the phase's weight prefetch had issued; on
// gfx950 a vector-memory instruction stalled behind a busy memory pipeline
// can read EXEC after that write, so the masked-off lanes' prefetch never
// landed (the K-split co-residency fault).
template <int N>
__device__ __forceinline__ void ks_stage(float* dst, const float* src, int w, int lane) {
  static_assert(N % 64 == 0 && N >= 128 && N <= 1024, "bias staging shape");
  constexpr int WAVES = N >= 256 ? 4 : N / 64, E = N / (64 * WAVES);
  if (w < WAVES) {                                 // w: an SGPR (readfirstlane)
    const int i = (w * 64 + lane) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) KS_TR(dst + i + e, 1);
    if constexpr (E == 4) st4(dst + i, ld4(src + i));
    else if constexpr (E == 2) {
      const float2 v = *reinterpret_cast<const float2*>(src + i);
      *reinterpret_cast<float2*>(dst + i) = v;
    } else {
      dst[i] = src[i];
    }
  }
}

// A-fragment item i of a K-deep phase (tile J = i / NM, this wave's k-slice
// s = w + 4·(i % NM)): three plane loads, each one contiguous 1 KB block of
// the xoff_ks layout (16 B per lane), straight from L2 into registers.
//
// Every load takes its whole offset from a VGPR (soffset 0, the plane as the
// 12-bit immediate) and all phases share ONE buffer resource over the fit's
// split weights (the matrix offset goes into the VGPR too).  Root cause of the
// K-split co-residency fault: with a compile-time item offset
// in the instruction's soffset, hipcc materialised it into an SGPR right
// before each load (s_mov_b32 s2, 0x12000; buffer_load … s2; s_mov_b32 s2,
// 0x12400; …) and rewrote that SGPR — and the resource SGPRs of a finished
// phase — one instruction after the load issued.  On gfx950 a vector-memory
// instruction that waits behind a backed-up memory pipeline reads its SGPR
// operands late, so under two workgroups per CU some loads fetched the NEXT
// item's offset (wrong weights, whole 16-row blocks wrong).  Eight wait states
// between every such load and the SALU write removed the fault
// (tools/r4/ks_patch.py nopsmov8, profiles/r04/ks_bisect.log); two did not.
// The compiler models this hazard for gfx10+ only, so the kernel avoids the
// pattern: the only SGPRs its loads read are the one resource, set once.
template <int K> struct KsPhase {
  static constexpr int NS = K / 32, NM = K / 128;
  static_assert(K % 128 == 0, "K-split needs K % 128 == 0");
  __amdgpu_buffer_rsrc_t rsrc;
  int voff;
  // lane (row c, k-group g) of wave w: its 16 B of the 1 KB (tile, slice
  // w + 4m, plane) block of the xoff_ks layout; mat: the phase's matrix,
  // in bf16 elements from the fit's split-weight base xs
  __device__ __forceinline__ KsPhase(const uint16_t* xs, int mat, int c, int g, int w)
      : rsrc(__builtin_amdgcn_make_buffer_rsrc((void*)xs, 0, 0x7fffffff, 0x00020000)),
#ifdef NERFHIP_EXP_KS_LINEAR   // diagnostic (timing only): lane-linear offsets
        voff(16 * (c + 16 * g) + 3072 * w + 2 * mat) {}
#else
        voff(64 * c + 16 * g + 3072 * w + 2 * mat) {}
#endif
  template <int I> __device__ __forceinline__ S8 load() const {
    constexpr int J = I / NM, m = I % NM;
    constexpr int base = (J * NS + 4 * m) * 3 * 512;     // plane 0 of slice 4m (+ w: voff)
    // the item's byte offset as a VGPR add the backend cannot split into an
    // SGPR soffset (see above); planes 1 KB apart fit the immediate field
    int v;
    asm("v_add_u32 %0, %1, %2" : "=v"(v) : "i"(2 * base), "v"(voff));
    S8 r;
    r.h = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v, 0, 0);
    r.m = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v + 1024, 0, 0);
    r.l = __builtin_amdgcn_raw_buffer_load_b128(rsrc, v + 2048, 0, 0);
    return r;
  }
};
// the first PD items of a phase into the ring (issued a phase ahead)
template <int K, int PD>
__device__ __forceinline__ void ks_prefetch(S8 (&ring)[PD], const uint16_t* xs, int mat, int c,
                                            int g, int w) {
  const KsPhase<K> ph(xs, mat, c, g, w);
  static_for<0, PD>([&](auto ic_i) {
    constexpr int i = decltype(ic_i)::value;
    ring[i] = ph.template load<i>();
  });
}

// One GEMM phase Zᵀ[JT·16][16 rows] = M[JT·16][K] · Hᵀ of the K-split kernel.
// b: this wave's k-slices s = w + 4m of the input (K/128 of them).  ring
// holds the phase's first PD items on entry (the previous phase issued them);
// before its last epilogue the phase issues the first items of the next one
// (next, KN deep; KN = 0: none).
// pre(J) → a per-lane float loaded one tile ahead of fin; fin(J, acc, pv) →
// the finalised element (feature 16J+4g+w, row c); own(J, f4) on the owner.
template <int K, int JT, int PD, int KN, class Pre, class Fin, class Own>
__device__ __forceinline__ void gemm_ks(const uint16_t* __restrict__ xs, int src, const S8 (&b)[K / 128],
                                        S8 (&ring)[PD], int next, int w, int c, int g,
                                        int lane, float* part, float* outb, Pre&& pre, Fin&& fin,
                                        Own&& own) {
  constexpr int NM = K / 128, NI = JT * NM;
  static_assert(NI >= PD, "phase shorter than the prefetch depth");
  const KsPhase<K> ph(xs, src, c, g, w);
  const f4 zero4 = {0.f, 0.f, 0.f, 0.f};
  // tiles go in pairs, one barrier per pair: LDS slot of tile J = 2·(pair parity) + (J & 1)
  auto slot = [](int J) { return 2 * ((J >> 1) & 1) + (J & 1); };
  auto finalize = [&](int J, float pv) {
    const float* p = part + slot(J) * 1024 + w * 64 + lane;
    KS_TR(p, 0); KS_TR(p + 256, 0); KS_TR(p + 512, 0); KS_TR(p + 768, 0);
    const float acc = ((p[0] + p[256]) + p[512]) + p[768];
    KS_TR(outb + slot(J) * 256 + w * 64 + lane, 1);
    outb[slot(J) * 256 + w * 64 + lane] = fin(J, acc, pv);
  };
  auto owner_read = [&](int J) {
    if (w == ks_owner(J)) {
      const float* o = outb + slot(J) * 256 + lane;
      KS_TR(o, 0); KS_TR(o + 64, 0); KS_TR(o + 128, 0); KS_TR(o + 192, 0);
      const f4 v = {o[0], o[64], o[128], o[192]};
      own(J, v);
    }
  };
  static_assert(JT % 2 == 0, "tile pairs");
  float pv_prev[2] = {0.f, 0.f};
  static_for<0, JT / 2>([&](auto Pc) {
    constexpr int Pp = decltype(Pc)::value;
    const float pv[2] = {pre(2 * Pp), pre(2 * Pp + 1)};
    f4 acc[2];
    static_for<0, 2>([&](auto tc) {
      constexpr int t = decltype(tc)::value, J = 2 * Pp + t;
      f4 hi = zero4, lo = zero4;
      static_for<0, NM>([&](auto mc) {
        constexpr int m = decltype(mc)::value, i = J * NM + m;
        mfma16x3(ring[i % PD], b[m], hi, lo);
        if constexpr (i + PD < NI) ring[i % PD] = ph.template load<i + PD>();
        if constexpr (Pp > 0 && m == 0) finalize(J - 2, pv_prev[t]);
      });
      acc[t] = hi + lo;
    });
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float* pw = part + slot(2 * Pp + t) * 1024 + w * 256 + lane;   // part[slot][w][q][lane]
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        KS_TR(pw + q * 64, 1);
        pw[q * 64] = acc[t][q];
      }
      pv_prev[t] = pv[t];
    }
    ks_barrier();
    if constexpr (Pp > 0) {
      owner_read(2 * Pp - 2);
      owner_read(2 * Pp - 1);
    }
  });
  if constexpr (KN > 0) {
    if (next >= 0) ks_prefetch<KN>(ring, xs, next, c, g, w);
  }
  finalize(JT - 2, pv_prev[0]);
  finalize(JT - 1, pv_prev[1]);
  ks_barrier();
  owner_read(JT - 2);
  owner_read(JT - 1);
}

template <int W, int D, int MODE>
__global__ void __launch_bounds__(256, 1) k_step_rows_ks(KArgs a) {
  FLIGHT_ENTER();
  static_assert(W >= 128 && D == 128, "K-split rows: W >= 128, D = 128");
  constexpr int JW = W / 16, JD = D / 16, PD = KsCfg<W>::PD;
  constexpr int NO = W / 64;                 // owned tiles of a W-wide output
  __shared__ __attribute__((aligned(16))) float part[4 * 4 * 4 * 64];   // [slot][wave][q][lane]
  __shared__ __attribute__((aligned(16))) float outb[4 * 4 * 64];       // [slot][q][lane]
  __shared__ __attribute__((aligned(16))) float bias[2 * W];
  __shared__ float lsum[4];
  int fit, rblk;
#ifdef NERFHIP_EXP_KS_ALTFIT
  // diagnostic build: a two-fit group with runs of 256 workgroups alternating
  // between the fits, so that the two workgroups sharing a CU (b, b + 256)
  // read different copies of the weights (tools/r3/ks_probe.py KS_FITS=2)
  if (a.n_fits == 2) {
    const int b = blockIdx.x;
    fit = (b >> 8) & 1;
    rblk = (b & 255) + 256 * (b >> 9);
    if (rblk >= a.n_pad / 16) return;
  } else
#endif
  if (!map_block(blockIdx.x, a.n_fits, a.n_pad / 16, fit, rblk)) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, g = lane >> 4;
  const int L = fit_layers_of(a, fit);
  FLIGHT_DEPTH(L, fit);
  const float om = a.fit_omega[fit];
  const int r = rblk * 16 + c;
  const bool valid = r < a.N;
  // one instantiation for both modes: the forward-only mode (a.mode = 1) runs
  // the same code with the stores and the backward skipped (see launch_rows)
  // MODE -1: one instantiation, mode read at run time; 0 / 1: compile-time
  // train / forward-only (diagnostic builds, NERFHIP_EXP_KS_MODES)
  const bool train = MODE < 0 ? a.mode == 0 : MODE == 0;
  // diagnostic builds: the mode compile-time in one part of the kernel only
#if defined(NERFHIP_EXP_KS_SPLIT_H)
  const bool train_h = train, train_f = a.mode == 0;
#elif defined(NERFHIP_EXP_KS_SPLIT_F)
  const bool train_h = a.mode == 0, train_f = train;
#else
  const bool train_h = train, train_f = train;
#endif
  const int n_pad = a.n_pad;
  const float* P = a.params + fit * a.p_stride;
  float* S = a.scratch + fit * a.s_stride;
  const int64_t WN = (int64_t)W * n_pad;
  float* SH = S;
  float* SZ = S + (int64_t)(a.L_max + 1) * WN;
  float* SG = S + 2 * (int64_t)(a.L_max + 1) * WN;
  float* SC = SG + (int64_t)D * n_pad;
  const uint16_t* XS = a.wsplit + fit * a.ws_stride;
  const int fe = 4 * g + w;                  // this wave's finalised feature inside a tile
  // row-block-major scratch element (feature 16J+fe, row c)
  const int64_t eoff = (int64_t)rblk * W * 16 + fe * 16 + c;
  const int64_t coff = (int64_t)rblk * JW * 256 + w * 64 + lane;   // private cos map

  float ho[NO][4];
  S8 hs[W / 128];
  S8 ys[1];
  auto split_out = [&](auto nslices) {
#pragma unroll
    for (int m = 0; m < decltype(nslices)::value; ++m) hs[m] = split_pair(ho[2 * m], ho[2 * m + 1]);
  };
  auto own = [&](int J, f4 v) {
#pragma unroll
    for (int q = 0; q < 4; ++q) ho[ks_local(J)][q] = v[q];
  };
  auto no_pre = [](int) { return 0.f; };
  S8 ring[PD];                               // A-fragment items in flight
  KSTAMP(0);
  // matrix offsets of the fit's split weights (bf16 elements; < 2^31 bytes)
  auto xm = [&](bool bwd_mat, int i) { return (int)xs_mat(W, D, L, bwd_mat, i); };
  ks_prefetch<W>(ring, XS, xm(false, 1), c, g, w);
#ifdef NERFHIP_EXP_KS_TRACE
  if (tid == 0)
    ks_tr_buf = a.pstamps && blockIdx.x < 2
                    ? reinterpret_cast<uint32_t*>(a.pstamps) +
                          (int64_t)(2 * a.mode + blockIdx.x) * 4 * kKsTrMax * 64
                    : nullptr;
  if (tid < 4) ks_tr_n[tid] = ks_tr_bc[tid] = 0;
  __syncthreads();
#endif

  // ---- layer 0 (K = 1, VALU): this wave's tiles J = 2s + h, s = w + 4m
  ks_stage<2 * W>(bias, P, w, lane);
  ks_sync();
  const float x = a.pos[r];
  float* SHt = SH + (int64_t)rblk * W * 16 + g * 64 + (c & 3) * 16 + (c >> 2) * 4;
#pragma unroll
  for (int t = 0; t < NO; ++t) {
    const int J = 2 * (w + 4 * (t >> 1)) + (t & 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = 16 * J + 4 * g + q;
      KS_TR(bias + f, 0); KS_TR(bias + W + f, 0);
      const float z = __fadd_rn(__fmul_rn(x, bias[f]), bias[W + f]);
      float s, co;
      sincos_fast(__fmul_rn(om, z), &s, &co);
      ho[t][q] = s;
    }
    if (train_h) {
      const f4 v = {ho[t][0], ho[t][1], ho[t][2], ho[t][3]};
      sst4(SHt + J * 256, quad_transpose(v, c));
    }
  }
  split_out(ic<W / 128>);
  ks_sync();
  KSTAMP(1);

  // ---- hidden SineLayers 1..L
  for (int i = 1; i <= L; ++i) {
    ks_stage<W>(bias, P + off_hidden_w(W, i) + W * W, w, lane);
    float* SHi = SH + (int64_t)i * WN + eoff;
    float* SCi = SC + (int64_t)i * WN + coff;
    gemm_ks<W, JW, PD, W>(
        XS, xm(false, i), hs, ring, xm(false, i + 1), w, c, g,
        lane, part, outb, no_pre,
        [&](int J, float acc, float) {
          KS_TR(bias + 16 * J + fe, 0);
          const float z = __fadd_rn(acc, bias[16 * J + fe]);
          float s, co;
          sincos_fast(__fmul_rn(om, z), &s, &co);
          if (train_h) {
            sst(SHi + J * 256, s);
            sst(SCi + J * 256, co);
          }
          return s;
        },
        own);
    split_out(ic<W / 128>);
  }

  // ---- final nn.Linear(W, D), MSE, dL/dŷ
  KSTAMP(2);
  ks_stage<D>(bias, P + off_final_w(W, L) + W * D, w, lane);
  const float* T = a.tnorm + fit * a.t_stride + (int64_t)r * D + fe;
  // no per-lane branches (EXEC writes) in this kernel: whether ŷ is written is
  // a wave-uniform scalar test of the kernel argument
  const bool has_y = a.y_out != nullptr;
  float* yo = has_y ? a.y_out + fit * a.y_stride + (int64_t)r * D + fe : nullptr;
  float* SGe = SG + (int64_t)rblk * D * 16 + fe * 16 + c;
  float sq = 0.f;
  gemm_ks<W, JD, PD, D>(
      XS, xm(false, L + 1), hs, ring, train_f ? xm(true, L + 1) : -1,
      w, c, g,
      lane, part, outb,
      [&](int J) { return train_f ? T[16 * J] : 0.f; },
      [&](int J, float acc, float t) {
        KS_TR(bias + 16 * J + fe, 0);
        const float y = __fadd_rn(acc, bias[16 * J + fe]);
        if (has_y) yo[16 * J] = y;
        float gv = 0.f;
        if (train_f) {
          const float diff = y - t;
          sq = valid ? fmaf(diff, diff, sq) : sq;
          gv = valid ? a.grad_scale * diff : 0.f;
          sst(SGe + J * 256, gv);
        }
        return gv;
      },
      own);
  KSTAMP(3);
  if (!train_f) return;
  sq = wave_sum(sq);
  KS_TR(lsum + w, 1);
  lsum[w] = sq;                  // every lane holds the wave's sum
  ys[0] = split_pair(ho[0], ho[1]);

  // ---- backward: dZ = (dH ⊙ cos(ωz))·ω, stored for the weight gradients
  // (the phase after W_iᵀ is W_{i-1}ᵀ, down to W_1ᵀ: xs_mat(.., true, i - 1))
  auto bwd = [&](int Mt, const auto& bop, int layer, int next) {
    const float* SCl = SC + (int64_t)layer * WN + coff;
    float* SZl = SZ + (int64_t)layer * WN + eoff;
    constexpr int K = (sizeof(bop) / sizeof(bop[0])) * 128;
    gemm_ks<K, JW, PD, W>(
        XS, Mt, bop, ring, next, w, c, g, lane, part, outb, [SCl](int J) { return SCl[J * 256]; },
        [&, SZl](int J, float acc, float cs) {
          const float dz = __fmul_rn(__fmul_rn(acc, cs), om);
          sst(SZl + J * 256, dz);
          return dz;
        },
        own);
    split_out(ic<W / 128>);
  };
  bwd(xm(true, L + 1), ys, L, xm(true, L));   // W_fᵀ [W][D]
  KSTAMP(4);
  for (int i = L; i >= 2; --i)
    bwd(xm(true, i), hs, i - 1, xm(true, i - 1));
  KSTAMP(5);
  // layer 0: cos(ω(x·w0 + b0)) recomputed; dZ0 reduced over the 16 rows at once
  ks_stage<2 * W>(bias, P, w, lane);
  float* PZ = SZ + (int64_t)rblk * 2 * W;
  gemm_ks<W, JW, PD, 0>(
      XS, xm(true, 1), hs, ring, -1, w, c, g, lane, part, outb, no_pre,
      [&](int J, float acc, float) {
        const int f = 16 * J + fe;
        KS_TR(bias + f, 0); KS_TR(bias + W + f, 0);
        const float z = __fadd_rn(__fmul_rn(x, bias[f]), bias[W + f]);
        float s, co;
        sincos_fast(__fmul_rn(om, z), &s, &co);
        const float dz = __fmul_rn(__fmul_rn(acc, co), om);
        float sx = __fmul_rn(dz, x), s1 = dz;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {
          sx += __shfl_xor(sx, o, 64);
          s1 += __shfl_xor(s1, o, 64);
        }
        // all 16 lanes of the group hold both sums: lane c = 1 stores Σdz, the
        // others Σdz·x (identical values to one address) — one store, no EXEC write
        const bool one = c == 1;
        sst(one ? PZ + W + f : PZ + f, one ? s1 : sx);
        return 0.f;
      },
      [](int, f4) {});
  if (w == 0) {                  // scalar branch; the wave's lanes store one value
    KS_TR(lsum, 0); KS_TR(lsum + 1, 0); KS_TR(lsum + 2, 0); KS_TR(lsum + 3, 0);
    a.loss_partial[fit * a.lp_stride + (int64_t)a.epoch * (n_pad / 16) + rblk] =
        ((lsum[0] + lsum[1]) + lsum[2]) + lsum[3];
  }
  KSTAMP(6);
}

// Opt-in variants (NERFHIP_VARIANTS builds only, tools/build_variant.py): the
// 32-row row kernel and the fused split-K reduction.  Both are correct and
// measured slower than the defaults, so the product library
// does not instantiate them; nerfhip_build_flags() reports a variant build.
#ifdef NERFHIP_VARIANTS
// ---------------------------------------------------------------------------
// 32-row row step (bf16x3; W = 256, D = 128): k_step_rows32.
//
// k_step_rows' contract — the same scratch (H, dZ, G row-block-major, the
// dZ0 partials, the loss partials), so the parameter kernel is shared — with
// every GEMM on v_mfma_f32_32x32x16_bf16 over 32 data rows per wave:
//  * one A fragment (a 32-feature × 16-k weight slice, three planes) feeds
//    32 rows instead of 16, and four waves × 32 rows share one staged copy of
//    the weights: LDS fragment reads and LDS-DMA staging per FLOP halve;
//  * a 32 × 32 × 16 MFMA holds its SIMD's vector issue for 8 of its 32
//    cycles, a 16 × 16 × 32 one for 8 of 16: 1.5x the free VALU issue per
//    FLOP for the sincos / split epilogue (MI355X_MICROARCH.md cycle table);
//  * the layer input — the B operand, 32 rows × W k in three planes, 192
//    registers at W = 256 — lives in the accumulator registers (AGPRs), which
//    gfx950 MFMAs read as sources (to_agpr); the layer output (128 VGPRs) and
//    the accumulators stay in VGPRs (this kernel's translation unit is built
//    with -amdgpu-mfma-vgpr-form, _build.py).  One wave per SIMD.
// Orientation as k_step_rows (Zᵀ = W·Hᵀ).  The 32 × 32 accumulator tile of
// output features 32J.. holds, in lane (row j = lane & 31, h = lane >> 5),
// register e = feature 32J + 8(e>>2) + 4h + (e&3) of row j; registers
// 8s..8s+7 are exactly the next layer's B fragment of k-step 2J + s under
// the k order perm32 (cdna_hip_programming.md §3), which the weight planes
// use (xoff32, written by the Adam epilogue and the prologue).
// The k sums are grouped differently from k_step_rows (32 × 32 × 16 instead
// of 16 × 16 × 32 MFMAs), so the two agree to rounding, not bitwise
// (test_rows32_matches_regular).
// ---------------------------------------------------------------------------
template <int K> struct R32Cfg {
  static constexpr int KC = 128, NH = K / KC, KT = KC / 16;   // sub-chunk: 32 rows × KC
  static constexpr int CH = 3 * 32 * KC;                       // bf16 per ring buffer (24 KB)
  static constexpr int PLB = 2 * 32 * KC;                      // bytes per plane
  static constexpr int NDMA = 3 * 32 * (KC / 8) / 256;         // DMAs per wave and sub-chunk
  static_assert(K % KC == 0, "rows32: K must be a multiple of 128");
};
// sub-chunk buffers of the LDS ring: sub-chunk u + NR32 - 1 is issued at the
// top of sub-chunk u and waited for at the end of u + NR32 - 2
#ifndef NERFHIP_R32_RING
#define NERFHIP_R32_RING 3
#endif
constexpr int NR32 = NERFHIP_R32_RING;
static_assert(NR32 >= 3, "rows32 ring: at least 3 buffers");
constexpr int kRing32 = NR32 * R32Cfg<128>::CH;

// a B fragment moved into accumulator registers: an MFMA reads it from there
// directly (the compiler emits the v_accvgpr_write copies and the hazards)
__device__ __forceinline__ S8 to_agpr(const S8& v) {
  S8 r;
  asm("" : "=a"(r.h) : "0"(v.h));
  asm("" : "=a"(r.m) : "0"(v.m));
  asm("" : "=a"(r.l) : "0"(v.l));
  return r;
}

// LDS-DMA of sub-chunk u (a 32-row × 128-k slice of all three planes, one
// contiguous 24 KB run of the xoff32 layout) of the matrix at src into ring
// slot u % NR32.  Round m moves physical slots tid + 256m (16 slots per row):
// row tid/16 + 16m of the [3][32] plane rows, slot tid % 16; its swizzle
// (row & 15 = tid/16) is the same in every round, so one per-lane source
// offset serves all rounds (+16m rows: a compile-time addend).  The DMA
// image is lane-linear; the bank swizzle (16-B slot s of row r at
// s ^ (r & 15)) lives on the source address.
struct R32Dma {
  static constexpr int KC = 128, CH = 3 * 32 * KC, NDMA = 6;
  __amdgpu_buffer_rsrc_t rsrc;
  int voff, wave;
  __device__ __forceinline__ R32Dma(const uint16_t* src, int tid)
      : rsrc(__builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7fffffff, 0x00020000)),
        voff(2 * ((tid >> 4) * KC + 8 * ((tid & 15) ^ (tid >> 4)))),
        wave(__builtin_amdgcn_readfirstlane(tid >> 6)) {}
  // The whole source offset goes into the per-lane VGPR (an asm add the
  // backend cannot split): as an SGPR soffset, hipcc materialised each
  // constant into an SGPR right before its load and rewrote that SGPR one
  // instruction later — the pattern behind the K-split co-residency fault
  // (KsPhase).
  template <int U> __device__ __forceinline__ void issue(uint16_t* ring) const {
    typedef __attribute__((address_space(3))) void lds_void;
    uint16_t* buf = ring + (U % NR32) * CH;
    static_for<0, NDMA>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
      int v;
      asm("v_add_u32 %0, %1, %2" : "=v"(v) : "i"(2 * U * CH + 32 * m * KC), "v"(voff));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)(buf + 8 * (256 * m + 64 * wave)),
                                               16, v, 0, 0, 0);
    });
  }
};
// a phase's first NR32 - 1 sub-chunks, issued ahead of it (by the previous
// phase right after its last barrier, or by the kernel before layer 0)
__device__ __forceinline__ void r32_prefetch(const uint16_t* src, uint16_t* ring, int tid) {
  const R32Dma d(src, tid);
  static_for<0, NR32 - 1>([&](auto uc) { d.template issue<decltype(uc)::value>(ring); });
}

// One GEMM phase Zᵀ[32·JT][32 rows] = M[32·JT][K] · Hᵀ of the 32-row kernel
// (gemm_phase_x3's pipeline on 32-row sub-chunks): sub-chunk u = J·NH + hh
// (output tile J, k-chunk hh) of the xoff32 planes arrives by LDS-DMA into an
// NR32-deep ring NR32 - 1 sub-chunks ahead; each of its KT k-steps is three
// ds_read_b128 (one per plane; every 16-lane group reads one bank row once)
// and six 32 × 32 × 16 MFMAs.
//   pre(J)      issues tile J's per-lane loads at the top of tile J;
//   epre(J, ep) issues tile J's NEP epilogue operands from LDS (bias, w0 / b0:
//               inline-asm ds_read_b128 into ep) together with the first A
//               fragment of tile J+1, so they land in that fragment's wait —
//               a compiler-placed LDS read inside the k-steps would get an
//               lgkmcnt(0) that also waits for the next k-step's fragments
//               and exposes their latency at every k-step;
//   elem(J, e, ep)  epilogue of element e of tile J, spread over tile J+1's
//               k-steps (16 / (KT·NH) per k-step);
//   done(J, hi, lo)  hands over tile J's accumulators at its end;
//   flush(J, t) tile J's stores of register group t (0..3), in k-step t of
//               tile J+2 (after that sub-chunk's DMA): spread over the
//               k-steps, a 16-B store's issue stall sits beside MFMAs
//               instead of in a burst ahead of them (≈870 cycles per tile
//               as a burst, profiles/r05/stamps32b_*.log).
// NST / NLD: the store / load instruction counts of a whole flush(J) / pre,
// exact or fewer (fewer only over-waits).  The final layer passes the count
// of a plain training flush (4); on a probe epoch (y_out set) its flush also
// stores ŷ and issues 8, an undercount of the same safe kind, and so does
// the next phase's NAFTER.
// Phase boundaries.  The phase's first NR32 - 1 sub-chunks were issued before
// it (r32_prefetch), followed by NAFTER vector-memory ops (the previous
// phase's last two flushes, or layer 0's stores; fewer only over-waits), and
// the phase issues the NEXT phase's first sub-chunks (`next`, nullptr: none)
// right after its last barrier, before its own last epilogue and stores: the
// in-order vmcnt then never makes a phase's first wait cover the previous
// phase's stores.  (With each phase issuing its own first sub-chunks, and the
// bias loaded from global memory at every phase, the compiler's vmcnt(0) for
// that load and the end-of-phase waits drained every store and exposed the
// first sub-chunk's latency: ≈30 K of a wave's ≈480 K cycles per phase,
// profiles/r05/stamps32_*.log.)
// The B operand b[k-step] is split from the previous layer's f32 output
// tiles `hs` lazily, one k-step ahead, inside tile 0 (whose k-steps carry no
// epilogue): hs (the caller's output array) is rewritten only from the end
// of tile 0 on.  Split between the phases instead, ≈1,100 VALU per phase
// (128 elements and 192 accumulator-register writes) ran with nothing to
// overlap at one wave per SIMD.
template <int K, int JT, int NST, int NLD, int NEP, int NAFTER, int SSLOT, int NB, int NTS,
          class Pre, class Epre, class Elem, class Done, class Flush>
__device__ __forceinline__ void gemm32(const uint16_t* __restrict__ src,
                                       const uint16_t* __restrict__ next, uint16_t* ring,
                                       S8 (&b)[NB], const float (&hs)[NTS][16], int tid,
                                       int lane, Pre&& pre, Epre&& epre, Elem&& elem,
                                       Done&& done, Flush&& flush,
                                       unsigned long long (&sacc)[32]) {
  constexpr int sslot = SSLOT;
  using C = R32Cfg<K>;
  constexpr int NH = C::NH, KT = C::KT, U = JT * NH, CH = C::CH, PLB = C::PLB;
  constexpr int NDMA = C::NDMA, EPK = 16 / (KT * NH);
  static_assert(NB >= K / 16 && 2 * NTS >= K / 16 && EPK * KT * NH == 16, "rows32 phase shape");
  static_assert(NDMA == R32Dma::NDMA && CH == R32Dma::CH && U >= NR32 - 1, "rows32 DMA shape");
  constexpr int KS = K / 16;   // k-steps of the B operand
  auto split_b = [&](auto kc) {
    constexpr int kk = decltype(kc)::value;
    float x8[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) x8[e] = hs[kk >> 1][8 * (kk & 1) + e];
    b[kk] = to_agpr(split8(x8));
  };
  const R32Dma dm(src, tid);
  // lane (row j, half h): k-step kt reads logical slot 2kt + h of row j
  const int j = lane & 31;
  const uint32_t arow = lds_addr(ring) + 2 * C::KC * j;
  const uint32_t ax = (uint32_t)(((lane >> 5) ^ (j & 15)) << 4);
  auto aread = [&](auto uc, auto ktc) {
    constexpr int OFF = (decltype(uc)::value % NR32) * 2 * CH;
    constexpr int kt = decltype(ktc)::value;
    const uint32_t ad = arow + (((uint32_t)kt << 5) ^ ax);
    S8 r;
    if constexpr (OFF + 2 * PLB < 65536) {
      r.h = ds_read16<OFF>(ad);
      r.m = ds_read16<OFF + PLB>(ad);
      r.l = ds_read16<OFF + 2 * PLB>(ad);
    } else {
      const uint32_t ad2 = ad + OFF;
      r.h = ds_read16<0>(ad2);
      r.m = ds_read16<PLB>(ad2);
      r.l = ds_read16<2 * PLB>(ad2);
    }
    return r;
  };
  auto lgkm_wait = [](S8& r) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r.h), "+v"(r.m), "+v"(r.l));
  };
  u4 ep[NEP > 0 ? NEP : 1];
  auto ep_wait = [&]() {   // the epilogue operands land with the fragment wait
#pragma unroll
    for (int i = 0; i < NEP; ++i) asm volatile("" : "+v"(ep[i]));
  };
  auto vm_wait_barrier = [&](auto nc) {
    if constexpr (decltype(nc)::value >= 0)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(decltype(nc)::value));
    asm volatile("s_waitcnt lgkmcnt(0)");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // vector-memory ops issued after sub-chunk d's DMA and before the wait for
  // it at the end of iteration `upto` (d = 0, upto = -1: the phase's first
  // wait), in the issue order [prefetch DMA 0 .. NR32-2][NAFTER]
  // [iteration 0: pre, DMA(NR32-1), flush][iteration 1] ...
  auto younger = [](int d, int upto) {
    auto loads = [](int v) { return v % NH == 0 ? NLD : 0; };
    auto stores = [](int v) { return v % NH == 0 && v / NH >= 2 ? NST : 0; };
    auto dmas = [](int v) { return v + NR32 - 1 < U ? NDMA : 0; };
    int n = 0, v0 = 0;
    if (d < NR32 - 1) {
      n += (NR32 - 2 - d) * NDMA + NAFTER;   // the rest of the prefetch, NAFTER
    } else {
      const int vd = d - NR32 + 1;           // the iteration that issued DMA(d)
      if (vd <= upto) n += stores(vd);       // its flush comes after the DMA
      v0 = vd + 1;
    }
    for (int v = v0; v <= upto; ++v) n += loads(v) + dmas(v) + stores(v);
    return n;
  };
  const unsigned long long t_p0 = MEMTIME();
  vm_wait_barrier(std::integral_constant<int, younger(0, -1)>{});   // sub-chunk 0 landed
  const unsigned long long t_p1 = MEMTIME();
  split_b(ic<0>);
  S8 a_cur = aread(ic<0>, ic<0>);
  lgkm_wait(a_cur);
#ifdef NERFHIP_STAMPS
  R32STAMP_ADD(sacc, 29, t_p1 - t_p0);          // phase heads: wait for sub-chunk 0
  R32STAMP_ADD(sacc, 30, MEMTIME() - t_p1);     // phase heads: first split + fragment
#else
  (void)t_p0; (void)t_p1;
#endif
  f16v hi, lo;
  static_for<0, U>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    constexpr int J = u / NH, hh = u % NH;
    const unsigned long long t_f0 = MEMTIME();
    if constexpr (hh == 0) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        hi[e] = 0.f;
        lo[e] = 0.f;
      }
      pre(ic<J>);
    }
    __builtin_amdgcn_sched_barrier(0);   // pre before the DMA, flush after it: vmcnt counts in order
    const unsigned long long t_d0 = MEMTIME();
    if constexpr (u + NR32 - 1 < U) dm.template issue<u + NR32 - 1>(ring);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t_d1 = MEMTIME();
    static_for<0, KT>([&](auto ktc) {
      constexpr int kt = decltype(ktc)::value;
      S8 a_nxt = a_cur;
      if constexpr (kt + 1 < KT) a_nxt = aread(uc, ic<kt + 1>);
      // the next fragment's reads stay ahead of this k-step's MFMAs (left
      // free, the scheduler sank them below two MFMAs, and their LDS latency
      // showed at the k-step's closing wait)
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (J == 0 && hh * KT + kt + 1 < KS) split_b(ic<hh * KT + kt + 1>);
      if constexpr (hh == 0 && J >= 2 && kt < 4) flush(ic<J - 2>, ic<kt>);
      mfma32x3(a_cur, b[hh * KT + kt], hi, lo);
      if constexpr (J > 0) {
        static_for<0, EPK>([&](auto ec) {
          elem(ic<J - 1>, ic<(hh * KT + kt) * EPK + decltype(ec)::value>, ep);
        });
      }
#ifndef NERFHIP_R32_VPG
#define NERFHIP_R32_VPG 6
#endif
      // one MFMA, then up to VPG vector ALU instructions, six times: at one
      // wave per SIMD nothing else fills an MFMA's shadow (it holds the
      // SIMD's vector issue for 8 of its 32 cycles: ~6 four-cycle VALU fit
      // beside it), and the free schedule clustered the epilogue VALU after
      // the MFMAs, where every instruction cost its full issue time
      if constexpr (NERFHIP_R32_VPG > 0) {
        static_for<0, 6>([&](auto) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, NERFHIP_R32_VPG, 0);
        });
      }
      // keep the MFMAs (and the epilogue VALU) ahead of the wait for the next
      // fragment: left free, the scheduler sank five of the six MFMAs below
      // it and the LDS latency showed in every k-step (at one wave per SIMD
      // nothing else covers it; gemm_phase_x3's PIN)
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (kt + 1 < KT) lgkm_wait(a_nxt);
      __builtin_amdgcn_sched_barrier(0);
      a_cur = a_nxt;
    });
    if constexpr (hh == NH - 1) done(ic<J>, hi, lo);
    const unsigned long long t_w0 = MEMTIME();
    // sub-chunk u+1 landed everywhere (the last iteration waits for no DMA:
    // its barrier only frees the ring for the next phase's prefetch)
    vm_wait_barrier(std::integral_constant<int, (u + 1 < U ? younger(u + 1, u) : -1)>{});
#ifdef NERFHIP_STAMPS
    const unsigned long long t_w1 = MEMTIME();
    R32STAMP_ADD(sacc, sslot, t_d1 - t_d0);      // DMA issue
    R32STAMP_ADD(sacc, sslot + 1, t_w0 - t_d1);  // k-steps (MFMA + epilogue VALU + LDS reads + split)
    R32STAMP_ADD(sacc, sslot + 2, t_w1 - t_w0);  // vm wait + barrier
    R32STAMP_ADD(sacc, sslot + 3, 1ull);         // sub-chunks
    R32STAMP_ADD(sacc, 31, t_d0 - t_f0);         // flush + pre (all phases)
#else
    (void)t_d0; (void)t_d1; (void)t_w0; (void)sacc; (void)sslot; (void)t_f0;
#endif
    if constexpr (u + 1 < U) {
      // tile J's epilogue operands, read now for its epilogue in tile J+1
      if constexpr (NEP > 0 && (u + 1) % NH == 0) epre(ic<J>, ep);
      a_cur = aread(ic<u + 1>, ic<0>);
      lgkm_wait(a_cur);
      if constexpr (NEP > 0 && (u + 1) % NH == 0) ep_wait();
    }
#ifdef NERFHIP_STAMPS
    R32STAMP_ADD(sacc, 20, MEMTIME() - t_w1);    // first fragment of the next sub-chunk
#endif
  });
  if (next) r32_prefetch(next, ring, tid);   // (wave-uniform)
  const unsigned long long t_e0 = MEMTIME();
  auto flush_all = [&](auto Jc) { static_for<0, 4>([&](auto tc) { flush(Jc, tc); }); };
  if constexpr (JT >= 2) flush_all(ic<JT - 2>);
  if constexpr (NEP > 0) {
    epre(ic<JT - 1>, ep);
    asm volatile("s_waitcnt lgkmcnt(0)");
    ep_wait();
  }
  static_for<0, 16>([&](auto ec) { elem(ic<JT - 1>, ec, ep); });
  flush_all(ic<JT - 1>);
#ifdef NERFHIP_STAMPS
  R32STAMP_ADD(sacc, 28, MEMTIME() - t_e0);   // phase tails
#else
  (void)t_e0;
#endif
}

template <int W, int D, bool TRAIN>
__global__ void __launch_bounds__(256, 1) k_step_rows32(KArgs a) {
  static_assert(W == 256 && (D == 128), "rows32: W = 256, D = 128");
  constexpr int JW = W / 32, JD = D / 32;
  __shared__ __attribute__((aligned(16))) uint16_t ring[kRing32];
  // every bias of the fit, staged once: w0 ‖ b0 ‖ b_1 .. b_L ‖ b_f
  __shared__ __attribute__((aligned(16))) float bias[(2 + NERFHIP_MAX_LAYERS) * W + D];
  int fit, tile;
  if (!map_block(blockIdx.x, a.n_fits, a.n_pad / 128, fit, tile)) return;
#ifdef NERFHIP_STAMPS
  unsigned long long* const stp = a.pstamps && TRAIN ? a.pstamps + 262144 : nullptr;
#else
  unsigned long long* const stp = nullptr;
#endif
  unsigned long long sacc[32] = {};   // register stamp sums (stamps builds only)
  R32STAMP(stp, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, h = lane >> 5;
  const int L = fit_layers_of(a, fit);
  const float om = a.fit_omega[fit];
  const int n_pad = a.n_pad;
  const int r0 = tile * 128 + 32 * wave;       // the wave's first row
  const int r = r0 + j;                        // this lane's row (B / D column)
  const bool valid = r < a.N;
  constexpr bool train = TRAIN;
  const float* P = a.params + fit * a.p_stride;
  float* S = a.scratch + fit * a.s_stride;
  const int64_t WN = (int64_t)W * n_pad;
  float* SH = S;
  float* SZ = S + (int64_t)(a.L_max + 1) * WN;
  float* SG = S + 2 * (int64_t)(a.L_max + 1) * WN;
  float* SC = SG + (int64_t)D * n_pad;
  const uint16_t* XS = a.wsplit + fit * a.ws_stride;
  // row-block-major stores after quad_transpose: lane (j = 4a + b, h) writes
  // feature 32J + 8t + 4h + b of rows 4a..4a+3 (16 contiguous bytes)
  const int blk = (r0 >> 4) + (j >> 4);        // this lane's 16-row block
  const int tq = (4 * h + (j & 3)) * 16 + 4 * ((j >> 2) & 3);
  float* SHt = SH + (int64_t)blk * W * 16 + tq;
  float* SZt = SZ + (int64_t)blk * W * 16 + tq;
  float* SGt = SG + (int64_t)blk * D * 16 + tq;
  // private cos map [n_pad/32][W/32][4][64 lanes][4]: one 1 KB run per (tile, t)
  const int64_t coff = (int64_t)(r0 >> 5) * JW * 4 * 256 + lane * 4;
  // register group t (features 32J + 8t + 4h + 0..3) of a tile
  auto tile_store = [&](float* base, auto Jc, auto tc, const float (&v)[16]) {
    constexpr int J = decltype(Jc)::value, t = decltype(tc)::value;
    const f4 x = {v[4 * t], v[4 * t + 1], v[4 * t + 2], v[4 * t + 3]};
    sst4(base + (32 * J + 8 * t) * 16, quad_transpose(x, j));
  };
  // (element e of a tile is feature 32J + 8(e>>2) + 4h + (e&3))
  float ho[JW][16];    // a layer's output tiles (raw accumulators until their epilogue)
  S8 hb[W / 16];       // the layer input as split k-steps, in AGPRs
  auto done = [&](auto Jc, const f16v& hi, const f16v& lo) {
    constexpr int J = decltype(Jc)::value;
#pragma unroll
    for (int e = 0; e < 16; ++e) ho[J][e] = hi[e] + lo[e];
  };
  auto no_pre = [](auto) {};
  auto no_epre = [](auto, auto&) {};
  auto xsm = [&](bool bwd, int i) { return XS + xs_mat(W, D, L, bwd, i); };
  // a tile's 16 epilogue constants from LDS (bias: ep[t][q] = bias[bo + 32J + 8t + 4h + q])
  const uint32_t bias_lane = lds_addr(bias) + 16 * h;
  auto bias_epre = [&](uint32_t bo) {
    const uint32_t base = bias_lane + 4 * bo;
    return [base](auto Jc, u4 (&ep)[4]) {
      constexpr int J = decltype(Jc)::value;
      static_for<0, 4>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        ep[t] = ds_read16<(32 * J + 8 * t) * 4>(base);
      });
    };
  };
  auto epv = [](const u4* ep, int e) { return __uint_as_float(ep[e >> 2][e & 3]); };

  // ---- every bias once (nothing is in flight yet, so the compiler's vmcnt(0)
  // for these loads drains nothing), then the first hidden phase's weights
  {
    const int nb = (2 + L) * W + D;
    for (int i = tid; i < nb; i += 256) {
      float v;
      if (i < 2 * W) v = P[i];
      else if (i < (2 + L) * W) v = P[off_hidden_w(W, (i - 2 * W) / W + 1) + W * W + (i % W)];
      else v = P[off_final_w(W, L) + W * D + (i - (2 + L) * W)];
      bias[i] = v;
    }
  }
  __syncthreads();
  r32_prefetch(xsm(false, 1), ring, tid);

  // ---- layer 0: SineLayer(1, W, is_first), K = 1 (VALU), in the accumulator layout
  const float x = a.pos[r];
  static_for<0, JW>([&](auto Tc) {
    constexpr int T = decltype(Tc)::value;
    u4 wb[8];        // w0, b0 of the tile's 16 features (inline-asm reads: no vmcnt drain
                     // of the prefetch in flight, as a compiler-visible LDS read would get)
    static_for<0, 4>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      wb[t] = ds_read16<(32 * T + 8 * t) * 4>(bias_lane);
      wb[4 + t] = ds_read16<(W + 32 * T + 8 * t) * 4>(bias_lane);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wb[0]), "+v"(wb[1]), "+v"(wb[2]), "+v"(wb[3]),
                 "+v"(wb[4]), "+v"(wb[5]), "+v"(wb[6]), "+v"(wb[7]));
    float c0[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float z = __fadd_rn(__fmul_rn(x, epv(wb, e)), epv(wb + 4, e));
      float s, co;
      sincos_fast(__fmul_rn(om, z), &s, &co);
      ho[T][e] = s;
      c0[e] = co;
    }
    if (train) {
      static_for<0, 4>([&](auto tc) { tile_store(SHt, Tc, tc, ho[T]); });
      // cos(ωz0) for the layer-0 backward (the 16-row kernel recomputes it
      // there; at one wave per SIMD that phase's k-steps were VALU-bound)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f4 v = {c0[4 * t], c0[4 * t + 1], c0[4 * t + 2], c0[4 * t + 3]};
        cst4(SC + coff + (T * 4 + t) * 256, v);
      }
    }
  });
  R32STAMP(stp, 1);

  // ---- hidden SineLayers 1..L: Zᵀ = Wᵢ·Hᵀ (+b), H = sin(ωZ); each phase
  // prefetches the next (hidden i+1, or the final layer's W_f = matrix L + 1)
  for (int i = 1; i <= L; ++i) {
    float* SHi = SHt + (int64_t)i * WN;
    float* SCi = SC + (int64_t)i * WN + coff;
    float cp[16];
    gemm32<W, JW, TRAIN ? 8 : 0, 0, 4, TRAIN ? 16 : 0, 8>(
        xsm(false, i), xsm(false, i + 1), ring, hb, ho, tid, lane, no_pre,
        bias_epre((uint32_t)((1 + i) * W)),
        [&](auto Jc, auto ec, const auto& ep) {
          constexpr int J = decltype(Jc)::value, e = decltype(ec)::value;
          const float z = __fadd_rn(ho[J][e], epv(ep, e));
          float s, co;
          sincos_fast(__fmul_rn(om, z), &s, &co);
          ho[J][e] = s;
          cp[e] = co;
        },
        done,
        [&](auto Jc, auto tc) {
          constexpr int J = decltype(Jc)::value, t = decltype(tc)::value;
          if (train) {
            const f4 v = {cp[4 * t], cp[4 * t + 1], cp[4 * t + 2], cp[4 * t + 3]};
            cst4(SCi + (J * 4 + t) * 256, v);
            tile_store(SHi, Jc, tc, ho[J]);
          }
        }, sacc);
  }

  // ---- final nn.Linear(W, D): ŷᵀ = W_f·H_Lᵀ + b_f ; MSE ; dL/dŷ
  R32STAMP(stp, 2);
  const float* T = a.tnorm + fit * a.t_stride + (int64_t)r * D + 4 * h;
  // wave-uniform scalar test (no EXEC write near the tile stores)
  const bool has_y = a.y_out != nullptr;
  float* yo = has_y ? a.y_out + fit * a.y_stride + (int64_t)r * D + 4 * h : nullptr;
  float pv[2][16];     // per-lane operands of tiles J (J & 1), loaded a tile ahead
  float yp[16];
  float sq = 0.f;
  gemm32<W, JD, TRAIN ? 4 : 0, TRAIN ? 4 : 0, 4, TRAIN ? 16 : 0, 12>(
      xsm(false, L + 1), train ? xsm(true, L + 1) : nullptr, ring, hb, ho, tid, lane,
      [&](auto Jc) {
        constexpr int J = decltype(Jc)::value;
        if (train) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const f4 v = ld4(T + 32 * J + 8 * t);
#pragma unroll
            for (int q = 0; q < 4; ++q) pv[J & 1][4 * t + q] = v[q];
          }
        }
      },
      bias_epre((uint32_t)((2 + L) * W)),
      [&](auto Jc, auto ec, const auto& ep) {
        constexpr int J = decltype(Jc)::value, e = decltype(ec)::value;
        const float y = __fadd_rn(ho[J][e], epv(ep, e));
        yp[e] = y;
        if (train) {
          const float diff = y - pv[J & 1][e];
          sq = valid ? fmaf(diff, diff, sq) : sq;
          ho[J][e] = valid ? a.grad_scale * diff : 0.f;
        }
      },
      done,
      [&](auto Jc, auto tc) {
        constexpr int J = decltype(Jc)::value, t = decltype(tc)::value;
        if (has_y) {
          const f4 v = {yp[4 * t], yp[4 * t + 1], yp[4 * t + 2], yp[4 * t + 3]};
          st4(yo + 32 * J + 8 * t, v);        // ŷ[r][32J + 8t + 4h + q]
        }
        if (train) tile_store(SGt, Jc, tc, ho[J]);
      }, sacc);
  R32STAMP(stp, 3);
  if (!train) return;
  // loss partials per 16-row block: lanes 0..15 (and their h = 1 partners)
  // hold the wave's first block, lanes 16..31 its second
  sq += __shfl_xor(sq, 32, 64);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) sq += __shfl_xor(sq, o, 64);
  if ((lane & 47) == 0)                          // lanes 0 and 16
    a.loss_partial[fit * a.lp_stride + (int64_t)a.epoch * (n_pad / 16) + blk] = sq;

  // ---- backward: dZ = (dH ⊙ cos(ωz))·ω, stored for the weight gradients
  // (the phase after W_iᵀ is W_{i-1}ᵀ, down to W_1ᵀ = xsm(true, 1), whose
  // phase is layer 0's; NAFTER: the previous phase's last two G or dZ flushes)
  auto bwd = [&](const uint16_t* Mt, const uint16_t* next, auto Kc, int layer) {
    constexpr int K = decltype(Kc)::value;
    const float* SCl = SC + (int64_t)layer * WN + coff;
    float* SZl = SZt + (int64_t)layer * WN;
    gemm32<K, JW, 4, 4, 0, 8, 16>(
        Mt, next, ring, hb, ho, tid, lane,
        [&](auto Jc) {
          constexpr int J = decltype(Jc)::value;
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const f4 v = ld4(SCl + (J * 4 + t) * 256);
#pragma unroll
            for (int q = 0; q < 4; ++q) pv[J & 1][4 * t + q] = v[q];
          }
        },
        no_epre,
        [&](auto Jc, auto ec, const auto&) {
          constexpr int J = decltype(Jc)::value, e = decltype(ec)::value;
          ho[J][e] = __fmul_rn(__fmul_rn(ho[J][e], pv[J & 1][e]), om);
        },
        done, [&](auto Jc, auto tc) { tile_store(SZl, Jc, tc, ho[decltype(Jc)::value]); }, sacc);
  };
  bwd(xsm(true, L + 1), xsm(true, L), ic<D>, L);               // W_fᵀ [W][D]
  R32STAMP(stp, 4);
  for (int i = L; i >= 2; --i) bwd(xsm(true, i), xsm(true, i - 1), ic<W>, i - 1);

  // layer 0: cos(ωz0) from the forward's cos map; dZ0 is only ever summed
  // (dw0 = Σ dZ0·x, db0 = Σ dZ0), so each
  // tile's 16 × 2 per-row values are reduce-scattered over the 16 lanes of a
  // 16-row block (xor 8, 4, 2, 1) and stored as [n_pad/16][2][W] partials:
  // lane c ends with the sums of registers 2(c & 7), 2(c & 7) + 1 — two
  // adjacent features — of Σdz·x (c < 8) or Σdz (c >= 8)
  const int c16 = lane & 15;
  float* PZ = SZ + (int64_t)blk * 2 * W + (c16 >> 3) * W + 4 * h + 8 * ((c16 >> 1) & 3) +
              2 * (c16 & 1);
  const float* SC0 = SC + coff;
  gemm32<W, JW, 1, 4, 0, 8, 24>(
      xsm(true, 1), nullptr, ring, hb, ho, tid, lane,
      [&](auto Jc) {
        constexpr int J = decltype(Jc)::value;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const f4 v = ld4(SC0 + (J * 4 + t) * 256);
#pragma unroll
          for (int q = 0; q < 4; ++q) pv[J & 1][4 * t + q] = v[q];
        }
      },
      no_epre,
      [&](auto Jc, auto ec, const auto&) {
        constexpr int J = decltype(Jc)::value, e = decltype(ec)::value;
        ho[J][e] = __fmul_rn(__fmul_rn(ho[J][e], pv[J & 1][e]), om);
      },
      done,
      [&](auto Jc, auto tc) {
        constexpr int J = decltype(Jc)::value;
        if constexpr (decltype(tc)::value != 0) return;   // the whole tile at t = 0
        float v[32];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          v[e] = __fmul_rn(ho[J][e], x);
          v[16 + e] = ho[J][e];
        }
        const bool b8 = c16 & 8, b4 = c16 & 4, b2 = c16 & 2, b1 = c16 & 1;
        float w16[16], w8[8], w4[4], w2[2];
#pragma unroll
        for (int i = 0; i < 16; ++i)
          w16[i] = (b8 ? v[i + 16] : v[i]) + __shfl_xor(b8 ? v[i] : v[i + 16], 8, 64);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          w8[i] = (b4 ? w16[i + 8] : w16[i]) + __shfl_xor(b4 ? w16[i] : w16[i + 8], 4, 64);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          w4[i] = (b2 ? w8[i + 4] : w8[i]) + __shfl_xor(b2 ? w8[i] : w8[i + 4], 2, 64);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          w2[i] = (b1 ? w4[i + 2] : w4[i]) + __shfl_xor(b1 ? w4[i] : w4[i + 2], 1, 64);
        typedef float f2 __attribute__((ext_vector_type(2)));
        const f2 o2 = {w2[0], w2[1]};
        __builtin_nontemporal_store(o2, reinterpret_cast<f2*>(PZ + 32 * J));
      }, sacc);
  R32STAMP(stp, 5);
#ifdef NERFHIP_STAMPS
  if (stp && (threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 8; q < 32; ++q) stp[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + q] = sacc[q];
#endif
}

#endif  // NERFHIP_VARIANTS (k_step_rows32)

// ---------------------------------------------------------------------------
// Parameter-parallel step: weight/bias gradients reduced over all rows, then
// Adam.  Tiles per fit: L·(W/T)² hidden + (D/TD)(W/T) final + W/64 first.
//
// A tile dW[j0:j0+TJ][k0:k0+TK] = Σ_r dZ[r][j]·H[r][k] streams the two
// operands 16 rows at a time: each 16-row block of a 128-feature slice is one
// contiguous 8 KB run of the row-block-major scratch.  Blocks go global →
// registers (two blocks in flight) → padded LDS (feature stride 20 floats:
// conflict-free ds_read_b128) → v_mfma_f32_32x32x2_f32, whose k index walks
// the 16 rows as 8h+s so each lane reads its 8 rows with two ds_read_b128.
// ---------------------------------------------------------------------------
constexpr int kFs = 20;  // LDS floats per feature per 16-row block (16 + pad)

template <int TJ, int TK, int NW, bool WT = false>
__device__ __forceinline__ void dw_tile(const KArgs& a, const float* __restrict__ A, int FA,
                                        const float* __restrict__ B, int FB, int j0, int k0,
                                        int rb0, int n_blocks, float* G,
                                        float* P, float* M, float* V, float* PT, int64_t pw,
                                        int64_t pb, int64_t ptw, int out_dim, bool do_bias_tile,
                                        float step_size, float bc2s, float* lds) {
  // NW waves as 2 (j) × NW/2 (k); each owns a (TJ/2)×(TK/WK) sub-tile.
  constexpr int NTH = 64 * NW, WK = NW / 2;
  constexpr int NA = TJ / 64, NB = TK / WK / 32;       // 32×32 MFMA tiles per wave
  constexpr int NF4 = (TJ + TK) * 4;                   // f4 per 16-row block
  constexpr int NPT = (NF4 + NTH - 1) / NTH;           // f4 per thread per block
  constexpr int BUF = (TJ + TK) * kFs;
  static_assert(NA >= 1 && NB >= 1, "tile too small for the wave grid");
  static_assert((TJ * 4) % NTH == 0, "A rows must fill whole staging slots");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wj = wave / WK, wk = wave % WK, h = lane >> 5, lr = lane & 31;
  // rows [16·rb0, 16·(rb0+n_blocks)); G != nullptr: write the partial
  // gradient there (split-K) instead of applying Adam
  const int64_t sA = (int64_t)FA * 16, sB = (int64_t)FB * 16;
  const float* Ab = A + (int64_t)j0 * 16 + rb0 * sA;
  const float* Bb = B + (int64_t)k0 * 16 + rb0 * sB;

  auto gload = [&](f4 (&st)[NPT], int rb) {
#pragma unroll
    for (int m = 0; m < NPT; ++m) {
      const int i = tid + NTH * m;      // m < TJ*4/NTH reads A, the rest B: uniform per m
      const int sl = stage_slot<false>(i);
      if (m < TJ * 4 / NTH)
        st[m] = ld4(Ab + rb * sA + sl * 4);
      else if (NF4 % NTH == 0 || i < NF4)
        st[m] = ld4(Bb + rb * sB + (sl - TJ * 4) * 4);
    }
  };
  auto lstore = [&](const f4 (&st)[NPT], float* buf) {
#pragma unroll
    for (int m = 0; m < NPT; ++m) {
      const int i = tid + NTH * m;
      const int sl = stage_slot<false>(i);   // feature sl/4, quarter sl%4 (A then B)
      if (NF4 % NTH == 0 || i < NF4) st4(buf + (sl >> 2) * kFs + (sl & 3) * 4, st[m]);
    }
  };

  f16v acc[NA][NB];
#pragma unroll
  for (int x = 0; x < NA; ++x)
#pragma unroll
    for (int y = 0; y < NB; ++y)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[x][y][q] = 0.f;
  float bsum[NA];
#pragma unroll
  for (int x = 0; x < NA; ++x) bsum[x] = 0.f;
  const bool do_bias = do_bias_tile && wk == 0;

  // n_blocks is even (nerfhip_group_sizes picks the split).  Prefetches past the end re-read
  // the last block instead of branching: a conditional load makes the waitcnt
  // pass assume the worst at the join and drain the fresh prefetch each block.
  f4 st0[NPT], st1[NPT];
  gload(st0, 0);
  lstore(st0, lds);
  gload(st1, 1);
  __syncthreads();
  const float* a_base = lds + (wj * (TJ / 2) + lr) * kFs + 8 * h;
  const float* b_base = lds + (TJ + wk * (TK / WK) + lr) * kFs + 8 * h;

  auto block = [&](int rb, f4 (&st_next)[NPT], f4 (&st_fill)[NPT]) {
    // st_next ← block rb+2 ; compute block rb ; LDS[(rb+1)&1] ← st_fill (block rb+1)
    gload(st_next, rb + 2 < n_blocks ? rb + 2 : n_blocks - 1);
    __builtin_amdgcn_sched_barrier(0);   // loads at the top (as in dw_tile_x3)
    const int off = (rb & 1) * BUF;
    f4 av[NA][2], bv[NB][2];
#pragma unroll
    for (int x = 0; x < NA; ++x) {
      av[x][0] = ld4(a_base + off + x * 32 * kFs);
      av[x][1] = ld4(a_base + off + x * 32 * kFs + 4);
    }
#pragma unroll
    for (int y = 0; y < NB; ++y) {
      bv[y][0] = ld4(b_base + off + y * 32 * kFs);
      bv[y][1] = ld4(b_base + off + y * 32 * kFs + 4);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int x = 0; x < NA; ++x)
#pragma unroll
        for (int y = 0; y < NB; ++y)
          acc[x][y] = mfma32(av[x][s >> 2][s & 3], bv[y][s >> 2][s & 3], acc[x][y]);
    if (do_bias) {
#pragma unroll
      for (int x = 0; x < NA; ++x)
        bsum[x] += ((av[x][0][0] + av[x][0][1]) + (av[x][0][2] + av[x][0][3])) +
                   ((av[x][1][0] + av[x][1][1]) + (av[x][1][2] + av[x][1][3]));
    }
    lstore(st_fill, lds + ((rb + 1) & 1) * BUF);   // last block: an unread buffer
    __syncthreads();
  };
  for (int rb = 0; rb < n_blocks; rb += 2) {
    block(rb, st0, st1);
    block(rb + 1, st1, st0);
  }

  // Adam on the wave's (TJ/2)×(TK/WK) part; lane holds rows (q&3)+8(q>>2)+4h, col lr.
  // Streamed as in dw_tile_x3: the P/M/V loads of the next half sub-tile are
  // issued before the current one's Adam and stores.
  if (G) {
#pragma unroll
    for (int x = 0; x < NA; ++x)
#pragma unroll
      for (int y = 0; y < NB; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int j = j0 + wj * (TJ / 2) + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * h;
          const int kcol = k0 + wk * (TK / WK) + 32 * y + lr;
          slab_store<WT>(G + pw + (int64_t)j * a.W + kcol, acc[x][y][e]);
        }
  } else {
    constexpr int NS = NA * NB;
    const int64_t nbytes = (int64_t)out_dim * a.W * 4;
    const __amdgpu_buffer_rsrc_t rp = rsrc_over(P + pw, nbytes), rm = rsrc_over(M + pw, nbytes),
                                 rv = rsrc_over(V + pw, nbytes);
    const uint32_t lb =
        (uint32_t)(((j0 + wj * (TJ / 2) + 4 * h) * a.W + k0 + wk * (TK / WK) + lr) * 4);
    auto eoff = [&](int sub, int e) {
      return lb + (uint32_t)(((32 * (sub / NB) + 8 * (e >> 2) + (e & 3)) * a.W + 32 * (sub % NB)) * 4);
    };
    float pq[2][8], mq[2][8], vq[2][8];
    auto fetch = [&](int c, int buf) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t o = eoff(c >> 1, 8 * (c & 1) + e);
        pq[buf][e] = bload_f32(rp, o);
        mq[buf][e] = bload_f32(rm, o);
        vq[buf][e] = bload_f32(rv, o);
      }
    };
    fetch(0, 0);
#pragma unroll
    for (int c = 0; c < 2 * NS; ++c) {
      const int buf = c & 1, sub = c >> 1, x = sub / NB, y = sub % NB;
      if (c + 1 < 2 * NS) fetch(c + 1, buf ^ 1);
      const int jrow0 = j0 + wj * (TJ / 2) + 32 * x;
      const int kcol = k0 + wk * (TK / WK) + 32 * y + lr;
#pragma unroll
      for (int qb = 2 * (c & 1); qb < 2 * (c & 1) + 2; ++qb) {
        f4 pt;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int e = qb * 4 + qq;
          const uint32_t o = eoff(sub, e);
          float p = pq[buf][e & 7], mm = mq[buf][e & 7], vv = vq[buf][e & 7];
          adam_update(p, mm, vv, acc[x][y][e], step_size, bc2s);
          bstore_f32(rp, o, p);
          bstore_f32(rm, o, mm);
          bstore_f32(rv, o, vv);
          pt[qq] = p;
        }
        st4(PT + ptw + (int64_t)kcol * out_dim + jrow0 + 8 * qb + 4 * h, pt);
      }
    }
  }
  if (do_bias) {
#pragma unroll
    for (int x = 0; x < NA; ++x) {
      const float s = bsum[x] + __shfl_xor(bsum[x], 32, 64);
      if (h == 0) {
        const int64_t idx = pb + j0 + wj * (TJ / 2) + 32 * x + lr;
        if (G) {
          slab_store<WT>(G + idx, s);
          continue;
        }
        float p = P[idx], mm = M[idx], vv = V[idx];
        adam_update(p, mm, vv, s, step_size, bc2s);
        P[idx] = p; M[idx] = mm; V[idx] = vv;
      }
    }
  }
}

// bf16x3 form of dw_tile.  Each staged f4 (feature s/4, rows 4(s%4)..+3 of a
// 16-row block, s = stage_slot(i)) is split once, at the LDS store, into three
// bf16 planes [3][TJ+TK features][kFx] (48-B feature stride: every
// ds_read_b128 lane group covers a bank row once, and with stage_slot's lane
// order every 16-lane ds_write_b64 group too; a layout change that freed both,
// 32-B features plus 16 B of pad per 16, measured 8-10 % slower in round 2:
// more LDS bytes per block); a lane then reads its 8 rows of a feature
// as one 16-B slice per plane, and each (x, y) sub-tile takes six
// v_mfma_f32_32x32x16_bf16 per 16-row block (hi and correction accumulators)
// instead of eight v_mfma_f32_32x32x2_f32.  Bias sums come from the fp32
// staging registers.  The Adam epilogue writes P/M/V and, instead of the
// transposed fp32 copy, both split copies of the weights for the row kernel.
constexpr int kFx = 24;
#ifndef NERFHIP_PARAMS_VPG
#define NERFHIP_PARAMS_VPG 6
#endif
constexpr int kParamsVpg = NERFHIP_PARAMS_VPG;   // VALU per MFMA in dw_tile_x3's block schedule

template <int TJ, int TK, int NW, int WW, int OD, int KSX, bool WT = false>
__device__ __forceinline__ void dw_tile_x3(const KArgs& a, const float* __restrict__ A, int FA,
                                           const float* __restrict__ B, int FB, int j0, int k0,
                                           int rb0, int n_blocks, float* G, float* P, float* M,
                                           float* V, uint16_t* XS, int64_t pw, int64_t pb,
                                           int64_t xf, int64_t xb, int out_dim,
                                           bool do_bias_tile, float step_size, float bc2s,
                                           float* lds_f) {
  constexpr int NTH = 64 * NW, WK = NW / 2;
  constexpr int NA = TJ / 64, NB = TK / WK / 32;
  constexpr int NF4 = (TJ + TK) * 4, NPT = (NF4 + NTH - 1) / NTH;
  constexpr int NA4 = TJ * 4, NPA = (NA4 + NTH - 1) / NTH;   // A's f4 / rounds holding A
  constexpr int PLX = (TJ + TK) * kFx, BUFX = 3 * PLX;
  static_assert(NA >= 1 && NB >= 1 && NPA >= 1, "tile too small for the wave grid");
  uint16_t* lds = reinterpret_cast<uint16_t*>(lds_f);
  // W and out_dim at compile time (the kernel's template W, and W or D):
  // the xoff() split-copy addresses fold to shifts and masks instead of
  // runtime integer divisions in the Adam epilogue (parameter kernel −0.8 %,
  // 200-epoch sweep +0.5 %, profiles/r02/ab_params_ct_width.log)
  constexpr int W = WW, kOD = OD;
  // KSX: the layout of the split copies (kLayX / kLayKs / kLay32, the
  // group's row kernel's).  Compile-time: a runtime layout select here put the epilogue's
  // staging arrays in scratch (576 B/lane) and made the W = 512 parameter
  // kernel 7x slower.
  (void)a;
  (void)out_dim;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wj = wave / WK, wk = wave % WK, h = lane >> 5, lr = lane & 31;
  const int64_t sA = (int64_t)FA * 16, sB = (int64_t)FB * 16;
  const float* Ab = A + (int64_t)j0 * 16 + rb0 * sA;
  const float* Bb = B + (int64_t)k0 * 16 + rb0 * sB;
  float bpart[NPA];
#pragma unroll
  for (int m = 0; m < NPA; ++m) bpart[m] = 0.f;

  static_assert(NA4 % 64 == 0, "A rows must fill whole waves (stage_slot permutes within 64)");
  auto gload = [&](f4 (&st)[NPT], int rb) {
#ifdef NERFHIP_EXP_HOTBLOCK   // diagnostic timing build, WRONG numerics: every block re-reads block 0/1
    rb &= 1;
#endif
#pragma unroll
    for (int m = 0; m < NPT; ++m) {
      const int i = tid + NTH * m;
      const int so = stage_slot<true>(i);
      if (NA4 % NTH == 0 ? m < NPA : i < NA4)   // wave-uniform (NA4 % 64 == 0)
        st[m] = ld4(Ab + rb * sA + so * 4);
      else if (NF4 % NTH == 0 || i < NF4)
        st[m] = ld4(Bb + rb * sB + (so - TJ * 4) * 4);
    }
  };
  auto lstore = [&](const f4 (&st)[NPT], uint16_t* buf, bool count) {
#pragma unroll
    for (int m = 0; m < NPT; ++m) {
      const int i = tid + NTH * m;
      if (NF4 % NTH == 0 || i < NF4) {
        const f4 v = st[m];
        uint32_t sh[4], sm[4], sl[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) split3(v[s], sh[s], sm[s], sl[s]);
        const int so = stage_slot<true>(i);
        uint16_t* d = buf + (so >> 2) * kFx + (so & 3) * 4;
        const u2 vh = {pk_top(sh[0], sh[1]), pk_top(sh[2], sh[3])};
        const u2 vm = {pk_top(sm[0], sm[1]), pk_top(sm[2], sm[3])};
        const u2 vl = {pk_top(sl[0], sl[1]), pk_top(sl[2], sl[3])};
        *reinterpret_cast<u2*>(d) = vh;
        *reinterpret_cast<u2*>(d + PLX) = vm;
#if NERFHIP_X2P(16)
        (void)vl;
#else
        *reinterpret_cast<u2*>(d + 2 * PLX) = vl;
#endif
        if (m < NPA && i < NA4 && count) bpart[m] += (v[0] + v[1]) + (v[2] + v[3]);
      }
    }
  };

  f16v hi[NA][NB], lo[NA][NB];
#pragma unroll
  for (int x = 0; x < NA; ++x)
#pragma unroll
    for (int y = 0; y < NB; ++y)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        hi[x][y][q] = 0.f;
        lo[x][y][q] = 0.f;
      }

  const uint16_t* a_base = lds + (wj * (TJ / 2) + lr) * kFx + 8 * h;
  const uint16_t* b_base = lds + (TJ + wk * (TK / WK) + lr) * kFx + 8 * h;
  auto rd = [&](const uint16_t* q) {
    S8 r;
    r.h = *reinterpret_cast<const u4*>(q);
    r.m = *reinterpret_cast<const u4*>(q + PLX);
#if NERFHIP_X2P(16)
    r.l = r.m;
#else
    r.l = *reinterpret_cast<const u4*>(q + 2 * PLX);
#endif
    return r;
  };

  auto mfma_block = [&](int rb) {
    const int off = (rb & 1) * BUFX;
    S8 av[NA], bv[NB];
#pragma unroll
    for (int x = 0; x < NA; ++x) av[x] = rd(a_base + off + x * 32 * kFx);
#pragma unroll
    for (int y = 0; y < NB; ++y) bv[y] = rd(b_base + off + y * 32 * kFx);
#pragma unroll
    for (int x = 0; x < NA; ++x)
#pragma unroll
      for (int y = 0; y < NB; ++y) mfma32x3(av[x], bv[y], hi[x][y], lo[x][y]);
    // (measured slower, each 7-14 %: one accumulator per sub-tile; product-major
    // issue order across sub-tiles; operands loaded straight to registers
    // without LDS; a conflict-free LDS layout — this order and staging stay)
  };
  // stream the blocks: two in flight in registers, one in each LDS buffer.
  // (Issuing every block's loads up front for split-K slices of 8 blocks —
  // config 2's 224-workgroup grid — was bitwise equal and no faster: 20.7 vs
  // 19.4 µs; its diagnostic stamps put the time in the prologue's dependent
  // scalar loads, ≈3.3 µs, and the partial-slab stores, ≈6.5 µs, not in the
  // block loads, profiles/r03/params_split_stamps.log)
  f4 st0[NPT], st1[NPT];
  gload(st0, 0);
  PSTAMP(1);
  lstore(st0, lds, true);
  gload(st1, 1);
  __syncthreads();
  PSTAMP(2);
#ifdef NERFHIP_STAMPS
  // slot 7: clock cycles (s_memtime) this wave spent from each block's last
  // MFMA/split issue to leaving its barrier, summed (low 32 bits), and the
  // whole block loop (high 32 bits)
  uint64_t bwait = 0;
  const uint64_t tloop = __builtin_amdgcn_s_memtime();
#endif
  auto block = [&](int rb, f4 (&st_next)[NPT], f4 (&st_fill)[NPT]) {
    // st_next ← block rb+2 ; compute block rb ; LDS[(rb+1)&1] ← st_fill (block rb+1)
    gload(st_next, rb + 2 < n_blocks ? rb + 2 : n_blocks - 1);
    // the block loads stay at the top: left free, the scheduler sank them to
    // just before the barrier, and the next block's split (interleaved with
    // its MFMAs) then waited on them at once — a full load latency exposed
    // per block instead of hidden behind one block of MFMAs
    __builtin_amdgcn_sched_barrier(0);
#ifdef NERFHIP_EXP_PARAMS_PRIO   // diagnostic: raised wave priority over the MFMA section
    __builtin_amdgcn_s_setprio(NERFHIP_EXP_PARAMS_PRIO);
#endif
    mfma_block(rb);
#ifdef NERFHIP_EXP_SPLIT_AFTER_MFMA   // diagnostic: no interleaving of the split with the MFMAs
    __builtin_amdgcn_sched_barrier(0);
#endif
    lstore(st_fill, lds + ((rb + 1) & 1) * BUFX, rb + 1 < n_blocks);   // last: unread buffer
    // An even interleave of the split with the MFMAs (sched_group_barrier):
    // the fragment reads first, then per MFMA kParamsVpg VALU and every other
    // MFMA one LDS store.  Deep × 40 isolated: 6 per MFMA 0.320 ms against
    // 0.331 for the compiler's own order (3: 0.336, 4: 0.327, 8: 0.325,
    // 12: 0.331; tools/sessions/r6/s6_27.sh, s6_28.sh).  Bitwise equal.
    __builtin_amdgcn_sched_group_barrier(0x100, 3 * (NA + NB), 0);
#pragma unroll
    for (int i = 0; i < 6 * NA * NB; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, kParamsVpg, 0);
      if (i & 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    }
#ifdef NERFHIP_EXP_PARAMS_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
#ifdef NERFHIP_STAMPS
    const uint64_t tb = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#ifdef NERFHIP_STAMPS
    bwait += __builtin_amdgcn_s_memtime() - tb;
#endif
  };
  for (int rb = 0; rb < n_blocks; rb += 2) {
    block(rb, st0, st1);
    block(rb + 1, st1, st0);
  }
  PSTAMP(3);
#ifdef NERFHIP_STAMPS
  if (a.pstamps && (threadIdx.x & 63) == 0)
    a.pstamps[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + 7] =
        (bwait & 0xffffffffull) | ((__builtin_amdgcn_s_memtime() - tloop) << 32);
#endif

  // Adam on the wave's (TJ/2)×(TK/WK) part; lane holds rows (q&3)+8(q>>2)+4h, col lr.
  // The gradient is hi + lo.  The epilogue streams the (x, y) sub-tiles: the
  // P/M/V loads of sub-tile s + 1 are issued before sub-tile s's Adam and
  // stores, so a wave waits on one memory round trip per sub-tile instead of
  // one per parameter (in-order vmcnt: a load issued after a store cannot be
  // waited on without that store's acknowledgement too).  Buffer loads and
  // stores over the layer's weights with one lane offset: no per-element
  // 64-bit address arithmetic.  Arithmetic and its order are unchanged.
#pragma unroll
  for (int x = 0; x < NA; ++x)
#pragma unroll
    for (int y = 0; y < NB; ++y)
#pragma unroll
      for (int q = 0; q < 16; ++q) hi[x][y][q] += lo[x][y][q];
  if (G) {
#pragma unroll
    for (int x = 0; x < NA; ++x)
#pragma unroll
      for (int y = 0; y < NB; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int j = j0 + wj * (TJ / 2) + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * h;
          const int kcol = k0 + wk * (TK / WK) + 32 * y + lr;
          slab_store<WT>(G + pw + (int64_t)j * W + kcol, hi[x][y][e]);
        }
  } else {
    constexpr int NS = NA * NB;
    constexpr int64_t kBytes = (int64_t)kOD * W * 4;
    const __amdgpu_buffer_rsrc_t rp = rsrc_over(P + pw, kBytes), rm = rsrc_over(M + pw, kBytes),
                                 rv = rsrc_over(V + pw, kBytes);
    const uint32_t lb =
        (uint32_t)(((j0 + wj * (TJ / 2) + 4 * h) * W + k0 + wk * (TK / WK) + lr) * 4);
    auto eoff = [&](int sub, int e) {
      return lb + (uint32_t)(((32 * (sub / NB) + 8 * (e >> 2) + (e & 3)) * W + 32 * (sub % NB)) * 4);
    };
    // half sub-tiles (8 parameters per lane) per round trip, double-buffered
    float pq[2][8], mq[2][8], vq[2][8];
    auto fetch = [&](int c, int buf) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t o = eoff(c >> 1, 8 * (c & 1) + e);
        pq[buf][e] = bload_f32(rp, o);
        mq[buf][e] = bload_f32(rm, o);
        vq[buf][e] = bload_f32(rv, o);
      }
    };
    fetch(0, 0);
#pragma unroll
    for (int c = 0; c < 2 * NS; ++c) {
      const int buf = c & 1, sub = c >> 1, x = sub / NB, y = sub % NB;
      if (c + 1 < 2 * NS) fetch(c + 1, buf ^ 1);
      const int jrow0 = j0 + wj * (TJ / 2) + 32 * x;
      const int kcol = k0 + wk * (TK / WK) + 32 * y + lr;
#pragma unroll
      for (int qb = 2 * (c & 1); qb < 2 * (c & 1) + 2; ++qb) {
        uint32_t th[4], tm[4], tl[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int e = qb * 4 + qq, j = jrow0 + qq + 8 * qb + 4 * h;
          const uint32_t o = eoff(sub, e);
          float p = pq[buf][e & 7], mm = mq[buf][e & 7], vv = vq[buf][e & 7];
          adam_update(p, mm, vv, hi[x][y][e], step_size, bc2s);
          bstore_f32(rp, o, p);
          bstore_f32(rm, o, mm);
          bstore_f32(rv, o, vv);
          split3(p, th[qq], tm[qq], tl[qq]);
#ifndef NERFHIP_EXP_NO_FWDCOPY   // diagnostic build only: timing of the copy's stores
          // forward copy M[j][kcol] of [out_dim][W]
          XS[xf + xoff_any(KSX, kOD, W, j, kcol, 0)] = (uint16_t)(th[qq] >> 16);
          XS[xf + xoff_any(KSX, kOD, W, j, kcol, 1)] = (uint16_t)(tm[qq] >> 16);
          XS[xf + xoff_any(KSX, kOD, W, j, kcol, 2)] = (uint16_t)(tl[qq] >> 16);
#endif
        }
        // transposed copy: Mᵀ[kcol][j..j+3] is one 8-B run per plane
        const int jb = jrow0 + 8 * qb + 4 * h;
        const u2 vh = {pk_top(th[0], th[1]), pk_top(th[2], th[3])};
        const u2 vm = {pk_top(tm[0], tm[1]), pk_top(tm[2], tm[3])};
        const u2 vl = {pk_top(tl[0], tl[1]), pk_top(tl[2], tl[3])};
        *reinterpret_cast<u2*>(XS + xb + xoff_any(KSX, W, kOD, kcol, jb, 0)) = vh;
        *reinterpret_cast<u2*>(XS + xb + xoff_any(KSX, W, kOD, kcol, jb, 1)) = vm;
        *reinterpret_cast<u2*>(XS + xb + xoff_any(KSX, W, kOD, kcol, jb, 2)) = vl;
      }
    }
  }
  if (do_bias_tile) {
#pragma unroll
    for (int m = 0; m < NPA; ++m) {
      float s = bpart[m];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      if ((tid & 3) == 0 && tid + NTH * m < NA4) {
        const int64_t idx = pb + j0 + (stage_slot<true>(tid + NTH * m) >> 2);
        if (G) {
          slab_store<WT>(G + idx, s);
        } else {
          float p = P[idx], mm = M[idx], vv = V[idx];
          adam_update(p, mm, vv, s, step_size, bc2s);
          P[idx] = p; M[idx] = mm; V[idx] = vv;
        }
      }
    }
  }
  PSTAMP(4);
}

#ifdef NERFHIP_VARIANTS
// Fused split-K reduction (KArgs.split_fused): the slices of one parameter
// tile arrive in any order; each publishes its partial slab (release fence,
// then one agent-scope atomic add on the tile's counter) and the last to
// arrive (acquire) sums the n_split slabs of the tile in slice order —
// exactly k_adam_split's order, so the result is bitwise the same — runs Adam
// and writes the weight copies.
// NS slices compile-time: every slice's load of a 4-parameter batch in flight.
template <int NS, int W, int D, bool X3>
__device__ __forceinline__ void split_finish_run(const KArgs& a, int fit, int L, int64_t pw,
                                                 int rows, int cols, int j0, int k0, int layer,
                                                 int nbias, int64_t pb) {
  const int tid = threadIdx.x, nth = blockDim.x;
  const float* g = a.gpart + fit * a.gp_stride;
  float* P = a.params + fit * a.p_stride;
  float* M = a.m + fit * a.p_stride;
  float* V = a.v + fit * a.p_stride;
  float* PT = a.params_t + fit * a.pt_stride;
  uint16_t* XS = X3 ? a.wsplit + fit * a.ws_stride : nullptr;
  const float step_size = a.sched[2 * a.epoch], bc2s = a.sched[2 * a.epoch + 1];
  const int lay = wlayout(a);
  const int64_t ps = a.p_stride;
  // biases first, their loads in flight beside the first weight batch (a
  // clamped index, not a branch around the loads)
  const bool hb = tid < nbias;
  const int64_t ib = pb + (hb ? tid : 0);
  float bg[NS];
#pragma unroll
  for (int sp = 0; sp < NS; ++sp) bg[sp] = g[sp * ps + ib];
  float bp = P[ib], bm = M[ib], bv = V[ib];
  // weights as 16-B runs along k (cols is a multiple of 64, every run aligned):
  // a thread's whole batch — B runs × NS slabs, and P/M/V — is loaded before
  // any is used, so a batch costs one dependent round trip
  const int n4 = rows * cols / 4;
  constexpr int B = 16 / NS > 0 ? 16 / NS : 1;   // <= 16 slab runs (64 floats) in flight
  for (int q0 = tid; q0 < n4; q0 += B * nth) {
    f4 gv[B][NS], pv[B], mv[B], vv[B];
    int64_t ix[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const int q = q0 + b * nth < n4 ? q0 + b * nth : q0;
      const int e = 4 * q;
      ix[b] = pw + (int64_t)(j0 + e / cols) * W + k0 + e % cols;
#pragma unroll
      for (int sp = 0; sp < NS; ++sp) gv[b][sp] = *reinterpret_cast<const f4*>(g + sp * ps + ix[b]);
      pv[b] = *reinterpret_cast<const f4*>(P + ix[b]);
      mv[b] = *reinterpret_cast<const f4*>(M + ix[b]);
      vv[b] = *reinterpret_cast<const f4*>(V + ix[b]);
    }
    if (q0 == tid && hb) {
      float gs = bg[0];
#pragma unroll
      for (int sp = 1; sp < NS; ++sp) gs += bg[sp];   // slice order
      adam_update(bp, bm, bv, gs, step_size, bc2s);
      P[ib] = bp; M[ib] = bm; V[ib] = bv;
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
      if (q0 + b * nth >= n4) break;
      const int e = 4 * (q0 + b * nth);
      const int j = j0 + e / cols, k = k0 + e % cols;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float gs = gv[b][0][c];
#pragma unroll
        for (int sp = 1; sp < NS; ++sp) gs += gv[b][sp][c];   // slice order
        float p = pv[b][c], mm = mv[b][c], v2 = vv[b][c];
        adam_update(p, mm, v2, gs, step_size, bc2s);
        pv[b][c] = p; mv[b][c] = mm; vv[b][c] = v2;
      }
      *reinterpret_cast<f4*>(P + ix[b]) = pv[b];
      *reinterpret_cast<f4*>(M + ix[b]) = mv[b];
      *reinterpret_cast<f4*>(V + ix[b]) = vv[b];
      if (layer > 0) {
        const float p4[4] = {pv[b][0], pv[b][1], pv[b][2], pv[b][3]};
        if constexpr (X3) {
          // the layout as a compile-time constant per branch (a run-time
          // select inside the unrolled copies spills them to scratch)
          auto copies = [&](auto lay_c) {
#pragma unroll
            for (int c = 0; c < 4; ++c) put_w(XS, decltype(lay_c)::value, W, D, L, layer, j, k + c, p4[c]);
          };
          if (lay == kLayKs) copies(std::integral_constant<int, kLayKs>{});
          else if (lay == kLay32) copies(std::integral_constant<int, kLay32>{});
          else copies(std::integral_constant<int, kLayX>{});
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (layer <= L) PT[(int64_t)(layer - 1) * W * W + (int64_t)(k + c) * W + j] = p4[c];
            else PT[(int64_t)L * W * W + (int64_t)(k + c) * D + j] = p4[c];
          }
        }
      }
    }
  }
  if (tid >= n4 && hb) {   // (only if some bias thread had no weight batch)
    float gs = bg[0];
#pragma unroll
    for (int sp = 1; sp < NS; ++sp) gs += bg[sp];
    adam_update(bp, bm, bv, gs, step_size, bc2s);
    P[ib] = bp; M[ib] = bm; V[ib] = bv;
  }
}

// Arrival + (if last) the tile's reduction.  Tile t of ParamsCfg C: hidden
// layer tiles, then the final layer's, then the first layer's (k_step_params).
// The hand-off is cdna_hip_programming.md's in-launch split-K recipe in its
// write-through form: the slabs were stored sc1 (slab_store), every wave
// drains them (vmcnt 0), then one lane draws a ticket from the tile's
// monotonic counter (agent-scope relaxed add, no release fence needed), and
// the reducer's lane acquires (this CU's L1 invalidated) before any wave
// reads a slab.  Under the HIP/C++ memory model a relaxed ticket after relaxed
// stores is NOT a happens-before edge: correctness rests on gfx950's sc1
// write-through stores having reached the agent-coherent L2 once vmcnt has
// drained — an ISA-level argument, one reason this path stays an opt-in
// variant (a default would take a release RMW on the ticket).  The "I am last" word lives in the block's one LDS array (a second
// __shared__ object can de-pipeline the staging loop).
template <class C, int W, int D, bool X3>
__device__ void split_finish(const KArgs& a, int fit, int L, int t, float* lds) {
  int* flag = reinterpret_cast<int*>(lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // every wave's stores drained; the staging array is free
  if (threadIdx.x == 0) {
    // the counter only grows (zeroed by the prologue): epoch e's last
    // arrival is the one that brings it to (e + 1) · n_split
    int* ctr = reinterpret_cast<int*>(a.gpart + fit * a.gp_stride + a.ctr_off) + t;
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (old + 1) % a.n_split == 0;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  // weights: rows × cols at pw + (j0 + r)·W + k0 + c; biases: nbias at pb
  int64_t pw, pb;
  int rows, cols, j0, k0, layer, nbias;
  if (t < L * C::TH) {
    const int u = t % C::TH;
    layer = t / C::TH + 1;
    pw = off_hidden_w(W, layer);
    rows = C::T; cols = C::TK; j0 = (u / C::NTK) * C::T; k0 = (u % C::NTK) * C::TK;
    pb = pw + (int64_t)W * W + j0;
    nbias = (u % C::NTK) == 0 ? rows : 0;
  } else if (t < L * C::TH + C::TF) {
    const int u = t - L * C::TH;
    layer = L + 1;
    pw = off_final_w(W, L);
    rows = C::TD; cols = C::TK; j0 = (u / C::NTK) * C::TD; k0 = (u % C::NTK) * C::TK;
    pb = pw + (int64_t)W * D + j0;
    nbias = (u % C::NTK) == 0 ? rows : 0;
  } else {
    // first layer, features f0 .. f0 + 16·NW: w0[f] at f, b0[f] at W + f
    const int f0 = (t - L * C::TH - C::TF) * (16 * C::NW);
    layer = 0;
    pw = 0; rows = 1; cols = 16 * C::NW; j0 = 0; k0 = f0;
    pb = W + f0;
    nbias = 16 * C::NW;
  }
  switch (a.n_split) {
    case 2: split_finish_run<2, W, D, X3>(a, fit, L, pw, rows, cols, j0, k0, layer, nbias, pb); break;
    case 4: split_finish_run<4, W, D, X3>(a, fit, L, pw, rows, cols, j0, k0, layer, nbias, pb); break;
    case 8: split_finish_run<8, W, D, X3>(a, fit, L, pw, rows, cols, j0, k0, layer, nbias, pb); break;
    default: split_finish_run<16, W, D, X3>(a, fit, L, pw, rows, cols, j0, k0, layer, nbias, pb); break;
  }
}

#endif  // NERFHIP_VARIANTS (split_finish)

// SK: the fused split-K instantiation (NERFHIP_SPLIT_FUSED=1: write-through
// slabs and the in-kernel reduction).  Every other launch — unsplit, or
// split-K with the k_adam_split pass — runs SK = false, whose slab path is
// the run-time `G` test alone.
template <int W, int D, bool X3, bool SMALL = false, int KSX = kLayX, bool SK = false>
__global__ void __launch_bounds__((ParamsCfg<W, D, X3, SMALL>::THREADS),
                                  (ParamsCfg<W, D, X3, SMALL>::MINB))
    k_step_params(KArgs a) {
  FLIGHT_ENTER();
  using C = ParamsCfg<W, D, X3, SMALL>;
  constexpr int LDS_F = X3 ? 2 * 3 * (C::T + C::TK) * kFx / 2 : 2 * (2 * C::T) * kFs;
  __shared__ __attribute__((aligned(16))) float lds[LDS_F];
  int fit, t;
  const int nt = C::tiles(a.L_max);
  PSTAMP(0);
  PSTAMP_HW();
  if (!map_block(blockIdx.x, a.n_fits, nt * a.n_split, fit, t)) return;
  const int split = t / nt;
  t -= split * nt;
  const int L = fit_layers_of(a, fit);
  FLIGHT_DEPTH(L, fit);
  if (t >= C::tiles(L)) return;
  const int nb = a.n_pad / 16 / a.n_split, rb0 = split * nb;
  // (the unsplit kernel keeps the run-time test: with G a compile-time null
  // the compiler schedules the Adam epilogue differently and spills, 100-132
  // B per lane at W = 256 bf16x3)
  float* G = SK || a.n_split > 1 ? a.gpart + fit * a.gp_stride + split * a.p_stride : nullptr;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n_pad = a.n_pad;
  const float step_size = a.sched[2 * a.epoch], bc2s = a.sched[2 * a.epoch + 1];

  float* P = a.params + fit * a.p_stride;
  float* PT = a.params_t + fit * a.pt_stride;
  float* M = a.m + fit * a.p_stride;
  float* V = a.v + fit * a.p_stride;
  const float* S = a.scratch + fit * a.s_stride;
  const int64_t WN = (int64_t)W * n_pad;
  const float* SH = S;
  const float* SZ = S + (int64_t)(a.L_max + 1) * WN;
  const float* SG = S + 2 * (int64_t)(a.L_max + 1) * WN;

  uint16_t* XS = X3 ? a.wsplit + fit * a.ws_stride : nullptr;
  if (t < L * C::TH) {
    const int layer = t / C::TH + 1, u = t % C::TH;
    const int64_t pw = off_hidden_w(W, layer);
    if constexpr (X3)
      dw_tile_x3<C::T, C::TK, C::NW, W, W, KSX, SK>(a, SZ + (int64_t)layer * WN, W,
                                     SH + (int64_t)(layer - 1) * WN, W, (u / C::NTK) * C::T,
                                     (u % C::NTK) * C::TK, rb0, nb, G, P, M, V, XS, pw,
                                     pw + (int64_t)W * W, xs_mat(W, D, L, false, layer),
                                     xs_mat(W, D, L, true, layer), W, (u % C::NTK) == 0,
                                     step_size, bc2s, lds);
    else
      dw_tile<C::T, C::T, C::NW, SK>(a, SZ + (int64_t)layer * WN, W, SH + (int64_t)(layer - 1) * WN,
                                 W, (u / C::NTK) * C::T, (u % C::NTK) * C::T, rb0, nb, G, P, M, V,
                                 PT, pw, pw + (int64_t)W * W, (int64_t)(layer - 1) * W * W, W,
                                 (u % C::NTK) == 0, step_size, bc2s, lds);
  } else if (t < L * C::TH + C::TF) {
    const int u = t - L * C::TH;
    const int64_t pw = off_final_w(W, L);
    if constexpr (X3)
      dw_tile_x3<C::TD, C::TK, C::NW, W, D, KSX, SK>(a, SG, D, SH + (int64_t)L * WN, W, (u / C::NTK) * C::TD,
                                      (u % C::NTK) * C::TK, rb0, nb, G, P, M, V, XS, pw,
                                      pw + (int64_t)W * D, xs_mat(W, D, L, false, L + 1),
                                      xs_mat(W, D, L, true, L + 1), D, (u % C::NTK) == 0,
                                      step_size, bc2s, lds);
    else
      dw_tile<C::TD, C::T, C::NW, SK>(a, SG, D, SH + (int64_t)L * WN, W, (u / C::NTK) * C::TD,
                                  (u % C::NTK) * C::T, rb0, nb, G, P, M, V, PT, pw,
                                  pw + (int64_t)W * D, (int64_t)L * W * W, D, (u % C::NTK) == 0,
                                  step_size, bc2s, lds);
  } else {
    // first SineLayer(1, W): dw0 = dZ0ᵀ·x, db0 = Σ_rows dZ0.  Lane = (feature
    // f = lane/4 of the wave's 16, m = lane%4: every 4th 16-row block).
    const int u = t - L * C::TH - C::TF;
    const int f = lane >> 2, m = lane & 3;
    const int j = u * (16 * C::NW) + wave * 16 + f;
    float sw = 0.f, sb = 0.f;
    // the row kernel left per-16-row-block partial sums [n_pad/16][2][W]
    // (+0.6 % on the sweep over storing dZ0 and reducing it here)
    const float* pz = SZ + j;
#pragma unroll 4
    for (int rb = rb0 + m; rb < rb0 + nb; rb += 4) {
      sw += pz[(int64_t)rb * 2 * W];
      sb += pz[(int64_t)rb * 2 * W + W];
    }
    sw += __shfl_xor(sw, 1, 64);
    sw += __shfl_xor(sw, 2, 64);
    sb += __shfl_xor(sb, 1, 64);
    sb += __shfl_xor(sb, 2, 64);
    if (m == 0 && G) {
      slab_store<SK>(G + j, sw);
      slab_store<SK>(G + W + j, sb);
    } else if (m == 0) {
      float p = P[j], mm = M[j], vv = V[j];
      adam_update(p, mm, vv, sw, step_size, bc2s);
      P[j] = p; M[j] = mm; V[j] = vv;
      p = P[W + j]; mm = M[W + j]; vv = V[W + j];
      adam_update(p, mm, vv, sb, step_size, bc2s);
      P[W + j] = p; M[W + j] = mm; V[W + j] = vv;
    }
  }
#ifdef NERFHIP_VARIANTS
  if constexpr (SK)
    if (a.split_fused) split_finish<C, W, D, X3>(a, fit, L, t, lds);
#endif
}

// Split-K second pass: g = Σ_split gpart[split][i] in split order (fixed, so
// deterministic), then Adam on parameter i and, for weights, the transposed
// copy.  One thread per canonical parameter index; grid (ceil(P/256), n_fits).
// (W, D compile-time: the index splits and split-copy addresses fold to
// shifts and multiplies)
//
// Straight-line, with EXEC never narrowed: every lane loads from a valid
// (clamped) index, and every store is a buffer store whose offset is pushed
// past the resource's range for lanes that must not store (the hardware drops
// it).  The round-5 version returned early for the lanes past the fit's last
// parameter and branched per lane between the final-layer, hidden-layer and
// bias cases, so EXEC was rewritten right after its stores; with this grid
// running beside other groups' kernels, a store that waited behind the busy
// memory pipeline wrote through lanes whose address registers were never set
// (the concurrent split-K fault).  The wave also drains its
// stores before it ends.
template <int W, int D, int NS>
__global__ void __launch_bounds__(256) k_adam_split(KArgs a) {
  FLIGHT_ENTER();
  const int fit = blockIdx.y;
  const int L = fit_layers_of(a, fit);
  FLIGHT_DEPTH(L, fit);
  const int64_t n = n_params(W, D, L);
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool ok = i0 < n;
  const int64_t i = ok ? i0 : 0;                  // a valid index for every lane's loads
  const float* g = a.gpart + fit * a.gp_stride + i;
  // every slice's load in flight at once (NS = n_split, compile-time): a
  // runtime-count loop compiled to load → vmcnt(0) → add per slice, 15 serial
  // L2/HBM round trips (10.5 µs of config 2's 93 µs epoch)
  float gv[NS];
#pragma unroll
  for (int sp = 0; sp < NS; ++sp) gv[sp] = g[sp * a.p_stride];
  float gs = gv[0];
#pragma unroll
  for (int sp = 1; sp < NS; ++sp) gs += gv[sp];   // slice order
  const float* P = a.params + fit * a.p_stride;
  const float* M = a.m + fit * a.p_stride;
  const float* V = a.v + fit * a.p_stride;
  float p = P[i], mm = M[i], vv = V[i];
  adam_update(p, mm, vv, gs, a.sched[2 * a.epoch], a.sched[2 * a.epoch + 1]);
  const int64_t pbytes = 4 * a.p_stride;
  const uint32_t po = lane_off(ok, (uint32_t)(4 * i));
  const __amdgpu_buffer_rsrc_t pr = rsrc_over(P, pbytes), mr = rsrc_over(M, pbytes),
                               vr = rsrc_over(V, pbytes);
  bstore_f32(pr, po, p);
  bstore_f32(mr, po, mm);
  bstore_f32(vr, po, vv);
#ifdef NERFHIP_EXP_ADAM_NO_SPLIT_COPIES   // diagnostic (wrong results): cost of the split-copy stores
  if (a.x3) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    keep_live(pr, mr, vr);
    return;
  }
#endif
  // which weight (if any) parameter i is: matrix mi (1..L hidden, L+1 final),
  // element [j][k]; `wt` false for biases and the first layer.  32-bit
  // arithmetic with compile-time divisors (a 64-bit division would branch
  // per lane on the operands' high words)
  const int ii = (int)i, fw = (int)off_final_w(W, L);
  const bool fin = ii >= fw;
  const int ih = ii - 2 * W < 0 ? 0 : ii - 2 * W;
  const int rh = ih % (W * W + W);
  const int r = fin ? ii - fw : rh;
  // (bitwise, not short-circuit: && here compiled to EXEC-masked branches)
  const bool wt = ok & ((fin & (r < D * W)) | (!fin & (ii >= 2 * W) & (rh < W * W)));
  const int mi = fin ? L + 1 : ih / (W * W + W) + 1;
  const int j = wt ? r / W : 0, k = wt ? r % W : 0;
  if (a.x3) {                                     // (kernel arguments: scalar branches)
    const uint16_t* XS = a.wsplit + fit * a.ws_stride;
    const __amdgpu_buffer_rsrc_t xr = rsrc_over(XS, 2 * a.ws_stride);
    const int R = mi <= L ? W : D;
    const int f = (int)xs_mat(W, D, L, false, mi), bk = (int)xs_mat(W, D, L, true, mi);
    uint32_t h, m, l;
    split3(p, h, m, l);
    const uint16_t part[3] = {(uint16_t)(h >> 16), (uint16_t)(m >> 16), (uint16_t)(l >> 16)};
    auto copies = [&](auto lay_c) {
      constexpr int lay = decltype(lay_c)::value;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        bstore_u16(xr, lane_off(wt, (uint32_t)(2 * (f + (int)xoff_any(lay, R, W, j, k, pl)))), part[pl]);
        bstore_u16(xr, lane_off(wt, (uint32_t)(2 * (bk + (int)xoff_any(lay, W, R, k, j, pl)))), part[pl]);
      }
    };
    if (a.rows_ks) copies(std::integral_constant<int, kLayKs>{});
    else copies(std::integral_constant<int, kLayX>{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    keep_live(xr, xr, xr);
  } else {
    // both candidates computed by every lane, then selected (a `fin ? a : b`
    // of the two expressions compiled to an EXEC-masked branch)
    uint32_t tf = (uint32_t)(4 * (L * W * W + k * D + j)), th = (uint32_t)(4 * ((mi - 1) * W * W + k * W + j));
    asm volatile("" : "+v"(tf), "+v"(th));
    const __amdgpu_buffer_rsrc_t tr = rsrc_over(a.params_t + fit * a.pt_stride, 4 * a.pt_stride);
    bstore_f32(tr, lane_off(wt, fin ? tf : th), p);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    keep_live(tr, tr, tr);
  }
  // every store drained before the wave ends, and its resource registers kept
  // until then (the compiler otherwise reuses them right after the last store)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  keep_live(pr, mr, vr);
}

// ---------------------------------------------------------------------------
// Prologue / epilogue helpers
// ---------------------------------------------------------------------------

// target_mean = y.mean(0); target_std = y.std(0).clamp(min=1e-3);
// targets_norm = (y − mean)/std   (siren.py:85-87).  One workgroup per (64
// columns, fit): lane = column (64 consecutive floats of a row: coalesced), the
// 16 waves take every 16th row, fp64 partial sums are combined in a fixed
// order through LDS (deterministic), then every thread normalises its rows.
constexpr int kNormCols = 64, kNormRowGroups = 16;
__global__ void __launch_bounds__(kNormCols * kNormRowGroups) k_normalize(KArgs a) {
  FLIGHT_ENTER();
  __shared__ double part[kNormRowGroups][kNormCols];
  const int fit = blockIdx.y;
  const int c = threadIdx.x & (kNormCols - 1), rg = threadIdx.x / kNormCols;
  const int j = blockIdx.x * kNormCols + c;
  const bool col = j < a.D;
  const float* T = a.target + fit * a.t_stride;
  float* TN = a.tnorm + fit * a.t_stride;
  auto reduce = [&](double v) {     // Σ over the row groups, in order
    part[rg][c] = v;
    __syncthreads();
    double t = 0.0;
    for (int k = 0; k < kNormRowGroups; ++k) t += part[k][c];
    __syncthreads();
    return t;
  };
  double s = 0.0;
  if (col)
    for (int r = rg; r < a.N; r += kNormRowGroups) s += (double)T[(int64_t)r * a.D + j];
  const float mean = (float)(reduce(s) / a.N);
  double ss = 0.0;
  if (col)
    for (int r = rg; r < a.N; r += kNormRowGroups) {
      const double d = (double)T[(int64_t)r * a.D + j] - (double)mean;
      ss += d * d;
    }
  float sd = (float)sqrt(reduce(ss) / (double)(a.N - 1));
  sd = sd < 1e-3f ? 1e-3f : sd;
  if (col && rg == 0) {
    a.mean[fit * a.D + j] = mean;
    a.stdv[fit * a.D + j] = sd;
  }
  if (col)
    for (int r = rg; r < a.n_pad; r += kNormRowGroups) {
      const int64_t o = (int64_t)r * a.D + j;
      TN[o] = r < a.N ? (T[o] - mean) / sd : 0.f;
    }
}

// params_t ← transposed copies of every hidden weight and of the final weight
// (fp32 precision); wsplit ← both split copies (bf16x3 precision).
__global__ void k_transpose_params(KArgs a) {
  FLIGHT_ENTER();
  const int fit = blockIdx.y;
  // the same depth the step kernels train (a one-fit group: L_max, nerfhip.h)
  const int L = fit_layers_of(a, fit);
  FLIGHT_DEPTH(L, fit);
  const int W = a.W, D = a.D;
  const int64_t nh = (int64_t)L * W * W, total = nh + (int64_t)W * D;
  const float* P = a.params + fit * a.p_stride;
  float* PT = a.params_t ? a.params_t + fit * a.pt_stride : nullptr;
  uint16_t* XS = a.x3 ? a.wsplit + fit * a.ws_stride : nullptr;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (e < nh) {
      const int64_t i = e / ((int64_t)W * W), u = e % ((int64_t)W * W);
      const int64_t k = u / W, j = u % W;  // PT_i[k][j] = W_i[j][k]
      const float p = P[off_hidden_w(W, (int)i + 1) + j * W + k];
      if (PT) PT[e] = p;
      if (XS) put_w(XS, wlayout(a), W, D, L, (int)i + 1, (int)j, (int)k, p);
    } else {
      const int64_t u = e - nh;
      const int64_t k = u / D, j = u % D;  // WfT[k][j] = Wf[j][k]
      const float p = P[off_final_w(W, L) + j * W + k];
      if (PT) PT[e] = p;
      if (XS) put_w(XS, wlayout(a), W, D, L, L + 1, (int)j, (int)k, p);
    }
  }
}

// Per-row metrics of pred_real = ŷ·std + mean against the raw target:
// F.cosine_similarity(pred, y, dim=1) (eps 1e-8) and Σ_j (pred−y)².
// (siren.py:109-111, 122-125).  One wave per row.
__global__ void k_row_metrics(KArgs a, const float* ybuf, int64_t ystride,
                              float* row_cos, float* row_sq, int64_t rstride) {
  FLIGHT_ENTER();
  const int fit = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= a.n_pad) return;
  const int D = a.D;
  float* rc = row_cos + fit * rstride;
  float* rs = row_sq + fit * rstride;
  if (r >= a.N) {
    if (lane == 0) { rc[r] = 0.f; rs[r] = 0.f; }
    return;
  }
  const float* Y = ybuf + fit * ystride + (int64_t)r * D;
  const float* T = a.target + fit * a.t_stride + (int64_t)r * D;
  const float* mu = a.mean + fit * D;
  const float* sd = a.stdv + fit * D;
  float pp = 0.f, tt = 0.f, pt = 0.f, dd = 0.f;
  for (int j = lane; j < D; j += 64) {
    const float p = __fadd_rn(__fmul_rn(Y[j], sd[j]), mu[j]);
    const float t = T[j];
    const float d = p - t;
    pp = fmaf(p, p, pp);
    tt = fmaf(t, t, tt);
    pt = fmaf(p, t, pt);
    dd = fmaf(d, d, dd);
  }
  pp = wave_sum(pp); tt = wave_sum(tt); pt = wave_sum(pt); dd = wave_sum(dd);
  if (lane == 0) {
    const float n1 = fmaxf(sqrtf(pp), 1e-8f), n2 = fmaxf(sqrtf(tt), 1e-8f);
    rc[r] = pt / (n1 * n2);
    rs[r] = dd;
  }
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------

bool width_ok(int W) { return W == 64 || W == 128 || W == 256 || W == 512; }
bool dim_ok(int D) { return D == 64 || D == 128; }

int validate(int W, int D, int N, int L_max, int epochs) {
  if (!width_ok(W)) return NERFHIP_ERR_BAD_WIDTH;
  if (!dim_ok(D)) return NERFHIP_ERR_BAD_HEAD_DIM;
  if (L_max < 1 || L_max > NERFHIP_MAX_LAYERS) return NERFHIP_ERR_BAD_LAYERS;
  if (N < 2 || epochs < 0) return NERFHIP_ERR_BAD_SHAPE;
  return NERFHIP_OK;
}

// The 32-row kernel (k_step_rows32) for bf16x3 groups with W = 256, D = 128
// whose rows fill whole 128-row workgroups, unless the group takes the
// K-split kernel.  Opt-in while it is slower than the 16-row kernel
// (NERFHIP_ROWS32 = 1; kRows32Default).
constexpr bool kRows32Default = false;
bool rows32_for(const nerfhip_group* g, const nerfhip_sizes& s, bool ks) {
  if (ks || g->precision != NERFHIP_PRECISION_BF16X3 || g->W != 256 || g->D != 128 ||
      s.n_pad % 128 != 0)
    return false;
#ifdef NERFHIP_VARIANTS
  const char* e = getenv("NERFHIP_ROWS32");
  return e ? e[0] == '1' : kRows32Default;
#else
  return kRows32Default;   // not compiled into the product library
#endif
}

KArgs make_args(const nerfhip_group* g, const nerfhip_sizes& s) {
  KArgs a{};
  a.W = g->W; a.D = g->D; a.N = g->N; a.n_pad = (int32_t)s.n_pad;
  a.n_fits = g->n_fits; a.L_max = g->L_max; a.epochs = g->epochs;
  a.p_stride = s.params; a.pt_stride = s.params_t; a.s_stride = s.scratch;
  a.t_stride = s.target; a.lp_stride = s.loss_partial; a.y_stride = s.target;
  a.fit_layers = g->fit_layers; a.fit_omega = g->fit_omega; a.pos = g->positions;
  a.target = g->target; a.tnorm = g->target_norm; a.mean = g->mean; a.stdv = g->std;
  a.params = g->params; a.params_t = g->params_t; a.m = g->adam_m; a.v = g->adam_v;
  a.scratch = g->scratch; a.sched = g->sched; a.loss_partial = g->loss_partial;
  // F.mse_loss backward: grad = (2/numel)·(ŷ−y), the 2/numel a python float
  // rounded to fp32 (TORCH/_decomp/decompositions.py:393-397).
  a.grad_scale = (float)(2.0 / ((double)g->N * (double)g->D));
  bool small = false;
  a.n_split = (g->grad_partial && g->n_fits < kXcdMinFits) ? split_for(g, s, &small) : 1;
  a.small_tiles = small && a.n_split > 1;
  a.gp_stride = s.grad_partial;
  a.gpart = g->grad_partial;
  a.ctr_off = s.grad_split * s.params;
  // NERFHIP_SPLIT_FUSED = 1: the last-arriving slice reduces each tile inside
  // the parameter kernel (two launches per epoch; bitwise equal, measured
  // slower: DESIGN.md §12); default the separate k_adam_split pass
#ifdef NERFHIP_VARIANTS
  {
    const char* e = getenv("NERFHIP_SPLIT_FUSED");
    a.split_fused = a.n_split > 1 && e && e[0] == '1' ? 1 : 0;
  }
#endif
  a.x3 = g->precision == NERFHIP_PRECISION_BF16X3;
  a.ws_stride = s.wsplit;
  a.wsplit = static_cast<uint16_t*>(g->wsplit);
  a.rows_ks = rows_ks_for(g, s) ? 1 : 0;
  a.rows32 = rows32_for(g, s, a.rows_ks != 0) ? 1 : 0;
#ifdef NERFHIP_DIAG_ENV
  // diagnostic builds only — NERFHIP_ROWS_LDS_PAD / NERFHIP_PARAMS_LDS_PAD:
  // dynamic LDS per workgroup of the regular row / parameter kernels, KB
  // (schedule experiments), clamped to the CU's 160 KB
  auto pad_kb = [](const char* e) { const int k = atoi(e); return 1024u * (uint32_t)(k < 0 ? 0 : k > 96 ? 96 : k); };
  if (const char* e = getenv("NERFHIP_ROWS_LDS_PAD")) a.rows_dyn_lds = pad_kb(e);
  if (const char* e = getenv("NERFHIP_PARAMS_LDS_PAD")) a.params_dyn_lds = pad_kb(e);
#endif
#ifdef NERFHIP_DIAG_FLIGHT
  if (const char* e = getenv("NERFHIP_FLIGHT"))
    a.flight = reinterpret_cast<unsigned char*>(strtoull(e, nullptr, 0));
#endif
#if defined(NERFHIP_STAMPS) || defined(NERFHIP_EXP_KS_TRACE)
  if (const char* e = getenv("NERFHIP_PSTAMPS"))
    a.pstamps = reinterpret_cast<unsigned long long*>(strtoull(e, nullptr, 0));
#endif
  return a;
}


}  // namespace

namespace nerfhip_detail {
template <int W, int D, bool X3>
int launch_rows(const KArgs& a, hipStream_t st) {
  if constexpr (X3 && W >= 128 && D == 128) {
    if (a.rows_ks) {
      const int grid = grid_for(a.n_fits, a.n_pad / 16);
      // One K-split workgroup per CU, alone (kKsDynLds fills the CU's LDS;
      // the co-residency containment, see kKsDynLds).  This single
      // runtime-mode kernel has measured correct with and without sharing in
      // every probe (tests/test_gpu_parity.py::test_rows_ks_coresident pins
      // it): up to 64 regular workgroups its grid fits the 256 CUs, up to
      // kKsMaxWorkgroups (128) it takes two rounds (still faster,
      // rows_ks_for).  NERFHIP_KS_SHARE_CU=1 (tests / diagnostics only)
      // drops the padding so that two workgroups may share a CU.
      const char* e = getenv("NERFHIP_KS_SHARE_CU");
      unsigned dyn = (e && e[0] == '1') ? 0u : kKsDynLds;
      // never more than the kernel's own static LDS leaves of the CU's 160 KB
      // (an over-sized request aborts the queue)
      static const unsigned dyn_cap = [] {
        hipFuncAttributes fa;
        return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&k_step_rows_ks<W, D, -1>)) ==
                       hipSuccess
                   ? 163840u - (unsigned)fa.sharedSizeBytes
                   : kKsDynLds;
      }();
      if (dyn > dyn_cap) dyn = dyn_cap;
#ifdef NERFHIP_DIAG_ENV
      // diagnostic builds only: an explicit pad (clamped to what fits the CU)
      if (const char* k = getenv("NERFHIP_KS_PAD_KB")) {
        const int kb = atoi(k);
        dyn = 1024u * (unsigned)(kb < 0 ? 0 : kb) < kKsDynLds ? 1024u * (unsigned)(kb < 0 ? 0 : kb)
                                                             : kKsDynLds;
      }
#endif
#ifdef NERFHIP_EXP_KS_MODES
      if (a.mode == 0)
        hipLaunchKernelGGL((k_step_rows_ks<W, D, 0>), dim3(grid), dim3(256), dyn, st, NERFHIP_KA(a, 200000 + W * 100 + D, grid));
      else
        hipLaunchKernelGGL((k_step_rows_ks<W, D, 1>), dim3(grid), dim3(256), dyn, st, NERFHIP_KA(a, 200000 + W * 100 + D, grid));
#else
      hipLaunchKernelGGL((k_step_rows_ks<W, D, -1>), dim3(grid), dim3(256), dyn, st,
                         NERFHIP_KA(a, 200000 + W * 100 + D, grid));
#endif
      return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
    }
  }
#ifdef NERFHIP_VARIANTS
  if constexpr (X3 && W == 256 && D == 128) {
    if (a.rows32) return launch_rows32<W, D>(a, st);   // its own translation unit (NERFHIP_KIND 3)
  }
#endif
  const int grid = grid_for(a.n_fits, a.n_pad / RowsCfg<W>::ROWS);
  if (a.mode == 0)
    hipLaunchKernelGGL((k_step_rows<W, D, X3, true>), dim3(grid), dim3(RowsCfg<W>::THREADS),
                       a.rows_dyn_lds, st, NERFHIP_KA(a, 100000 + W * 100 + D, grid));
  else
    hipLaunchKernelGGL((k_step_rows<W, D, X3, false>), dim3(grid), dim3(RowsCfg<W>::THREADS), 0,
                       st, NERFHIP_KA(a, 100000 + W * 100 + D, grid));
  return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
}

// split-K second pass with the slice count compile-time (a power of two,
// 2..kMaxSplitK: fill_sizes / split_for)
template <int W, int D>
int launch_adam_split(const KArgs& a, hipStream_t st) {
  const dim3 grid((unsigned)((n_params(W, D, a.L_max) + 255) / 256), a.n_fits);
  switch (a.n_split) {
    case 2: hipLaunchKernelGGL((k_adam_split<W, D, 2>), grid, dim3(256), 0, st, NERFHIP_KA(a, 400000 + W * 100 + D, grid.x * grid.y)); break;
    case 4: hipLaunchKernelGGL((k_adam_split<W, D, 4>), grid, dim3(256), 0, st, NERFHIP_KA(a, 400000 + W * 100 + D, grid.x * grid.y)); break;
    case 8: hipLaunchKernelGGL((k_adam_split<W, D, 8>), grid, dim3(256), 0, st, NERFHIP_KA(a, 400000 + W * 100 + D, grid.x * grid.y)); break;
    case 16: hipLaunchKernelGGL((k_adam_split<W, D, 16>), grid, dim3(256), 0, st, NERFHIP_KA(a, 400000 + W * 100 + D, grid.x * grid.y)); break;
    default: return NERFHIP_ERR_LAUNCH;
  }
  return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
}

template <int W, int D, bool X3>
int launch_params(const KArgs& a, hipStream_t st) {
  if constexpr (X3 && W >= 256) {
    if (a.small_tiles) {
      using CS = ParamsCfg<W, D, X3, true>;
      const int grid_s = grid_for(a.n_fits, CS::tiles(a.L_max) * a.n_split);
#ifdef NERFHIP_VARIANTS
      if (a.split_fused) {
        hipLaunchKernelGGL((k_step_params<W, D, X3, true, kLayX, true>), dim3(grid_s),
                           dim3(CS::THREADS), 0, st, a);
        return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
      }
#endif
      hipLaunchKernelGGL((k_step_params<W, D, X3, true>), dim3(grid_s), dim3(CS::THREADS), 0, st,
                         NERFHIP_KA(a, 300000 + W * 100 + D, grid_s));
      return launch_adam_split<W, D>(a, st);
    }
  }
  const int grid = grid_for(a.n_fits, ParamsCfg<W, D, X3>::tiles(a.L_max) * a.n_split);
  // (the K-split layout epilogue exists only for shapes the K-split row
  // kernel runs: bf16x3, W >= 128, D = 128 — rows_ks_for)
  if constexpr (X3 && W >= 128 && D == 128) {
    if (a.rows_ks && a.n_split == 1) {   // fused epilogue writes the K-split layout
      hipLaunchKernelGGL((k_step_params<W, D, X3, false, kLayKs>), dim3(grid),
                         dim3(ParamsCfg<W, D, X3>::THREADS), 0, st, NERFHIP_KA(a, 300000 + W * 100 + D, grid));
      return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
    }
  }
#ifdef NERFHIP_VARIANTS
  if constexpr (X3 && W == 256 && D == 128) {
    if (a.rows32 && a.n_split == 1) {    // ... or the 32-row kernel's
      hipLaunchKernelGGL((k_step_params<W, D, X3, false, kLay32>), dim3(grid),
                         dim3(ParamsCfg<W, D, X3>::THREADS), a.params_dyn_lds, st, a);
      return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
    }
  }
  if (a.split_fused) {
    hipLaunchKernelGGL((k_step_params<W, D, X3, false, kLayX, true>), dim3(grid),
                       dim3(ParamsCfg<W, D, X3>::THREADS), a.params_dyn_lds, st, a);
    return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
  }
#endif
  hipLaunchKernelGGL((k_step_params<W, D, X3>), dim3(grid), dim3(ParamsCfg<W, D, X3>::THREADS),
                     a.params_dyn_lds, st, NERFHIP_KA(a, 300000 + W * 100 + D, grid));
  if (a.n_split > 1) return launch_adam_split<W, D>(a, st);
  return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
}

// The 32-row kernel is compiled only in its own translation unit
// (NERFHIP_KIND 3: -amdgpu-mfma-vgpr-form, accumulators in VGPRs, the B
// operand in AGPRs); every other unit sees the declaration only.
#if defined(NERFHIP_VARIANTS) && (NERFHIP_KIND == 3 || NERFHIP_PART < 0)
template <int W, int D>
int launch_rows32(const KArgs& a, hipStream_t st) {
  const int grid = grid_for(a.n_fits, a.n_pad / 128);
  if (a.mode == 0)
    hipLaunchKernelGGL((k_step_rows32<W, D, true>), dim3(grid), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((k_step_rows32<W, D, false>), dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
}
#endif

// NERFHIP_KIND splits a part further: 1 = row kernels only, 2 = parameter
// kernels only (compiled with different flags, nerf_attention/_build.py),
// 3 = the 32-row kernel only, 0 = all
#ifndef NERFHIP_KIND
#define NERFHIP_KIND 0
#endif
#if NERFHIP_KIND == 3
#define NERFHIP_INST_ONE(W, D, X)
#if NERFHIP_PART == 6 && defined(NERFHIP_VARIANTS)
template int launch_rows32<256, 128>(const KArgs&, hipStream_t);
#endif
#elif NERFHIP_KIND == 1
#define NERFHIP_INST_ONE(W, D, X) template int launch_rows<W, D, X>(const KArgs&, hipStream_t);
#elif NERFHIP_KIND == 2
#define NERFHIP_INST_ONE(W, D, X) template int launch_params<W, D, X>(const KArgs&, hipStream_t);
#else
#define NERFHIP_INST_ONE(W, D, X) \
  template int launch_rows<W, D, X>(const KArgs&, hipStream_t); \
  template int launch_params<W, D, X>(const KArgs&, hipStream_t);
#endif
#define NERFHIP_INST(W, X) NERFHIP_INST_ONE(W, 64, X) NERFHIP_INST_ONE(W, 128, X)
#if NERFHIP_PART == 1
NERFHIP_INST(64, false)
#elif NERFHIP_PART == 2
NERFHIP_INST(64, true)
#elif NERFHIP_PART == 3
NERFHIP_INST(128, false)
#elif NERFHIP_PART == 4
NERFHIP_INST(128, true)
#elif NERFHIP_PART == 5
NERFHIP_INST(256, false)
#elif NERFHIP_PART == 6
NERFHIP_INST(256, true)
#elif NERFHIP_PART == 7
NERFHIP_INST(512, false)
#elif NERFHIP_PART == 8
NERFHIP_INST(512, true)
#elif NERFHIP_PART == 0
#define NERFHIP_EXTERN_ONE(W, D, X) \
  extern template int launch_rows<W, D, X>(const KArgs&, hipStream_t); \
  extern template int launch_params<W, D, X>(const KArgs&, hipStream_t);
#define NERFHIP_EXTERN(W) \
  NERFHIP_EXTERN_ONE(W, 64, false) NERFHIP_EXTERN_ONE(W, 64, true) \
  NERFHIP_EXTERN_ONE(W, 128, false) NERFHIP_EXTERN_ONE(W, 128, true)
NERFHIP_EXTERN(64)
NERFHIP_EXTERN(128)
NERFHIP_EXTERN(256)
NERFHIP_EXTERN(512)
#endif
}  // namespace nerfhip_detail

#if NERFHIP_PART <= 0
namespace {
using nerfhip_detail::launch_params;
using nerfhip_detail::launch_rows;

typedef int (*launch_fn)(const KArgs&, hipStream_t);

template <int W, bool X3>
void pick_d(int D, launch_fn* rows, launch_fn* params) {
  if (D == 64) { *rows = launch_rows<W, 64, X3>; *params = launch_params<W, 64, X3>; }
  else { *rows = launch_rows<W, 128, X3>; *params = launch_params<W, 128, X3>; }
}

template <bool X3>
void pick_w(int W, int D, launch_fn* rows, launch_fn* params) {
  switch (W) {
    case 64: pick_d<64, X3>(D, rows, params); break;
    case 128: pick_d<128, X3>(D, rows, params); break;
    case 256: pick_d<256, X3>(D, rows, params); break;
    default: pick_d<512, X3>(D, rows, params); break;
  }
}

void pick(int W, int D, bool x3, launch_fn* rows, launch_fn* params) {
  if (x3) pick_w<true>(W, D, rows, params);
  else pick_w<false>(W, D, rows, params);
}

int row_metrics(const KArgs& a, const float* ybuf, int64_t ystride, float* rc, float* rs,
                int64_t rstride, hipStream_t st) {
  dim3 grid((unsigned)((a.n_pad + 3) / 4), (unsigned)a.n_fits);
  hipLaunchKernelGGL(k_row_metrics, grid, dim3(256), 0, st, NERFHIP_KA(a, 700000, grid.x * grid.y), ybuf,
                     ystride, rc, rs, rstride);
  return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
}

}  // namespace

extern "C" {

int nerfhip_abi_version(void) { return NERFHIP_ABI_VERSION; }

// Diagnostic compile-time switches (nerfhip.h NERFHIP_BUILD_*).  Every
// NERFHIP_EXP_* / NERFHIP_DIAG_* name the source tests must be listed here
// (tests/test_capi.py checks the source against this list); variant builds
// (tools/build_variant.py) pass them to every translation unit, this one too.
int nerfhip_build_flags(void) {
  int f = 0;
#if defined(NERFHIP_EXP_ADAM_NO_SPLIT_COPIES) || defined(NERFHIP_EXP_DWORD_STORES) ||       \
    defined(NERFHIP_EXP_KS_ALTFIT) || defined(NERFHIP_EXP_KS_LINEAR) ||                      \
    defined(NERFHIP_EXP_KS_MODES) || defined(NERFHIP_EXP_KS_SPLIT_F) ||                      \
    defined(NERFHIP_EXP_KS_SPLIT_H) || defined(NERFHIP_EXP_KS_VMWAIT) ||                     \
    defined(NERFHIP_EXP_KS_TRACE) || defined(NERFHIP_EXP_HOTBLOCK) ||                        \
    defined(NERFHIP_EXP_SPLIT_AFTER_MFMA) || defined(NERFHIP_EXP_PARAMS_PRIO) ||             \
    defined(NERFHIP_EXP_NOBARRIER) || defined(NERFHIP_EXP_NOFLUSH) ||                        \
    defined(NERFHIP_EXP_NOSTAGE) || defined(NERFHIP_EXP_NO_FWDCOPY) ||                       \
    defined(NERFHIP_EXP_STAGE_IDENTITY) || defined(NERFHIP_EXP_X2PROXY) ||                   \
    (NERFHIP_SINCOS != 0)
  f |= NERFHIP_BUILD_EXP;
#endif
#ifdef NERFHIP_STAMPS
  f |= NERFHIP_BUILD_STAMPS;
#endif
#if defined(NERFHIP_DIAG_ROWS_TWICE) || defined(NERFHIP_DIAG_ENV) || defined(NERFHIP_DIAG_FLIGHT)
  f |= NERFHIP_BUILD_DIAG;
#endif
#ifdef NERFHIP_VARIANTS
  f |= NERFHIP_BUILD_VARIANTS;
#endif
  return f;
}

#ifdef NERFHIP_DIAG_FLIGHT
}  // extern "C"
// host side of the flight recorder: a launch's sequence number, argument hash
// and the slot header of what was launched (written before the launch)
KArgs nerfhip_detail::flight_stamp(const KArgs& a, int kid, unsigned grid) {
  static std::atomic<uint32_t> next{1};
  KArgs b = a;
  b.seq = next.fetch_add(1);
  b.hash = 0;
  b.hash = kargs_hash(b);
  if (b.flight) {
    unsigned char* s = b.flight + (size_t)(b.seq % kFlightRing) * kFlightSlot;
    memset(s, 0, kFlightSlot);
    volatile uint64_t* h = reinterpret_cast<volatile uint64_t*>(s);
    h[1] = (uint64_t)kid;
    h[2] = (uint64_t)(uint32_t)b.epoch | ((uint64_t)b.group << 32) | ((uint64_t)b.mode << 48);
    h[3] = grid;
    h[4] = b.hash;
    h[5] = (uint64_t)b.n_split | ((uint64_t)b.n_fits << 16) | ((uint64_t)b.L_max << 32);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    h[0] = b.seq;   // last: a slot whose word 0 is set is complete
  }
  return b;
}
extern "C" {
// diagnostic build only: the flight-recorder ring in host-mapped, coherent
// memory (the device writes it with system-scope stores; readable after a
// device fault)
void* nerfhip_debug_flight_alloc(void) {
  void* p = nullptr;
  const size_t n = (size_t)nerfhip_detail::kFlightRing * nerfhip_detail::kFlightSlot;
  if (hipHostMalloc(&p, n, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
  memset(p, 0, n);
  return p;
}
#endif

#ifdef NERFHIP_STAMPS
// diagnostic build only: device buffer of [blocks][4 waves][8] u64 stamps
int nerfhip_debug_set_stamps(unsigned long long* dev_ptr) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dev_ptr, sizeof(dev_ptr)) == hipSuccess
             ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
}
#endif

const char* nerfhip_status_string(int status) {
  switch (status) {
    case NERFHIP_OK: return "ok";
    case NERFHIP_ERR_BAD_WIDTH: return "hidden_features must be one of 64, 128, 256, 512";
    case NERFHIP_ERR_BAD_HEAD_DIM: return "d_head must be 64 or 128";
    case NERFHIP_ERR_BAD_LAYERS: return "hidden_layers must be in [1, 4]";
    case NERFHIP_ERR_BAD_SHAPE: return "bad shape (seq_len >= 2, n_fits >= 1, epochs >= 0)";
    case NERFHIP_ERR_NULL: return "a required device pointer is NULL";
    case NERFHIP_ERR_LAUNCH: return "kernel launch failed";
    case NERFHIP_ERR_BAD_PRECISION: return "precision must be NERFHIP_PRECISION_FP32 or _BF16X3";
    default: return "unknown nerfhip status";
  }
}

int nerfhip_group_sizes(int32_t W, int32_t D, int32_t N, int32_t L_max, int32_t epochs,
                        nerfhip_sizes* out) {
  if (!out) return NERFHIP_ERR_NULL;
  const int rc = validate(W, D, N, L_max, epochs);
  if (rc != NERFHIP_OK) return rc;
  fill_sizes(W, D, N, L_max, epochs, out);
  return NERFHIP_OK;
}

static int check_group(const nerfhip_group* g, bool train) {
  if (!g) return NERFHIP_ERR_NULL;
  const int rc = validate(g->W, g->D, g->N, g->L_max, g->epochs);
  if (rc != NERFHIP_OK) return rc;
  if (g->n_fits < 1) return NERFHIP_ERR_BAD_SHAPE;
  if (g->precision != NERFHIP_PRECISION_FP32 && g->precision != NERFHIP_PRECISION_BF16X3)
    return NERFHIP_ERR_BAD_PRECISION;
  if (!g->fit_layers || !g->fit_omega || !g->positions || !g->params || !g->eval_y)
    return NERFHIP_ERR_NULL;
  if (g->precision == NERFHIP_PRECISION_BF16X3 && !g->wsplit) return NERFHIP_ERR_NULL;
  if (train && (!g->target || !g->target_norm || !g->mean || !g->std || !g->params_t ||
                !g->adam_m || !g->adam_v || !g->scratch || !g->sched || !g->loss_partial ||
                !g->row_cos || !g->row_sq))
    return NERFHIP_ERR_NULL;
  if (train && g->log_every > 0 && g->epochs / g->log_every > 0 &&
      (!g->probe_y || !g->probe_row_cos || !g->probe_row_sq))
    return NERFHIP_ERR_NULL;
  return NERFHIP_OK;
}

namespace {

struct GroupRun {
  const nerfhip_group* g;
  hipStream_t st;
  nerfhip_sizes s;
  KArgs a;
  launch_fn rows, params;
  int n_probe;
  int64_t probe_stride;
};

int select_device(int dev, int* cur) {
  if (*cur == dev) return NERFHIP_OK;
  if (hipSetDevice(dev) != hipSuccess) return NERFHIP_ERR_LAUNCH;
  *cur = dev;
  return NERFHIP_OK;
}

int prologue(GroupRun& r) {
  const nerfhip_group* g = r.g;
  // Adam state ← 0 (torch.optim.Adam lazy state init), normalise the target,
  // transposed weight copies.
  const size_t pbytes = (size_t)g->n_fits * r.s.params * sizeof(float);
  if (hipMemsetAsync(g->adam_m, 0, pbytes, r.st) != hipSuccess) return NERFHIP_ERR_LAUNCH;
  if (hipMemsetAsync(g->adam_v, 0, pbytes, r.st) != hipSuccess) return NERFHIP_ERR_LAUNCH;
  // the fused split step's arrival counters start at 0 (split_finish)
  if (r.a.split_fused)
    for (int f = 0; f < g->n_fits; ++f)
      if (hipMemsetAsync(g->grad_partial + f * r.s.grad_partial + r.a.ctr_off, 0,
                         (size_t)(r.s.grad_partial - r.a.ctr_off) * sizeof(float), r.st) != hipSuccess)
        return NERFHIP_ERR_LAUNCH;
  hipLaunchKernelGGL(k_normalize, dim3((g->D + kNormCols - 1) / kNormCols, g->n_fits),
                     dim3(kNormCols * kNormRowGroups), 0, r.st,
                     NERFHIP_KA(r.a, 500000, ((g->D + kNormCols - 1) / kNormCols) * g->n_fits));
  hipLaunchKernelGGL(k_transpose_params, dim3(64, g->n_fits), dim3(256), 0, r.st,
                     NERFHIP_KA(r.a, 600000, 64 * g->n_fits));
  return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
}

// NERFHIP_SYNC_CHECK=1 (debugging): synchronise after every launch and name
// the failing step on stderr (group shape, epoch, which kernel)
bool sync_check_on() {
  static const bool on = [] {
    const char* e = getenv("NERFHIP_SYNC_CHECK");
    return e && e[0] == '1';
  }();
  return on;
}
int sync_check(const GroupRun& r, int e, const char* what, int rc) {
  if (rc != NERFHIP_OK || !sync_check_on()) return rc;
  const hipError_t err = hipStreamSynchronize(r.st);
  if (err == hipSuccess) return rc;
  fprintf(stderr, "nerfhip: %s failed: W=%d D=%d N=%d n_fits=%d L_max=%d epoch=%d split=%d rows_ks=%d: %s\n",
          what, r.g->W, r.g->D, r.g->N, r.g->n_fits, r.g->L_max, e, r.a.n_split, r.a.rows_ks,
          hipGetErrorString(err));
  return NERFHIP_ERR_LAUNCH;
}

int epoch_step(GroupRun& r, int e, hipEvent_t* ev /* 3 or NULL */) {
  KArgs& a = r.a;
  a.epoch = e;
  a.mode = 0;
  a.y_out = nullptr;
  if (r.n_probe > 0 && (e + 1) % r.g->log_every == 0) {
    a.y_out = r.g->probe_y + (int64_t)((e + 1) / r.g->log_every - 1) * r.s.target;
    a.y_stride = r.probe_stride;
  }
  if (ev) (void)hipEventRecord(ev[0], r.st);
  int rc = sync_check(r, e, "row step", r.rows(a, r.st));
#ifdef NERFHIP_DIAG_ROWS_TWICE
  // diagnostic build only: the row step again (same inputs, same outputs) with
  // its weight planes now resident in L2 — how much of it is cold weight reads
  if (rc == NERFHIP_OK) rc = r.rows(a, r.st);
#endif
  if (ev) (void)hipEventRecord(ev[1], r.st);
  if (rc == NERFHIP_OK) rc = sync_check(r, e, "parameter step", r.params(a, r.st));
  if (ev) (void)hipEventRecord(ev[2], r.st);
  return rc;
}

int epilogue(GroupRun& r) {
  // final evaluation (siren.py:119-125) and the probe metrics (siren.py:109-111)
  KArgs& a = r.a;
  const nerfhip_group* g = r.g;
  a.mode = 1;
  a.y_out = g->eval_y;
  a.y_stride = r.s.target;
  int rc = r.rows(a, r.st);
  if (rc == NERFHIP_OK)
    rc = row_metrics(a, g->eval_y, r.s.target, g->row_cos, g->row_sq, r.s.rows, r.st);
  for (int k = 0; k < r.n_probe && rc == NERFHIP_OK; ++k)
    rc = row_metrics(a, g->probe_y + k * r.s.target, r.probe_stride,
                     g->probe_row_cos + k * r.s.rows, g->probe_row_sq + k * r.s.rows,
                     (int64_t)r.n_probe * r.s.rows, r.st);
  return rc;
}

GroupRun make_run(const nerfhip_group* g, void* stream) {
  GroupRun r;
  r.g = g;
  r.st = (hipStream_t)stream;
  fill_sizes(g->W, g->D, g->N, g->L_max, g->epochs, &r.s);
  r.a = make_args(g, r.s);
  pick(g->W, g->D, r.a.x3 != 0, &r.rows, &r.params);
  r.n_probe = g->log_every > 0 ? g->epochs / g->log_every : 0;
  r.probe_stride = (int64_t)r.n_probe * r.s.target;
  return r;
}

}  // namespace

// The timed variant brackets every kTimeStride-th epoch's two launches with
// hipEvents (all of them measured 0.5 % of the sweep's wall clock, bench
// --no-kernel-timing A/B, profiles/r02/bench_event_overhead.log); the
// averages are over the timed launches.  The sampled epochs are
// kTimeStride-1, 2·kTimeStride-1, …: the cold first launch (code-object load,
// cold L2) is never among them.
constexpr int kTimeStride = 4;
static int timed_epochs(int E) { return E / kTimeStride; }
static bool timed_epoch(int e) { return e % kTimeStride == kTimeStride - 1; }

static int fit_impl(const nerfhip_group* groups, int32_t n_groups, void* const* streams,
                    nerfhip_timing* timings) {
  if (!groups || !streams || n_groups < 1) return NERFHIP_ERR_NULL;
  for (int i = 0; i < n_groups; ++i) {
    const int rc = check_group(&groups[i], true);
    if (rc != NERFHIP_OK) return rc;
  }
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) return NERFHIP_ERR_LAUNCH;
  int cur = prev;
  GroupRun* runs = new GroupRun[n_groups];
  hipEvent_t** ev = timings ? new hipEvent_t*[n_groups]() : nullptr;
  int rc = NERFHIP_OK, max_epochs = 0;
  for (int i = 0; i < n_groups && rc == NERFHIP_OK; ++i) {
    runs[i] = make_run(&groups[i], streams[i]);
    runs[i].a.group = (uint32_t)i;
    if (groups[i].epochs > max_epochs) max_epochs = groups[i].epochs;
    rc = select_device(groups[i].device, &cur);
    if (rc == NERFHIP_OK) rc = prologue(runs[i]);
    if (ev && rc == NERFHIP_OK) {
      // 3 events per timed epoch (every kTimeStride-th): before the row step,
      // between, after the param step
      const int ne = 3 * timed_epochs(groups[i].epochs);
      ev[i] = new hipEvent_t[ne > 0 ? ne : 1]();
      for (int k = 0; k < ne && rc == NERFHIP_OK; ++k)
        if (hipEventCreate(&ev[i][k]) != hipSuccess) rc = NERFHIP_ERR_LAUNCH;
    }
  }
  for (int e = 0; e < max_epochs && rc == NERFHIP_OK; ++e)
    for (int i = 0; i < n_groups && rc == NERFHIP_OK; ++i) {
      if (e >= groups[i].epochs) continue;
      rc = select_device(groups[i].device, &cur);
      if (rc == NERFHIP_OK)
        rc = epoch_step(runs[i], e, ev && timed_epoch(e) && e / kTimeStride < timed_epochs(groups[i].epochs)
                                          ? ev[i] + 3 * (e / kTimeStride) : nullptr);
    }
  for (int i = 0; i < n_groups && rc == NERFHIP_OK; ++i) {
    rc = select_device(groups[i].device, &cur);
    if (rc == NERFHIP_OK) rc = epilogue(runs[i]);
  }
  if (ev) {
    for (int i = 0; i < n_groups; ++i) {
      if (!ev[i]) continue;
      const int E = timed_epochs(groups[i].epochs);
      if (rc == NERFHIP_OK) rc = select_device(groups[i].device, &cur);
      if (rc == NERFHIP_OK && hipStreamSynchronize(runs[i].st) != hipSuccess) rc = NERFHIP_ERR_LAUNCH;
      if (rc == NERFHIP_OK) {
        double rows_ms = 0.0, params_ms = 0.0;
        for (int e = 0; e < E; ++e) {
          float x = 0.f, y = 0.f;
          (void)hipEventElapsedTime(&x, ev[i][3 * e], ev[i][3 * e + 1]);
          (void)hipEventElapsedTime(&y, ev[i][3 * e + 1], ev[i][3 * e + 2]);
          rows_ms += x;
          params_ms += y;
        }
        timings[i].launches = E;
        timings[i].reserved = 0;
        timings[i].rows_ms = rows_ms;
        timings[i].params_ms = params_ms;
      }
      for (int k = 0; k < 3 * E; ++k)
        if (ev[i][k]) (void)hipEventDestroy(ev[i][k]);
      delete[] ev[i];
    }
    delete[] ev;
  }
  delete[] runs;
  if (cur != prev) (void)hipSetDevice(prev);
  return rc;
}

int nerfhip_siren_fit(const nerfhip_group* groups, int32_t n_groups, void* const* streams) {
  return fit_impl(groups, n_groups, streams, nullptr);
}

int nerfhip_siren_fit_timed(const nerfhip_group* groups, int32_t n_groups, void* const* streams,
                            nerfhip_timing* timings) {
  if (!timings) return NERFHIP_ERR_NULL;
  return fit_impl(groups, n_groups, streams, timings);
}

int nerfhip_siren_forward(const nerfhip_group* g, void* stream) {
  int rc = check_group(g, false);
  if (rc != NERFHIP_OK) return rc;
  GroupRun r = make_run(g, stream);
  r.a.mode = 1;
  r.a.y_out = g->eval_y;
  r.a.y_stride = r.s.target;
  if (r.a.x3) {   // the split weight copies of the current params
    hipLaunchKernelGGL(k_transpose_params, dim3(64, g->n_fits), dim3(256), 0, r.st,
                       NERFHIP_KA(r.a, 600000, 64 * g->n_fits));
    if (hipGetLastError() != hipSuccess) return NERFHIP_ERR_LAUNCH;
  }
  rc = r.rows(r.a, r.st);
  if (rc == NERFHIP_OK && g->target && g->mean && g->std && g->row_cos && g->row_sq)
    rc = row_metrics(r.a, g->eval_y, r.s.target, g->row_cos, g->row_sq, r.s.rows, r.st);
  return rc;
}

int nerfhip_group_plan(const nerfhip_group* g, nerfhip_plan* out) {
  if (!g || !out) return NERFHIP_ERR_NULL;
  int rc = validate(g->W, g->D, g->N, g->L_max, g->epochs);
  if (rc != NERFHIP_OK) return rc;
  if (g->n_fits < 1) return NERFHIP_ERR_BAD_SHAPE;
  if (g->precision != NERFHIP_PRECISION_FP32 && g->precision != NERFHIP_PRECISION_BF16X3)
    return NERFHIP_ERR_BAD_PRECISION;
  nerfhip_sizes s;
  fill_sizes(g->W, g->D, g->N, g->L_max, g->epochs, &s);
  const KArgs a = make_args(g, s);
  const int rows_per_wg = a.rows_ks ? 16 : a.rows32 ? 128 : 64;
  out->rows_variant = a.rows_ks ? NERFHIP_ROWS_KSPLIT
                                : a.rows32 ? NERFHIP_ROWS_32 : NERFHIP_ROWS_REGULAR;
  out->grad_split = a.n_split;
  out->rows_workgroups = grid_for(a.n_fits, (int)(s.n_pad / rows_per_wg));
  out->params_workgroups =
      grid_for(a.n_fits, (int)param_tiles(g->W, g->D, g->L_max, a.small_tiles != 0) * a.n_split);
  out->launches_per_epoch = a.n_split > 1 && !a.split_fused ? 3 : 2;
  out->reserved = 0;
  return NERFHIP_OK;
}

}  // extern "C"
#endif  // NERFHIP_PART <= 0
