// nerfhip_layout.h — index and layout functions of the SIREN KV-fit engine,
// shared by the HIP kernels (nerfhip.hip) and host-only checkers.
//
// Everything here is pure integer arithmetic on the group's shape: the
// split-plane weight layouts, the per-fit parameter offsets (state_dict order,
// reference siren.py:39-58), the XCD-aware block map, the parameter-kernel
// tiling and staging order, and the buffer sizes / split-K choices the host
// makes (nerfhip_group_sizes, nerfhip.h).  Compiled as __host__ __device__
// under hipcc and as plain C++ elsewhere, so that tools/r6/split_replay.cpp
// can replay the kernels' address generation on the CPU (under ASan) with the
// very functions the kernels use.
#ifndef NERFHIP_LAYOUT_H
#define NERFHIP_LAYOUT_H

#include <stdint.h>
#include <stdlib.h>

#include "nerfhip.h"

#ifdef __HIPCC__
#define NERFHIP_HD __host__ __device__
#define NERFHIP_HDI __host__ __device__ __forceinline__
#else
#define NERFHIP_HD
#define NERFHIP_HDI inline
#endif

#ifndef NERFHIP_ROWPAD
#define NERFHIP_ROWPAD 64
#endif
constexpr int kRowPad = NERFHIP_ROWPAD;   // n_pad granule: a whole number of row workgroups

// Split-plane layout of a weight matrix M[R][K] (R % 16 == 0, K % 32 == 0):
// [R/16][K/KC][3 planes][16 rows][KC] bf16, KC = min(K, 256), so a 16-row ×
// KC sub-chunk of all three planes is one contiguous run.  Inside every
// 32-wide k-block feature f sits at kperm(f): the order in which a lane
// (row c, group g) of the B operand holds accumulator tiles 2t and 2t+1 of
// the layer before — so a lane's 8 k-values are one 16-B read per plane.
NERFHIP_HD constexpr int kc_of(int K) { return K < 256 ? K : 256; }
NERFHIP_HD inline int kperm(int f) {
  return 8 * ((f & 15) >> 2) + 4 * (f >> 4) + (f & 3);
}
NERFHIP_HD inline int64_t xoff(int R, int K, int r, int k, int plane) {
  const int KC = kc_of(K);
  return ((((int64_t)(r >> 4) * (K / KC) + k / KC) * 3 + plane) * 16 + (r & 15)) * KC +
         ((k % KC) & ~31) + kperm(k & 31);
}
// The K-split row kernel's layout of the same planes (groups that run
// k_step_rows_ks, KArgs::rows_ks): [R/16][K/32][3 planes][16 rows][32]
// — every (16-row tile, 32-deep k-slice, plane) is one contiguous 1 KB block,
// the A-fragment item one wave loads with one fully coalesced 16-B-per-lane
// load per plane (kperm inside the slice as above).  Read through xoff's
// [.][K/KC][3][16][KC] chunks, that item was 16 rows x 64 B scattered over 16
// cache lines: lane-linear items took the K-split row step of one medium fit
// from 62.2 to 37.3 µs (diagnostic timing, profiles/r03/ks_layout.log).
NERFHIP_HD inline int64_t xoff_ks(int K, int r, int k, int plane) {
  return ((((int64_t)(r >> 4) * (K >> 5) + (k >> 5)) * 3 + plane) << 9) + ((r & 15) << 5) +
         kperm(k & 31);
}
// The 32-row kernel's layout (groups that run k_step_rows32, KArgs::rows32):
// [R/32][K/128][3 planes][32 rows][128] — one 32-row × 128-k sub-chunk of all
// three planes is one contiguous 24 KB run (its LDS-DMA unit) — with the k
// order inside every 16-deep k-step permuted to the 32 × 32 × 16 MFMA
// operand order: stored position 8h + j of a lane half h holds feature
// 8(j>>2) + 4h + (j&3), the order in which the 32 × 32 accumulator tile of
// the layer before hands a lane its next-layer B fragment.
NERFHIP_HD inline int perm32(int f) {   // f in [0, 16)
  return 8 * ((f >> 2) & 1) + 4 * (f >> 3) + (f & 3);
}
NERFHIP_HD inline int64_t xoff32(int K, int r, int k, int plane) {
  return ((((int64_t)(r >> 5) * (K >> 7) + (k >> 7)) * 3 + plane) * 32 + (r & 31)) * 128 +
         (k & 127 & ~15) + perm32(k & 15);
}
// weight-plane layouts (KArgs: rows_ks → xoff_ks, rows32 → xoff32, else xoff)
constexpr int kLayX = 0, kLayKs = 1, kLay32 = 2;
NERFHIP_HD inline int64_t xoff_any(int lay, int R, int K, int r, int k, int plane) {
  return lay == kLayKs ? xoff_ks(K, r, k, plane)
                       : lay == kLay32 ? xoff32(K, r, k, plane) : xoff(R, K, r, k, plane);
}
// per-fit split matrices: forward M_i [out][in] for i = 1..L (hidden) and
// i = L+1 (final, [D][W]), then the transposed M_iᵀ the backward streams
NERFHIP_HD inline int64_t xs_mat(int W, int D, int L, bool bwd, int i) {
  const int64_t base = bwd ? 3 * ((int64_t)L * W * W + (int64_t)D * W) : 0;
  return base + (int64_t)(i - 1) * 3 * W * W;
}
NERFHIP_HD inline int64_t xs_size(int W, int D, int L) {
  return 6 * ((int64_t)L * W * W + (int64_t)D * W);
}

// XCD-aware block → (fit, tile).  Blocks b and b+8 share an XCD (observed
// round-robin dispatch, MI355X_MICROARCH.md §Workgroup dispatch); every tile
// of a fit goes to the same b%8 class so its weights and scratch stay in one
// XCD's L2.  Speed only — correctness never depends on placement.
// Groups of fewer than 8 fits map linearly instead: pinning a lone fit to one
// XCD would leave 7/8 of the chip idle (BASELINE configs 2 and 5).
constexpr int kXcdMinFits = 8;
NERFHIP_HD inline int grid_for(int n_fits, int n_tiles) {
  return n_fits < kXcdMinFits ? n_fits * n_tiles : 8 * n_tiles * ((n_fits + 7) / 8);
}
NERFHIP_HDI bool map_block(int b, int n_fits, int n_tiles, int& fit, int& tile) {
  if (n_fits < kXcdMinFits) {
    fit = b / n_tiles;
    tile = b - fit * n_tiles;
    return true;
  }
  const int x = b & 7, idx = b >> 3;
  const int slot = idx / n_tiles;
  tile = idx - slot * n_tiles;
  fit = x + 8 * slot;
  return fit < n_fits;
}

NERFHIP_HD inline int64_t off_hidden_w(int W, int i) {  // i = 1..L
  return 2 * (int64_t)W + (int64_t)(i - 1) * ((int64_t)W * W + W);
}
NERFHIP_HD inline int64_t off_final_w(int W, int L) {
  return 2 * (int64_t)W + (int64_t)L * ((int64_t)W * W + W);
}
NERFHIP_HD inline int64_t n_params(int W, int D, int L) {
  return off_final_w(W, L) + (int64_t)W * D + D;
}

// Staging slot of thread-round index i (feature·4 + quarter, quarter = 4 rows
// of the 16-row block): a permutation inside every aligned group of 64 (one
// wave's round = 16 features × 4 quarters) that decides which feature each
// lane carries, so that the lane groups of the LDS store hit every bank once.
// Global loads stay whole 128-B lines (the wave still reads one contiguous
// 1 KB run); the LDS image, and so every result, is unchanged.
//   bf16x3 (ds_write_b64, 16-lane groups, 48-B feature stride): a group holds
//     features {0,2,4,6}, {1,3,5,7}, {8,10,12,14} or {9,11,13,15} — dword
//     starts 12f mod 32 = 0/24/16/8 (or 12/4/28/20), 8 dwords each.  The
//     identity (4 consecutive features per group) put two lanes on each of 8
//     banks: 33 % of the kernel's LDS-array cycles were conflict cycles
//     (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, profiles/r02/pmc_isolated_groups.json).
//   fp32 (ds_write_b128, 8-lane groups, 80-B feature stride): a group holds
//     features {f, f+4}: dword starts 20f mod 32 and 20f + 16.
template <bool X3> NERFHIP_HDI int stage_slot(int i) {
#ifdef NERFHIP_EXP_STAGE_IDENTITY   // diagnostic build: the round-2 (conflicted) lane order
  return i;
#endif
  const int l = i & 63;
  int f;
  if constexpr (X3) {
    const int g4 = l >> 4;
    f = (g4 >> 1) * 8 + 2 * ((l >> 2) & 3) + (g4 & 1);
  } else {
    const int g8 = l >> 3;
    f = (g8 >> 2) * 8 + (g8 & 3) + 4 * ((l >> 2) & 1);
  }
  return (i & ~63) | (f << 2) | (l & 3);
}

// Tiles: dW[j0:j0+T][k0:k0+TK] on 4 waves, two workgroups per CU.  (WIDE:
// T × 256 tiles on 8 waves, one workgroup per CU, reads each dZ column block
// once instead of W/128 times — a quarter less operand traffic — yet measured
// 7 % slower at W = 256 and 512.)
// SMALL: 64 × 64 tiles for the split-K launches of small bf16x3 groups with
// W >= 256 (split_for decides): 3.1x the tiles of 128 × 128, so the same grid
// needs fewer row slices — fewer partial-slab bytes written and read back by
// k_adam_split, the split step's floor.
template <int W, int D, bool X3, bool SMALL = false> struct ParamsCfg {
  static constexpr bool WIDE = false;
  static constexpr int T = SMALL ? 64 : (W < 128 ? W : 128);   // hidden-layer tile rows (j)
  static constexpr int TK = WIDE ? 256 : T;            // tile columns (k), hidden and final
  static constexpr int NW = WIDE ? 8 : 4, THREADS = 64 * NW;
  static constexpr int MINB = WIDE ? 1 : 2;            // workgroups per CU (launch bound)
  static constexpr int TD = D < T ? D : T;             // final-layer tile rows
  static constexpr int NTJ = W / T, NTK = W / TK;
  static constexpr int TH = NTJ * NTK, TF = (D / TD) * NTK, T0 = W / (16 * NW);
  NERFHIP_HD static int tiles(int L) { return L * TH + TF + T0; }
};

constexpr int kMaxSplitK = 16;   // most row slices of a split-K reduction (nerfhip_sizes.grad_split)

constexpr int64_t kMaxSplit = kMaxSplitK;
inline int64_t param_tiles(int W, int D, int L, bool small = false);
inline int64_t split_ctr_elems(int W, int D, int L_max) {
  const int64_t t = param_tiles(W, D, L_max, true), u = param_tiles(W, D, L_max, false);
  return ((t > u ? t : u) + 63) / 64 * 64;
}
inline void fill_sizes(int W, int D, int N, int L_max, int epochs, nerfhip_sizes* s) {
  const int64_t n_pad = ((int64_t)N + kRowPad - 1) / kRowPad * kRowPad;
  s->n_pad = n_pad;
  s->params = n_params(W, D, L_max);
  s->params_t = (int64_t)L_max * W * W + (int64_t)W * D;
  s->scratch = 3 * (int64_t)(L_max + 1) * W * n_pad + (int64_t)D * n_pad;
  s->target = n_pad * D;
  s->stats = D;
  s->loss_partial = (int64_t)epochs * (n_pad / 16);
  s->rows = n_pad;
  // split-K row slices for small groups: the largest power of two <= kMaxSplit
  // that leaves every slice an even number (>= 4) of 16-row blocks (the
  // workspace is sized for it; make_args may use fewer slices)
  const int64_t nb = n_pad / 16;
  int64_t sp = 1;
  while (sp < kMaxSplit && nb % (4 * sp) == 0 && nb / (2 * sp) >= 4) sp *= 2;
  s->grad_split = sp;
  // + one int32 arrival counter per parameter tile (the fused split step):
  // the most tiles any tiling of this shape has, rounded to 64 elements
  s->grad_partial = sp * s->params + split_ctr_elems(W, D, L_max);
  s->wsplit = xs_size(W, D, L_max);
}

// Split-K grid limit (see split_for).  Measured with 128 × 128 tiles
// (profiles/r02/ab_rows_ks.log "split 16"): one medium fit (14 tiles) 8 → 16
// slices −9 % parameter-kernel time; one wide fit at 8192 (60 tiles) 16
// slices +9 % (the grid passes 512 there).
constexpr int64_t kSplitGrid = 512;
inline int64_t param_tiles(int W, int D, int L, bool small) {   // ParamsCfg<W, D, X3, small>::tiles(L)
  const int T = small ? 64 : (W < 128 ? W : 128), nt = W / T, TD = D < T ? D : T;
  return (int64_t)L * nt * nt + (int64_t)(D / TD) * nt + W / 64;
}
// Row slices of a small group's split-K gradient reduction, and its tiles.
// A bf16x3 group with W >= 256 takes 64 × 64 tiles (ParamsCfg SMALL) when
// that grid still allows at least kSmallMinSplit slices: the split step's time
// is mostly its fixed costs and the partial-slab bytes (slices × params), and
// 3.1x the tiles reach the same grid with a quarter of the slices.  One
// medium fit at 2048: 44 tiles × 8 slices, parameter step 19.7 → 13.7 µs,
// config 2 0.0919 → 0.0846 ms per epoch; the wide fit at 8192 (216 small
// tiles would allow 2 slices) keeps 128 × 128 × 8, which measured 3.5 %
// faster than small tiles there (profiles/r03/split_small_tiles.log).
// Otherwise: the most slices the workspace allows (grad_split, <= 16) while
// fits × tiles × slices stays within kSplitGrid (two per CU).  Overrides:
// NERFHIP_GRAD_SPLIT_MAX caps the slices; NERFHIP_SPLIT_T128=1 keeps
// 128 × 128 tiles.
constexpr int64_t kSmallMinSplit = 8;
inline int32_t split_for(const nerfhip_group* g, const nerfhip_sizes& s, bool* small_tiles) {
  const char* e = getenv("NERFHIP_GRAD_SPLIT_MAX");
  const char* t128 = getenv("NERFHIP_SPLIT_T128");
  int64_t cap = s.grad_split;
  if (e)
    while (cap > 1 && cap > atoi(e)) cap /= 2;
  *small_tiles = false;
  if (g->precision == NERFHIP_PRECISION_BF16X3 && g->W >= 256 && !(t128 && t128[0] == '1')) {
    const int64_t grid = (int64_t)g->n_fits * param_tiles(g->W, g->D, g->L_max, true);
    int64_t sp = cap;
    while (sp > 2 && grid * sp > kSplitGrid) sp /= 2;
    if (sp >= kSmallMinSplit) {
      *small_tiles = true;
      return (int32_t)sp;
    }
  }
  if (e) return (int32_t)cap;
  int64_t sp = cap;
  const int64_t grid = (int64_t)g->n_fits * param_tiles(g->W, g->D, g->L_max);
  while (sp > 2 && grid * sp > kSplitGrid) sp /= 2;
  return (int32_t)sp;
}

// Row-step variant of a group.  The K-split kernel (k_step_rows_ks) gives a
// fit 4x the waves and a quarter of the serial GEMM chain per wave, at 4x the
// weight reads per row and one barrier per output tile: it pays only while the
// regular kernel leaves most CUs idle, i.e. for groups whose regular grid
// (n_fits · n_pad/64 workgroups) is at most kKsMaxWorkgroups.  Measured (rows
// kernel, bf16x3, medium): one fit at 1024 / 2048 / 4096 (16 / 32 / 64 regular
// workgroups) 0.093 → 0.066 ms each; two fits at 2048 (64) 0.093 → 0.068;
// three fits (96) 0.093 → 0.125; 8 fits 0.096 → 0.254; 5 large fits 0.29 →
// 0.62; one wide fit at 8192 (128) 0.36 → 0.59; one large fit at 2048 (32)
// 0.256 → 0.201 (profiles/r02/ks_threshold.log).  With the xoff_ks weight
// layout (round 3) the K-split kernel also wins at 128 regular workgroups
// (4 x 128 K-split workgroups, two rounds at one per CU), whole epochs of
// 200-epoch runs: one medium fit at 8192 0.139 → 0.133 ms, one wide fit at
// 8192 (config 5) 0.463 → 0.434, two medium at 4096 0.134 → 0.129, four at
// 2048 0.140 → 0.135, eight at 1024 0.180 → 0.168, sixteen at 512 0.159 →
// 0.148; at 256 it loses (eight medium at 2048 0.225 → 0.288;
// profiles/r03/ks_crossover.log).  NERFHIP_ROWS_KS = 0 / 1 forces the choice
// (supported shapes only: bf16x3, W >= 128, D = 128).
constexpr int64_t kKsMaxWorkgroups = 128;
inline bool rows_ks_for(const nerfhip_group* g, const nerfhip_sizes& s) {
  if (g->precision != NERFHIP_PRECISION_BF16X3 || g->W < 128 || g->D != 128) return false;
  const char* e = getenv("NERFHIP_ROWS_KS");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return (int64_t)g->n_fits * (s.n_pad / kRowPad) <= kKsMaxWorkgroups;
}

#endif  // NERFHIP_LAYOUT_H
