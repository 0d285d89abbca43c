// split_replay.cpp — CPU replay of every global-memory address the engine's
// kernels form for a set of group shapes, over exactly-sized heap buffers, so
// that AddressSanitizer flags any access outside the caller's allocations
// (the concurrent split-K fault).
//
// The index functions are the kernels' own (csrc/nerfhip_layout.h: weight
// layouts, parameter offsets, the XCD block map, ParamsCfg tiling, the
// staging slot order, fill_sizes / split_for / rows_ks_for).  The loops that
// walk blocks, waves, lanes and unrolled indices restate the kernels in
// csrc/nerfhip.hip, each next to the kernel it follows:
//   k_step_params (dw_tile / dw_tile_x3 + first layer)   nerfhip.hip k_step_params
//   k_adam_split + put_w                                 nerfhip.hip k_adam_split
//   k_step_rows (regular; LDS-DMA / register staging)    nerfhip.hip k_step_rows, gemm_phase*
//   k_step_rows_ks (K-split; KsPhase item loads)         nerfhip.hip k_step_rows_ks
//   k_transpose_params, k_normalize, k_row_metrics
// One epoch is replayed per group (every epoch forms the same addresses, up
// to the loss-partial row and the probe slot, which are replayed for the
// first and the last epoch).
//
// Input (stdin), one group per line:
//   W D N n_fits L_max precision(0 fp32 | 1 bf16x3) split(0|1) log_every L_0 L_1 ...
// Output: one line per group with the number of accesses replayed, then "OK".
// Build: g++ -std=c++17 -O1 -g -fsanitize=address,undefined -I include
//        -I nerf-attention_amd/csrc tools/r6/split_replay.cpp
#include <cstdio>
#include <cstring>
#include <vector>
#include <string>
#include <sstream>
#include <iostream>

#include "nerfhip.h"
#include "nerfhip_layout.h"

namespace {

long long g_acc = 0;

// an exactly-sized heap buffer; rd() / wr() are the only way in, so every
// replayed access is an ASan-checked heap access
template <class T>
struct Buf {
  T* p = nullptr;
  int64_t n = 0;
  const char* name;
  Buf(const char* nm, int64_t count) : n(count), name(nm) {
    p = new T[count > 0 ? count : 1];
    memset(p, 0, sizeof(T) * (count > 0 ? count : 1));
  }
  ~Buf() { delete[] p; }
  void rd(int64_t i, int len = 1) {
    for (int k = 0; k < len; ++k) {
      volatile T x = p[i + k];
      (void)x;
    }
    g_acc += len;
  }
  void wr(int64_t i, int len = 1) {
    for (int k = 0; k < len; ++k) p[i + k] = T(1);
    g_acc += len;
  }
};

struct Group {
  int W, D, N, n_fits, L_max, x3, split, log_every;
  std::vector<int> L;
};

struct Bufs {
  nerfhip_sizes s;
  Buf<float> pos, target, tnorm, mean, stdv, params, params_t, m, v, scratch, sched, loss,
      eval_y, row_cos, row_sq, gpart, probe_y, probe_rc, probe_rs;
  Buf<uint16_t> wsplit;
  Buf<int> layers;
  Buf<float> omega;
  Bufs(const Group& g, const nerfhip_sizes& z, int n_probe)
      : s(z),
        pos("positions", z.n_pad),
        target("target", g.n_fits * z.target),
        tnorm("target_norm", g.n_fits * z.target),
        mean("mean", g.n_fits * z.stats),
        stdv("std", g.n_fits * z.stats),
        params("params", g.n_fits * z.params),
        params_t("params_t", g.n_fits * z.params_t),
        m("adam_m", g.n_fits * z.params),
        v("adam_v", g.n_fits * z.params),
        scratch("scratch", g.n_fits * z.scratch),
        sched("sched", 2 * (int64_t)1),
        loss("loss_partial", g.n_fits * z.loss_partial),
        eval_y("eval_y", g.n_fits * z.target),
        row_cos("row_cos", g.n_fits * z.rows),
        row_sq("row_sq", g.n_fits * z.rows),
        gpart("grad_partial", g.split ? g.n_fits * z.grad_partial : 0),
        probe_y("probe_y", (int64_t)g.n_fits * n_probe * z.target),
        probe_rc("probe_row_cos", (int64_t)g.n_fits * n_probe * z.rows),
        probe_rs("probe_row_sq", (int64_t)g.n_fits * n_probe * z.rows),
        wsplit("wsplit", g.x3 ? g.n_fits * z.wsplit : 0),
        layers("fit_layers", g.n_fits),
        omega("fit_omega", g.n_fits) {}
};

// make_args' variant choices (nerfhip.hip make_args)
struct Plan {
  int n_split = 1, small_tiles = 0, rows_ks = 0, lay = kLayX;
};
Plan plan_of(const Group& g, const nerfhip_sizes& s) {
  nerfhip_group d{};
  d.W = g.W; d.D = g.D; d.N = g.N; d.n_fits = g.n_fits; d.L_max = g.L_max;
  d.precision = g.x3 ? NERFHIP_PRECISION_BF16X3 : NERFHIP_PRECISION_FP32;
  Plan p;
  bool small = false;
  p.n_split = (g.split && g.n_fits < kXcdMinFits) ? split_for(&d, s, &small) : 1;
  p.small_tiles = small && p.n_split > 1;
  p.rows_ks = rows_ks_for(&d, s) ? 1 : 0;
  p.lay = p.rows_ks ? kLayKs : kLayX;
  return p;
}
int fit_L(const Group& g, int fit) { return g.n_fits == 1 ? g.L_max : g.L[fit]; }

// put_w (nerfhip.hip): element M_i[j][k] into both split copies
void put_w(Bufs& B, int64_t xs0, int lay, int W, int D, int L, int i, int j, int k) {
  const int R = i <= L ? W : D;
  const int64_t f = xs_mat(W, D, L, false, i), b = xs_mat(W, D, L, true, i);
  for (int pl = 0; pl < 3; ++pl) {
    B.wsplit.wr(xs0 + f + xoff_any(lay, R, W, j, k, pl));
    B.wsplit.wr(xs0 + b + xoff_any(lay, W, R, k, j, pl));
  }
}

// ---- k_step_params: dw_tile_x3 / dw_tile -----------------------------------
template <int TJ, int TK, int NW, int WW, int OD>
void dw_tile_x3(Bufs& B, int lay, int64_t A, int FA, int64_t Bo, int FB, int j0, int k0, int rb0,
                int nb, bool G, int64_t gbase, int64_t pf, int64_t xs0, int64_t pw, int64_t pb,
                int64_t xf, int64_t xb, bool do_bias, int tid) {
  constexpr int NTH = 64 * NW, WK = NW / 2;
  constexpr int NA = TJ / 64, NB = TK / WK / 32;
  constexpr int NF4 = (TJ + TK) * 4, NPT = (NF4 + NTH - 1) / NTH;
  constexpr int NA4 = TJ * 4, NPA = (NA4 + NTH - 1) / NTH;
  constexpr int W = WW, kOD = OD;
  const int lane = tid & 63, wave = tid >> 6;
  const int wj = wave / WK, wk = wave % WK, h = lane >> 5, lr = lane & 31;
  const int64_t sA = (int64_t)FA * 16, sB = (int64_t)FB * 16;
  const int64_t Ab = A + (int64_t)j0 * 16 + rb0 * sA, Bb = Bo + (int64_t)k0 * 16 + rb0 * sB;
  for (int rb = 0; rb < nb; ++rb)            // every block gload() fetches (prefetch clamps)
    for (int m = 0; m < NPT; ++m) {
      const int i = tid + NTH * m;
      const int so = stage_slot<true>(i);
      if (NA4 % NTH == 0 ? m < NPA : i < NA4) B.scratch.rd(Ab + rb * sA + so * 4, 4);
      else if (NF4 % NTH == 0 || i < NF4) B.scratch.rd(Bb + rb * sB + (so - TJ * 4) * 4, 4);
    }
  for (int x = 0; x < NA; ++x)
    for (int y = 0; y < NB; ++y) {
      const int jrow0 = j0 + wj * (TJ / 2) + 32 * x;
      const int kcol = k0 + wk * (TK / WK) + 32 * y + lr;
      for (int qb = 0; qb < 4; ++qb) {
        for (int qq = 0; qq < 4; ++qq) {
          const int j = jrow0 + qq + 8 * qb + 4 * h;
          const int64_t idx = pw + (int64_t)j * W + kcol;
          if (G) { B.gpart.wr(gbase + idx); continue; }
          B.params.rd(pf + idx); B.m.rd(pf + idx); B.v.rd(pf + idx);
          B.params.wr(pf + idx); B.m.wr(pf + idx); B.v.wr(pf + idx);
          for (int pl = 0; pl < 3; ++pl) B.wsplit.wr(xs0 + xf + xoff_any(lay, kOD, W, j, kcol, pl));
        }
        if (!G) {
          const int jb = jrow0 + 8 * qb + 4 * h;
          for (int pl = 0; pl < 3; ++pl) B.wsplit.wr(xs0 + xb + xoff_any(lay, W, kOD, kcol, jb, pl), 4);
        }
      }
    }
  if (do_bias)
    for (int m = 0; m < NPA; ++m)
      if ((tid & 3) == 0 && tid + NTH * m < NA4) {
        const int64_t idx = pb + j0 + (stage_slot<true>(tid + NTH * m) >> 2);
        if (G) B.gpart.wr(gbase + idx);
        else { B.params.rd(pf + idx); B.params.wr(pf + idx); B.m.wr(pf + idx); B.v.wr(pf + idx); }
      }
}

template <int TJ, int TK, int NW>
void dw_tile(Bufs& B, int W, int64_t A, int FA, int64_t Bo, int FB, int j0, int k0, int rb0,
             int nb, bool G, int64_t gbase, int64_t pf, int64_t ptf, int64_t pw, int64_t pb,
             int64_t ptw, int out_dim, bool do_bias_tile, int tid) {
  constexpr int NTH = 64 * NW, WK = NW / 2;
  constexpr int NA = TJ / 64, NB = TK / WK / 32;
  constexpr int NF4 = (TJ + TK) * 4, NPT = (NF4 + NTH - 1) / NTH;
  const int lane = tid & 63, wave = tid >> 6;
  const int wj = wave / WK, wk = wave % WK, h = lane >> 5, lr = lane & 31;
  const int64_t sA = (int64_t)FA * 16, sB = (int64_t)FB * 16;
  const int64_t Ab = A + (int64_t)j0 * 16 + rb0 * sA, Bb = Bo + (int64_t)k0 * 16 + rb0 * sB;
  for (int rb = 0; rb < nb; ++rb)
    for (int m = 0; m < NPT; ++m) {
      const int i = tid + NTH * m;
      const int sl = stage_slot<false>(i);
      if (m < TJ * 4 / NTH) B.scratch.rd(Ab + rb * sA + sl * 4, 4);
      else if (NF4 % NTH == 0 || i < NF4) B.scratch.rd(Bb + rb * sB + (sl - TJ * 4) * 4, 4);
    }
  for (int x = 0; x < NA; ++x)
    for (int y = 0; y < NB; ++y) {
      const int jrow0 = j0 + wj * (TJ / 2) + 32 * x;
      const int kcol = k0 + wk * (TK / WK) + 32 * y + lr;
      for (int qb = 0; qb < 4; ++qb) {
        for (int qq = 0; qq < 4; ++qq) {
          const int j = jrow0 + qq + 8 * qb + 4 * h;
          const int64_t idx = pw + (int64_t)j * W + kcol;
          if (G) { B.gpart.wr(gbase + idx); continue; }
          B.params.rd(pf + idx); B.params.wr(pf + idx); B.m.wr(pf + idx); B.v.wr(pf + idx);
        }
        if (!G) B.params_t.wr(ptf + ptw + (int64_t)kcol * out_dim + jrow0 + 8 * qb + 4 * h, 4);
      }
    }
  if (do_bias_tile && wk == 0)
    for (int x = 0; x < NA; ++x)
      if (h == 0) {
        const int64_t idx = pb + j0 + wj * (TJ / 2) + 32 * x + lr;
        if (G) B.gpart.wr(gbase + idx);
        else { B.params.rd(pf + idx); B.params.wr(pf + idx); B.m.wr(pf + idx); B.v.wr(pf + idx); }
      }
}

template <int W, int D, bool X3, bool SMALL>
void k_step_params(const Group& g, Bufs& B, const Plan& p, int lay) {
  using C = ParamsCfg<W, D, X3, SMALL>;
  const nerfhip_sizes& s = B.s;
  const int nt = C::tiles(g.L_max);
  const int grid = grid_for(g.n_fits, nt * p.n_split);
  for (int b = 0; b < grid; ++b) {
    int fit, t;
    if (!map_block(b, g.n_fits, nt * p.n_split, fit, t)) continue;
    const int split = t / nt;
    t -= split * nt;
    if (fit < 0 || fit >= g.n_fits || split >= p.n_split) { fprintf(stderr, "bad block decode\n"); abort(); }
    B.layers.rd(fit);
    const int L = fit_L(g, fit);
    if (t >= C::tiles(L)) continue;
    const int nb = (int)(s.n_pad / 16 / p.n_split), rb0 = split * nb;
    const bool G = p.n_split > 1;
    const int64_t gbase = fit * s.grad_partial + split * s.params;
    const int64_t pf = fit * s.params, ptf = fit * s.params_t, xs0 = fit * s.wsplit;
    const int64_t S = fit * s.scratch, WN = (int64_t)W * s.n_pad;
    const int64_t SH = S, SZ = S + (int64_t)(g.L_max + 1) * WN, SG = S + 2 * (int64_t)(g.L_max + 1) * WN;
    B.sched.rd(0, 2);
    for (int tid = 0; tid < C::THREADS; ++tid) {
      if (t < L * C::TH) {
        const int layer = t / C::TH + 1, u = t % C::TH;
        const int64_t pw = off_hidden_w(W, layer);
        if constexpr (X3)
          dw_tile_x3<C::T, C::TK, C::NW, W, W>(B, lay, SZ + layer * WN, W, SH + (layer - 1) * WN, W,
                                              (u / C::NTK) * C::T, (u % C::NTK) * C::TK, rb0, nb, G,
                                              gbase, pf, xs0, pw, pw + (int64_t)W * W,
                                              xs_mat(W, D, L, false, layer), xs_mat(W, D, L, true, layer),
                                              (u % C::NTK) == 0, tid);
        else
          dw_tile<C::T, C::T, C::NW>(B, W, SZ + layer * WN, W, SH + (layer - 1) * WN, W,
                                     (u / C::NTK) * C::T, (u % C::NTK) * C::T, rb0, nb, G, gbase, pf,
                                     ptf, pw, pw + (int64_t)W * W, (int64_t)(layer - 1) * W * W, W,
                                     (u % C::NTK) == 0, tid);
      } else if (t < L * C::TH + C::TF) {
        const int u = t - L * C::TH;
        const int64_t pw = off_final_w(W, L);
        if constexpr (X3)
          dw_tile_x3<C::TD, C::TK, C::NW, W, D>(B, lay, SG, D, SH + L * WN, W, (u / C::NTK) * C::TD,
                                               (u % C::NTK) * C::TK, rb0, nb, G, gbase, pf, xs0, pw,
                                               pw + (int64_t)W * D, xs_mat(W, D, L, false, L + 1),
                                               xs_mat(W, D, L, true, L + 1), (u % C::NTK) == 0, tid);
        else
          dw_tile<C::TD, C::T, C::NW>(B, W, SG, D, SH + L * WN, W, (u / C::NTK) * C::TD,
                                      (u % C::NTK) * C::T, rb0, nb, G, gbase, pf, ptf, pw,
                                      pw + (int64_t)W * D, (int64_t)L * W * W, D, (u % C::NTK) == 0, tid);
      } else {
        const int u = t - L * C::TH - C::TF;
        const int lane = tid & 63, wave = tid >> 6, f = lane >> 2, m = lane & 3;
        const int j = u * (16 * C::NW) + wave * 16 + f;
        for (int rb = rb0 + m; rb < rb0 + nb; rb += 4) {
          B.scratch.rd(SZ + j + (int64_t)rb * 2 * W);
          B.scratch.rd(SZ + j + (int64_t)rb * 2 * W + W);
        }
        if (m == 0 && G) { B.gpart.wr(gbase + j); B.gpart.wr(gbase + W + j); }
        else if (m == 0) {
          B.params.rd(pf + j); B.params.wr(pf + j); B.m.wr(pf + j); B.v.wr(pf + j);
          B.params.rd(pf + W + j); B.params.wr(pf + W + j); B.m.wr(pf + W + j); B.v.wr(pf + W + j);
        }
      }
    }
  }
}

// ---- k_adam_split ------------------------------------------------------------
template <int W, int D>
void k_adam_split(const Group& g, Bufs& B, const Plan& p) {
  const nerfhip_sizes& s = B.s;
  const int gx = (int)((n_params(W, D, g.L_max) + 255) / 256);
  for (int fit = 0; fit < g.n_fits; ++fit) {
    B.layers.rd(fit);
    const int L = fit_L(g, fit);
    for (int bx = 0; bx < gx; ++bx)
      for (int tid = 0; tid < 256; ++tid) {
        const int64_t i = (int64_t)bx * 256 + tid;
        if (i >= n_params(W, D, L)) continue;
        for (int sp = 0; sp < p.n_split; ++sp) B.gpart.rd(fit * s.grad_partial + i + sp * s.params);
        const int64_t pf = fit * s.params;
        B.params.rd(pf + i); B.m.rd(pf + i); B.v.rd(pf + i);
        B.params.wr(pf + i); B.m.wr(pf + i); B.v.wr(pf + i);
        B.sched.rd(0, 2);
        const int64_t fw = off_final_w(W, L);
        if (i >= fw) {
          const int64_t r = i - fw;
          if (r < (int64_t)D * W) {
            if (g.x3) put_w(B, fit * s.wsplit, p.lay, W, D, L, L + 1, (int)(r / W), (int)(r % W));
            else B.params_t.wr(fit * s.params_t + (int64_t)L * W * W + (r % W) * D + r / W);
          }
        } else if (i >= 2 * W) {
          const int64_t r = (i - 2 * W) % ((int64_t)W * W + W);
          const int64_t layer = (i - 2 * W) / ((int64_t)W * W + W);
          if (r < (int64_t)W * W) {
            if (g.x3) put_w(B, fit * s.wsplit, p.lay, W, D, L, (int)layer + 1, (int)(r / W), (int)(r % W));
            else B.params_t.wr(fit * s.params_t + layer * W * W + (r % W) * W + r / W);
          }
        }
      }
  }
}

// ---- k_step_rows (regular) -------------------------------------------------------
// weight staging of one GEMM phase, gemm_phase_x3 (LDS-DMA) / gemm_phase
template <int K, int JT, int NTH>
void phase_loads(Bufs& B, bool x3, int64_t src_elems, int tid) {
  if (x3) {
    constexpr int KC = kc_of(K), NH = K / KC, U = JT * NH, SR = KC / 8;
    constexpr int SWM = (SR < 16 ? SR : 16) - 1;
    constexpr int SL = 3 * 16 * SR, NPT = (SL + NTH - 1) / NTH;
    constexpr int S_ROWS = NTH / SR, P = S_ROWS >= 16 ? 1 : 16 / S_ROWS;
    const int wave = tid >> 6;
    int soff[P];
    for (int m = 0; m < P; ++m) {
      const int i = tid + NTH * m;
      const int row = (i / SR) & 15, pl = i / (16 * SR), ps = i % SR;
      soff[m] = (pl * 16 + row) * KC + 8 * (ps ^ (row & SWM));
    }
    (void)SWM;
    for (int u = 0; u < U; ++u)
      for (int m = 0; m < NPT; ++m)
        if (SL % NTH == 0 || NTH * m + 64 * wave < SL) {
          // the DMA's byte offset (voffset + soffset), 16 B per lane, from the
          // phase's source: 2·soff + u·96·KC + 2·(m/P)·P·S_ROWS·KC
          const int64_t byte = 2 * (int64_t)soff[m % P] + (int64_t)u * 96 * KC +
                               2 * (int64_t)(m / P) * P * S_ROWS * KC;
          B.wsplit.rd(src_elems + byte / 2, 8);
        }
  } else {
    constexpr int C4 = K / 4, NF4 = 16 * C4, NPT = (NF4 + NTH - 1) / NTH;
    for (int chunk = 0; chunk < JT; ++chunk)
      for (int m = 0; m < NPT; ++m) {
        const int i = tid + NTH * m;
        if (NF4 % NTH == 0 || i < NF4) B.params.rd(src_elems + (int64_t)chunk * 16 * K + (i / C4) * K + (i % C4) * 4, 4);
      }
  }
}
// the same, for the params_t (transposed fp32) source
template <int K, int JT, int NTH>
void phase_loads_pt(Bufs& B, int64_t src, int tid) {
  constexpr int C4 = K / 4, NF4 = 16 * C4, NPT = (NF4 + NTH - 1) / NTH;
  for (int chunk = 0; chunk < JT; ++chunk)
    for (int m = 0; m < NPT; ++m) {
      const int i = tid + NTH * m;
      if (NF4 % NTH == 0 || i < NF4) B.params_t.rd(src + (int64_t)chunk * 16 * K + (i / C4) * K + (i % C4) * 4, 4);
    }
}

template <int W> struct RowsCfgR {   // RowsCfg (nerfhip.hip)
  static constexpr int NSPLIT = W >= 512 ? 2 : 1, NWAVES = 4, THREADS = 256, ROWS = 64;
};

template <int W, int D>
void k_step_rows(const Group& g, Bufs& B, bool train, int64_t y_out_base, int64_t y_stride,
                 bool probe, int epoch) {
  const nerfhip_sizes& s = B.s;
  constexpr int NWV = RowsCfgR<W>::NWAVES, NTH = RowsCfgR<W>::THREADS;
  constexpr int JW = W / 16, JD = D / 16, NS = RowsCfgR<W>::NSPLIT, JP = JW / NS;
  const int tiles = (int)(s.n_pad / RowsCfgR<W>::ROWS);
  const int grid = grid_for(g.n_fits, tiles);
  const int64_t WN = (int64_t)W * s.n_pad;
  for (int b = 0; b < grid; ++b) {
    int fit, tile;
    if (!map_block(b, g.n_fits, tiles, fit, tile)) continue;
    B.layers.rd(fit);
    B.omega.rd(fit);
    const int L = fit_L(g, fit);
    const int64_t P = fit * s.params, PT = fit * s.params_t, S = fit * s.scratch;
    const int64_t SH = S, SZ = S + (int64_t)(g.L_max + 1) * WN;
    const int64_t SG = S + 2 * (int64_t)(g.L_max + 1) * WN, SC = SG + (int64_t)D * s.n_pad;
    const int64_t XS = fit * s.wsplit;
    auto wsrc = [&](bool bwd, int i) -> int64_t {   // element offset in wsplit / params / params_t
      if (g.x3) return XS + xs_mat(W, D, L, bwd, i);
      if (bwd) return PT + (int64_t)(i - 1) * W * W;
      return i <= L ? P + off_hidden_w(W, i) : P + off_final_w(W, L);
    };
    for (int tid = 0; tid < NTH; ++tid) {
      const int lane = tid & 63, wave = tid >> 6, c = lane & 15, gg = lane >> 4;
      const int rblk = tile * NWV + wave, r = rblk * 16 + c;
      const int tq = gg * 64 + (c & 3) * 16 + (c >> 2) * 4;
      const int64_t SHt = SH + (int64_t)rblk * W * 16 + tq, SZt = SZ + (int64_t)rblk * W * 16 + tq;
      const int64_t SGt = SG + (int64_t)rblk * D * 16 + tq;
      auto wide_loads = [&](int64_t src, int K, bool bwd_pt) {
        for (int p = 0; p < NS; ++p) {
          if (g.x3) {
            const int64_t off = src + (int64_t)p * JP * K * 96 / 2;   // bytes → bf16 elements
            if (K == W) phase_loads<W, JP, NTH>(B, true, off, tid);
            else phase_loads<D, JP, NTH>(B, true, off, tid);
          } else {
            const int64_t off = src + (int64_t)p * JP * K * 64 / 4;   // bytes → floats
            if (bwd_pt) {
              if (K == W) phase_loads_pt<W, JP, NTH>(B, off, tid);
              else phase_loads_pt<D, JP, NTH>(B, off, tid);
            } else if (K == W) phase_loads<W, JP, NTH>(B, false, off, tid);
            else phase_loads<D, JP, NTH>(B, false, off, tid);
          }
        }
      };
      if (4 * tid < 2 * W) B.params.rd(P + 4 * tid, 4);            // stage_vec(w0 ‖ b0)
      B.pos.rd(r);
      for (int J = 0; J < JW; ++J)
        if (train) B.scratch.wr(SHt + J * 256, 4);
      for (int i = 1; i <= L; ++i) {
        if (4 * tid < W) B.params.rd(P + off_hidden_w(W, i) + (int64_t)W * W + 4 * tid, 4);
        wide_loads(wsrc(false, i), W, false);
        const int64_t SCi = SC + (int64_t)i * WN + (int64_t)rblk * JW * 256 + lane * 4;
        for (int J = 0; J < JW; ++J)
          if (train) {
            B.scratch.wr(SCi + J * 256, 4);
            B.scratch.wr(SHt + i * WN + J * 256, 4);
          }
      }
      if (4 * tid < D) B.params.rd(P + off_final_w(W, L) + (int64_t)W * D + 4 * tid, 4);
      if (g.x3) phase_loads<W, JD, NTH>(B, true, wsrc(false, L + 1), tid);
      else phase_loads<W, JD, NTH>(B, false, wsrc(false, L + 1), tid);
      for (int J = 0; J < JD; ++J) {
        if (train) B.tnorm.rd(fit * s.target + (int64_t)r * D + 4 * gg + 16 * J, 4);
        if (y_out_base >= 0) {
          const int64_t yo = y_out_base + fit * y_stride + (int64_t)r * D + 4 * gg + 16 * J;
          if (probe) B.probe_y.wr(yo, 4); else B.eval_y.wr(yo, 4);
        }
        if (train) B.scratch.wr(SGt + J * 256, 4);
      }
      if (!train) continue;
      if (lane == 0) B.loss.wr(fit * s.loss_partial + (int64_t)epoch * (s.n_pad / 16) + rblk);
      auto cos_reads = [&](int layer) {
        const int64_t SCl = SC + (int64_t)layer * WN + (int64_t)rblk * JW * 256 + lane * 4;
        for (int K = 0; K < JW; ++K) B.scratch.rd(SCl + K * 256, 4);
      };
      wide_loads(wsrc(true, L + 1), D, true);
      cos_reads(L);
      for (int K = 0; K < JW; ++K) B.scratch.wr(SZt + L * WN + K * 256, 4);
      for (int i = L; i >= 2; --i) {
        wide_loads(wsrc(true, i), W, true);
        cos_reads(i - 1);
        for (int K = 0; K < JW; ++K) B.scratch.wr(SZt + (i - 1) * WN + K * 256, 4);
      }
      if (4 * tid < 2 * W) B.params.rd(P + 4 * tid, 4);
      wide_loads(wsrc(true, 1), W, true);
      const int64_t PZ = SZ + (int64_t)rblk * 2 * W;
      for (int K = 0; K < JW; ++K)
        if (!(c & 1)) {
          const int idx = c >> 1;
          B.scratch.wr(PZ + (idx >> 2) * W + 16 * K + 4 * gg + (idx & 3));
        }
    }
  }
}

// ---- k_step_rows_ks (K-split) ---------------------------------------------------------
template <int W, int D, int PD>
void k_step_rows_ks(const Group& g, Bufs& B, bool train, int64_t y_out_base, int64_t y_stride,
                    bool probe, int epoch) {
  const nerfhip_sizes& s = B.s;
  constexpr int JW = W / 16, JD = D / 16, NO = W / 64;
  const int nblk = (int)(s.n_pad / 16);
  const int grid = grid_for(g.n_fits, nblk);
  const int64_t WN = (int64_t)W * s.n_pad;
  for (int b = 0; b < grid; ++b) {
    int fit, rblk;
    if (!map_block(b, g.n_fits, nblk, fit, rblk)) continue;
    B.layers.rd(fit);
    B.omega.rd(fit);
    const int L = fit_L(g, fit);
    const int64_t P = fit * s.params, S = fit * s.scratch, XS = fit * s.wsplit;
    const int64_t SH = S, SZ = S + (int64_t)(g.L_max + 1) * WN;
    const int64_t SG = S + 2 * (int64_t)(g.L_max + 1) * WN, SC = SG + (int64_t)D * s.n_pad;
    for (int tid = 0; tid < 256; ++tid) {
      const int lane = tid & 63, w = tid >> 6, c = lane & 15, gg = lane >> 4;
      const int r = rblk * 16 + c, fe = 4 * gg + w;
      const int64_t eoff = (int64_t)rblk * W * 16 + fe * 16 + c;
      const int64_t coff = (int64_t)rblk * JW * 256 + w * 64 + lane;
      // KsPhase<K>::load<I>: three 16-B plane loads at byte v = 2·base + voff
      auto phase = [&](int K, int JT, int mat) {
        const int NS = K / 32, NM = K / 128;
        const int64_t voff = 64 * c + 16 * gg + 3072 * w + 2 * (int64_t)mat;
        for (int I = 0; I < JT * NM; ++I) {
          const int J = I / NM, m = I % NM;
          const int64_t base = (int64_t)(J * NS + 4 * m) * 3 * 512;
          for (int pl = 0; pl < 3; ++pl) B.wsplit.rd(XS + (2 * base + voff + 1024 * pl) / 2, 8);
        }
      };
      auto prefetch = [&](int K, int mat) {    // the next phase's first PD items
        const int NS = K / 32, NM = K / 128;
        const int64_t voff = 64 * c + 16 * gg + 3072 * w + 2 * (int64_t)mat;
        for (int I = 0; I < PD; ++I) {
          const int J = I / NM, m = I % NM;
          const int64_t base = (int64_t)(J * NS + 4 * m) * 3 * 512;
          for (int pl = 0; pl < 3; ++pl) B.wsplit.rd(XS + (2 * base + voff + 1024 * pl) / 2, 8);
        }
      };
      auto xm = [&](bool bwd, int i) { return xs_mat(W, D, L, bwd, i); };
      // ks_stage<N>: waves w < WAVES copy E consecutive floats per lane
      auto ks_stage = [&](int N, int64_t src) {
        const int WAVES = N >= 256 ? 4 : N / 64, E = N / (64 * WAVES);
        if (w < WAVES) B.params.rd(src + (int64_t)(w * 64 + lane) * E, E);
      };
      prefetch(W, (int)xm(false, 1));
      // ks_stage<2W>: every lane of every wave copies 2W/256 floats
      ks_stage(2 * W, P);
      B.pos.rd(r);
      const int64_t SHt = SH + (int64_t)rblk * W * 16 + gg * 64 + (c & 3) * 16 + (c >> 2) * 4;
      for (int t = 0; t < NO; ++t) {
        const int J = 2 * (w + 4 * (t >> 1)) + (t & 1);
        if (train) B.scratch.wr(SHt + J * 256, 4);
      }
      for (int i = 1; i <= L; ++i) {
        ks_stage(W, P + off_hidden_w(W, i) + (int64_t)W * W);
        phase(W, JW, (int)xm(false, i));
        prefetch(W, (int)xm(false, i + 1));   // (i = L: the final matrix, K = W too)
        for (int J = 0; J < JW; ++J)
          if (train) {
            B.scratch.wr(SH + i * WN + eoff + J * 256);
            B.scratch.wr(SC + i * WN + coff + J * 256);
          }
      }
      ks_stage(D, P + off_final_w(W, L) + (int64_t)W * D);
      phase(W, JD, (int)xm(false, L + 1));
      if (train) prefetch(D, (int)xm(true, L + 1));   // W_fᵀ is [W][D]: K = D
      for (int J = 0; J < JD; ++J) {
        if (train) B.tnorm.rd(fit * s.target + (int64_t)r * D + fe + 16 * J);
        if (y_out_base >= 0) {
          const int64_t yo = y_out_base + fit * y_stride + (int64_t)r * D + fe + 16 * J;
          if (probe) B.probe_y.wr(yo); else B.eval_y.wr(yo);
        }
        if (train) B.scratch.wr(SG + (int64_t)rblk * D * 16 + fe * 16 + c + J * 256);
      }
      if (!train) continue;
      auto bwd = [&](int K, int mat, int layer, int next) {
        phase(K, JW, mat);
        if (next >= 0) prefetch(W, next);
        for (int J = 0; J < JW; ++J) {
          B.scratch.rd(SC + layer * WN + coff + J * 256);
          B.scratch.wr(SZ + layer * WN + eoff + J * 256);
        }
      };
      bwd(D, (int)xm(true, L + 1), L, (int)xm(true, L));
      for (int i = L; i >= 2; --i) bwd(W, (int)xm(true, i), i - 1, (int)xm(true, i - 1));
      ks_stage(2 * W, P);
      phase(W, JW, (int)xm(true, 1));
      const int64_t PZ = SZ + (int64_t)rblk * 2 * W;
      for (int J = 0; J < JW; ++J) {
        const int f = 16 * J + fe;
        B.scratch.wr(c == 1 ? PZ + W + f : PZ + f);
      }
      if (w == 0) B.loss.wr(fit * s.loss_partial + (int64_t)epoch * (s.n_pad / 16) + rblk);
    }
  }
}

// ---- prologue / epilogue kernels -----------------------------------------------------
void k_transpose_params(const Group& g, Bufs& B, int lay) {
  const nerfhip_sizes& s = B.s;
  for (int fit = 0; fit < g.n_fits; ++fit) {
    const int L = fit_L(g, fit), W = g.W, D = g.D;
    const int64_t nh = (int64_t)L * W * W, total = nh + (int64_t)W * D;
    for (int64_t e = 0; e < total; ++e) {
      if (e < nh) {
        const int64_t i = e / ((int64_t)W * W), u = e % ((int64_t)W * W), k = u / W, j = u % W;
        B.params.rd(fit * s.params + off_hidden_w(W, (int)i + 1) + j * W + k);
        if (!g.x3) B.params_t.wr(fit * s.params_t + e);
        else put_w(B, fit * s.wsplit, lay, W, D, L, (int)i + 1, (int)j, (int)k);
      } else {
        const int64_t u = e - nh, k = u / D, j = u % D;
        B.params.rd(fit * s.params + off_final_w(W, L) + j * W + k);
        if (!g.x3) B.params_t.wr(fit * s.params_t + e);
        else put_w(B, fit * s.wsplit, lay, W, D, L, L + 1, (int)j, (int)k);
      }
    }
  }
}
void k_normalize(const Group& g, Bufs& B) {
  const nerfhip_sizes& s = B.s;
  for (int fit = 0; fit < g.n_fits; ++fit)
    for (int j = 0; j < g.D; ++j) {
      for (int r = 0; r < g.N; ++r) B.target.rd(fit * s.target + (int64_t)r * g.D + j);
      B.mean.wr(fit * g.D + j);
      B.stdv.wr(fit * g.D + j);
      for (int r = 0; r < s.n_pad; ++r) B.tnorm.wr(fit * s.target + (int64_t)r * g.D + j);
    }
}
void k_row_metrics(const Group& g, Bufs& B, Buf<float>& y, int64_t y0, int64_t ystride,
                   Buf<float>& rc, Buf<float>& rs, int64_t r0, int64_t rstride) {
  const nerfhip_sizes& s = B.s;
  for (int fit = 0; fit < g.n_fits; ++fit)
    for (int r = 0; r < s.n_pad; ++r) {
      rc.wr(r0 + fit * rstride + r);
      rs.wr(r0 + fit * rstride + r);
      if (r >= g.N) continue;
      for (int j = 0; j < g.D; ++j) {
        y.rd(y0 + fit * ystride + (int64_t)r * g.D + j);
        B.target.rd(fit * s.target + (int64_t)r * g.D + j);
        B.mean.rd(fit * g.D + j);
        B.stdv.rd(fit * g.D + j);
      }
    }
}

template <int W, int D>
void replay_wd(const Group& g) {
  nerfhip_sizes s;
  const int E = 2;   // epochs replayed: the first and the last loss row
  fill_sizes(W, D, g.N, g.L_max, E, &s);
  const int n_probe = g.log_every > 0 ? E / g.log_every : 0;
  Bufs B(g, s, n_probe);
  const Plan p = plan_of(g, s);
  const long long a0 = g_acc;
  k_normalize(g, B);
  k_transpose_params(g, B, p.lay);
  for (int e = 0; e < E; ++e) {
    const bool pr = n_probe > 0 && (e + 1) % g.log_every == 0;
    const int64_t ybase = pr ? (int64_t)((e + 1) / g.log_every - 1) * s.target : -1;
    const int64_t ystr = (int64_t)n_probe * s.target;
    if constexpr (W >= 128 && D == 128) {
      if (g.x3 && p.rows_ks) k_step_rows_ks<W, D, W >= 512 ? 8 : 6>(g, B, true, ybase, ystr, pr, e);
      else k_step_rows<W, D>(g, B, true, ybase, ystr, pr, e);
    } else {
      k_step_rows<W, D>(g, B, true, ybase, ystr, pr, e);
    }
    if (g.x3) {
      if (W >= 256 && p.small_tiles) k_step_params<W, D, true, true>(g, B, p, kLayX);
      else k_step_params<W, D, true, false>(g, B, p, p.n_split == 1 ? p.lay : kLayX);
    } else {
      k_step_params<W, D, false, false>(g, B, p, kLayX);
    }
    if (p.n_split > 1) k_adam_split<W, D>(g, B, p);
  }
  // final evaluation + metrics (mode 1), then the probes' metrics
  if constexpr (W >= 128 && D == 128) {
    if (g.x3 && p.rows_ks) k_step_rows_ks<W, D, W >= 512 ? 8 : 6>(g, B, false, 0, s.target, false, 0);
    else k_step_rows<W, D>(g, B, false, 0, s.target, false, 0);
  } else {
    k_step_rows<W, D>(g, B, false, 0, s.target, false, 0);
  }
  k_row_metrics(g, B, B.eval_y, 0, s.target, B.row_cos, B.row_sq, 0, s.rows);
  for (int k = 0; k < n_probe; ++k)
    k_row_metrics(g, B, B.probe_y, k * s.target, (int64_t)n_probe * s.target, B.probe_rc, B.probe_rs,
                  k * s.rows, (int64_t)n_probe * s.rows);
  printf("group W=%d D=%d N=%d fits=%d L_max=%d %s split=%d (slices %d, %s tiles) rows=%s: %lld accesses\n",
         W, D, g.N, g.n_fits, g.L_max, g.x3 ? "bf16x3" : "fp32", g.split, p.n_split,
         p.small_tiles ? "64x64" : "regular", p.rows_ks ? "ksplit" : "regular", g_acc - a0);
}

template <int W>
void replay_w(const Group& g) {
  if (g.D == 64) replay_wd<W, 64>(g);
  else replay_wd<W, 128>(g);
}

}  // namespace

int main() {
  // self-test of the harness: one write one element past a buffer must be
  // reported by ASan (tests/test_split_replay.py)
  if (const char* e = getenv("NERFHIP_REPLAY_SELFTEST"))
    if (e[0] == '1') {
      Buf<float> b("selftest", 16);
      b.wr(16);
    }
  std::string line;
  int n = 0;
  while (std::getline(std::cin, line)) {
    if (line.empty() || line[0] == '#') continue;
    std::istringstream in(line);
    Group g;
    in >> g.W >> g.D >> g.N >> g.n_fits >> g.L_max >> g.x3 >> g.split >> g.log_every;
    int l;
    while (in >> l) g.L.push_back(l);
    if ((int)g.L.size() != g.n_fits) { fprintf(stderr, "need one depth per fit: %s\n", line.c_str()); return 2; }
    switch (g.W) {
      case 64: replay_w<64>(g); break;
      case 128: replay_w<128>(g); break;
      case 256: replay_w<256>(g); break;
      case 512: replay_w<512>(g); break;
      default: fprintf(stderr, "bad W %d\n", g.W); return 2;
    }
    ++n;
  }
  printf("OK %d groups, %lld accesses\n", n, g_acc);
  return 0;
}
