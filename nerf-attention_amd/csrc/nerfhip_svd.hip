// nerfhip_svd.hip — MI355X (gfx950) truncated-SVD baseline of the KV slices.
//
// Replaces the per-tensor CPU loop of the reference's SVD baseline
// (nerf_attention/experiments/svd.py:43-75): for every (layer, head, K|V)
// slice X [N × D] and every target compression, the rank-r reconstruction
// U_r·diag(S_r)·V_rᵀ and its per-row cosine similarity with X (svd.py:53-57).
//
// MI355X-first restatement, one batch of slices per call:
//   k_svd_gram     G = XᵀX in fp64 (the fp32 products are exact in fp64), one
//                  workgroup per (slice, 64×64 tile of G), X staged through LDS
//   k_svd_jacobi   cyclic two-sided Jacobi eigen-solver of G, one workgroup per
//                  slice: G lives in LDS (fp64, padded rows), the D/2 disjoint
//                  rotations of a round-robin round are applied in parallel
//                  (columns, then rows), V accumulates in global memory (L2);
//                  eigenvalues σ² sorted descending → the right singular
//                  vectors of X
//   k_svd_project  per row i: y = X_i·V (fp64); since the rank-r
//                  reconstruction is the orthogonal projection of X_i onto
//                  span(V_r), its cosine with X_i is ‖y_{<r}‖ / ‖X_i‖
//                  (F.cosine_similarity, svd.py:57), for every requested r
//   k_svd_stats    mean, min and unbiased std of each rank's row cosines
//                  (svd.py:67-69), fp64 reductions
// The Gram route squares the condition number; in fp64 that still resolves
// the dominant subspace to far below the fp32 rounding of the reference's own
// LAPACK sgesdd path (parity: tests/test_svd.py against the reference's
// svd_results.json).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "nerfhip.h"

namespace {

constexpr int kThreads = 256;

// ---- G = XᵀX ---------------------------------------------------------------
// grid (tiles, n_tensors); tile = (bi, bj) 64×64 block with bi <= bj.  Each
// thread owns a 4×4 patch; X rows are staged 32 at a time (both 64-column
// panels) through LDS.
template <int D>
__global__ void __launch_bounds__(kThreads) k_svd_gram(const float* __restrict__ X, int N,
                                                       double* __restrict__ G) {
  constexpr int NB = D / 64;
  constexpr int RB = 32;                       // rows per stage
  __shared__ float sa[RB][64 + 1], sb[RB][64 + 1];
  int t = blockIdx.x, bi = 0;
  while (t >= NB - bi) { t -= NB - bi; ++bi; }   // upper-triangle tile index → (bi, bj)
  const int bj = bi + t;
  const int ten = blockIdx.y;
  const float* x = X + (int64_t)ten * N * D;
  const int tid = threadIdx.x, ti = tid / 16, tj = tid % 16;   // 16×16 threads, 4×4 each
  double acc[4][4] = {};
  for (int r0 = 0; r0 < N; r0 += RB) {
    for (int e = tid; e < RB * 64; e += kThreads) {
      const int rr = e / 64, cc = e % 64, row = r0 + rr;
      sa[rr][cc] = row < N ? x[(int64_t)row * D + bi * 64 + cc] : 0.f;
      sb[rr][cc] = row < N ? x[(int64_t)row * D + bj * 64 + cc] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int rr = 0; rr < RB; ++rr) {
      double a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = (double)sa[rr][ti * 4 + u];
        b[u] = (double)sb[rr][tj * 4 + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = fma(a[u], b[v], acc[u][v]);
    }
    __syncthreads();
  }
  double* g = G + (int64_t)ten * D * D;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = bi * 64 + ti * 4 + u, j = bj * 64 + tj * 4 + v;
      g[(int64_t)i * D + j] = acc[u][v];
      g[(int64_t)j * D + i] = acc[u][v];
    }
}

// ---- eigen-decomposition of G (symmetric, D×D) --------------------------------
// Round-robin schedule: in round t the D/2 pairs (a_k, b_k) are disjoint and
// every pair (p, q) appears once per sweep of D−1 rounds.
__device__ __forceinline__ void rr_pair(int D, int t, int k, int& p, int& q) {
  const int a = k == 0 ? 0 : ((k - 1 + t) % (D - 1)) + 1;
  const int b = ((D - 2 - k + t) % (D - 1)) + 1;
  p = a < b ? a : b;
  q = a < b ? b : a;
}

// G is read into LDS and its buffer then reused for Vᵀ (row p = column p of V,
// so a rotation of columns p, q of V touches two contiguous rows: coalesced).
template <int D>
__global__ void __launch_bounds__(kThreads) k_svd_jacobi(double* __restrict__ G,
                                                         double* __restrict__ evec,
                                                         double* __restrict__ evals,
                                                         int32_t* __restrict__ order,
                                                         int max_sweeps) {
  constexpr int LD = D + 1;                   // padded fp64 rows
  constexpr int NP = D / 2;
  __shared__ double A[D * LD];
  __shared__ double cs[NP], sn[NP];
  __shared__ int pp[NP], qq[NP];
  __shared__ double red[kThreads / 64 * 2];
  const int ten = blockIdx.x, tid = threadIdx.x;
  double* vt = G + (int64_t)ten * D * D;
  for (int e = tid; e < D * D; e += kThreads) A[(e / D) * LD + e % D] = vt[e];
  __syncthreads();
  for (int e = tid; e < D * D; e += kThreads) vt[e] = (e / D == e % D) ? 1.0 : 0.0;
  __syncthreads();
  for (int sweep = 0; sweep < max_sweeps; ++sweep) {
    // convergence: off-diagonal mass against the diagonal (relative 1e-30 in squares)
    double off = 0.0, dia = 0.0;
    for (int e = tid; e < D * D; e += kThreads) {
      const int i = e / D, j = e % D;
      const double a = A[i * LD + j];
      if (i == j) dia += a * a;
      else off += a * a;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      off += __shfl_xor(off, o, 64);
      dia += __shfl_xor(dia, o, 64);
    }
    if ((tid & 63) == 0) {
      red[tid / 64] = off;
      red[kThreads / 64 + tid / 64] = dia;
    }
    __syncthreads();
    double offs = 0.0, dias = 0.0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
      offs += red[w];
      dias += red[kThreads / 64 + w];
    }
    __syncthreads();
    if (offs <= 1e-30 * dias) break;             // uniform across the block
    for (int t = 0; t < D - 1; ++t) {
      if (tid < NP) {
        int p, q;
        rr_pair(D, t, tid, p, q);
        const double app = A[p * LD + p], aqq = A[q * LD + q], apq = A[p * LD + q];
        double c = 1.0, s = 0.0;
        if (apq != 0.0 && fabs(apq) > 1e-300) {
          const double tau = (aqq - app) / (2.0 * apq);
          const double tt = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
          c = 1.0 / sqrt(1.0 + tt * tt);
          s = tt * c;
        }
        cs[tid] = c;
        sn[tid] = s;
        pp[tid] = p;
        qq[tid] = q;
      }
      __syncthreads();
      // A ← A·J and V ← V·J: columns p, q of every row (rows p, q of Vᵀ)
      for (int e = tid; e < NP * D; e += kThreads) {
        const int k = e / D, i = e % D;
        const int p = pp[k], q = qq[k];
        const double c = cs[k], s = sn[k];
        const double x = A[i * LD + p], y = A[i * LD + q];
        A[i * LD + p] = c * x - s * y;
        A[i * LD + q] = s * x + c * y;
        const double vx = vt[(int64_t)p * D + i], vy = vt[(int64_t)q * D + i];
        vt[(int64_t)p * D + i] = c * vx - s * vy;
        vt[(int64_t)q * D + i] = s * vx + c * vy;
      }
      __syncthreads();
      // A ← Jᵀ·A: rows p, q of every column
      for (int e = tid; e < NP * D; e += kThreads) {
        const int k = e / D, j = e % D;
        const int p = pp[k], q = qq[k];
        const double c = cs[k], s = sn[k];
        const double x = A[p * LD + j], y = A[q * LD + j];
        A[p * LD + j] = c * x - s * y;
        A[q * LD + j] = s * x + c * y;
      }
      __syncthreads();
    }
  }
  // eigenvalues in descending order (ties by index); eigenvector rows sorted alike
  __shared__ int rank_of[D];
  for (int k = tid; k < D; k += kThreads) {
    const double lk = A[k * LD + k];
    int rank = 0;
    for (int j = 0; j < D; ++j) {
      const double lj = A[j * LD + j];
      rank += (lj > lk) || (lj == lk && j < k);
    }
    evals[(int64_t)ten * D + rank] = lk;
    order[(int64_t)ten * D + rank] = k;
    rank_of[k] = rank;
  }
  __syncthreads();
  double* ev = evec + (int64_t)ten * D * D;
  for (int e = tid; e < D * D; e += kThreads) ev[(int64_t)rank_of[e / D] * D + e % D] = vt[e];
}

// ---- per-row cosines of the rank-r reconstructions ------------------------------
struct ProjArgs {
  int32_t n_ranks;
  int32_t ranks[NERFHIP_SVD_MAX_RANKS];
};

template <int D>
__global__ void __launch_bounds__(kThreads) k_svd_project(const float* __restrict__ X, int N,
                                                          const double* __restrict__ evec,
                                                          ProjArgs pa, float* __restrict__ cosv) {
  constexpr int KC = 16;                      // eigenvectors per pass
  __shared__ double vs[D * KC];               // eigenvectors k0..k0+KC, [j][kk]
  const int ten = blockIdx.y, tid = threadIdx.x;
  const int i = blockIdx.x * kThreads + tid;
  const float* x = X + ((int64_t)ten * N + (i < N ? i : 0)) * D;
  const double* ev = evec + (int64_t)ten * D * D;   // row k = k-th eigenvector (descending)
  double xx = 0.0;
  for (int j = 0; j < D; ++j) xx = fma((double)x[j], (double)x[j], xx);
  double cum = 0.0;
  double proj[NERFHIP_SVD_MAX_RANKS];
#pragma unroll
  for (int r = 0; r < NERFHIP_SVD_MAX_RANKS; ++r) proj[r] = 0.0;
  for (int k0 = 0; k0 < D; k0 += KC) {
    __syncthreads();
    for (int e = tid; e < D * KC; e += kThreads) {
      const int kk = e / D, j = e % D;
      vs[j * KC + kk] = ev[(int64_t)(k0 + kk) * D + j];
    }
    __syncthreads();
    double y[KC];
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) y[kk] = 0.0;
    for (int j = 0; j < D; ++j) {
      const double xj = (double)x[j];
#pragma unroll
      for (int kk = 0; kk < KC; ++kk) y[kk] = fma(xj, vs[j * KC + kk], y[kk]);
    }
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      cum = fma(y[kk], y[kk], cum);
#pragma unroll
      for (int r = 0; r < NERFHIP_SVD_MAX_RANKS; ++r)
        if (r < pa.n_ranks && pa.ranks[r] == k0 + kk + 1) proj[r] = cum;
    }
  }
  if (i >= N) return;
  // cos(rec, x) = rec·x / (‖rec‖‖x‖) = ‖Px‖² / (‖Px‖‖x‖); ε as F.cosine_similarity (1e-8)
  const double nx = sqrt(xx);
  for (int r = 0; r < pa.n_ranks; ++r) {
    const double np = sqrt(proj[r]);
    const double den = fmax(np * nx, 1e-8);
    cosv[((int64_t)ten * pa.n_ranks + r) * N + i] = (float)(proj[r] / den);
  }
}

// mean, min, unbiased std over the N row cosines of one (slice, rank)
__global__ void __launch_bounds__(kThreads) k_svd_stats(const float* __restrict__ cosv, int N,
                                                        double* __restrict__ stats) {
  __shared__ double s1[kThreads / 64], mn[kThreads / 64];
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* c = cosv + (int64_t)row * N;
  double s = 0.0, m = 1e300;
  for (int i = tid; i < N; i += kThreads) {
    s += (double)c[i];
    m = fmin(m, (double)c[i]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    m = fmin(m, __shfl_xor(m, o, 64));
  }
  if ((tid & 63) == 0) {
    s1[tid / 64] = s;
    mn[tid / 64] = m;
  }
  __syncthreads();
  double sum = 0.0, mi = 1e300;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) {
    sum += s1[w];
    mi = fmin(mi, mn[w]);
  }
  const double mean = sum / N;
  double q = 0.0;
  for (int i = tid; i < N; i += kThreads) {
    const double d = (double)c[i] - mean;
    q = fma(d, d, q);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  __syncthreads();
  if ((tid & 63) == 0) s1[tid / 64] = q;
  __syncthreads();
  if (tid == 0) {
    double qs = 0.0;
    for (int w = 0; w < kThreads / 64; ++w) qs += s1[w];
    stats[(int64_t)row * 3 + 0] = mean;
    stats[(int64_t)row * 3 + 1] = mi;
    stats[(int64_t)row * 3 + 2] = N > 1 ? sqrt(qs / (N - 1)) : 0.0;
  }
}

template <int D>
int run(const nerfhip_svd_batch* b, hipStream_t st) {
  constexpr int NB = D / 64;
  const int tiles = NB * (NB + 1) / 2;
  hipLaunchKernelGGL(k_svd_gram<D>, dim3(tiles, b->n_tensors), dim3(kThreads), 0, st, b->x,
                     b->N, b->gram);
  hipLaunchKernelGGL(k_svd_jacobi<D>, dim3(b->n_tensors), dim3(kThreads), 0, st, b->gram,
                     b->evec, b->eval, b->order, b->max_sweeps > 0 ? b->max_sweeps : 30);
  ProjArgs pa{};
  pa.n_ranks = b->n_ranks;
  for (int r = 0; r < b->n_ranks; ++r) pa.ranks[r] = b->ranks[r];
  hipLaunchKernelGGL(k_svd_project<D>, dim3((b->N + kThreads - 1) / kThreads, b->n_tensors),
                     dim3(kThreads), 0, st, b->x, b->N, b->evec, pa, b->row_cos);
  hipLaunchKernelGGL(k_svd_stats, dim3(b->n_tensors * b->n_ranks), dim3(kThreads), 0, st,
                     b->row_cos, b->N, b->stats);
  return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
}

}  // namespace

extern "C" int nerfhip_svd_rank_metrics(const nerfhip_svd_batch* b, void* stream) {
  if (!b) return NERFHIP_ERR_NULL;
  if (b->D != 64 && b->D != 128) return NERFHIP_ERR_BAD_HEAD_DIM;
  if (b->n_tensors < 1 || b->N < 2 || b->n_ranks < 1 || b->n_ranks > NERFHIP_SVD_MAX_RANKS)
    return NERFHIP_ERR_BAD_SHAPE;
  for (int r = 0; r < b->n_ranks; ++r)
    if (b->ranks[r] < 1 || b->ranks[r] > b->D || b->ranks[r] > b->N) return NERFHIP_ERR_BAD_SHAPE;
  if (!b->x || !b->gram || !b->evec || !b->eval || !b->order || !b->row_cos || !b->stats)
    return NERFHIP_ERR_NULL;
  hipStream_t st = (hipStream_t)stream;
  return b->D == 64 ? run<64>(b, st) : run<128>(b, st);
}
