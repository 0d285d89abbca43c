// nerfhip_analysis.hip — MI355X (gfx950) KV structure analysis.
//
// Replaces the per-dimension numpy loops of the reference's pre-fit analysis
// (nerf_attention/analyze.py:20-44, called from _analyze_tensor :61-71) for a
// batch of KV slices: for each sampled head dimension d of each slice X [N×D]
//   * the lag-k autocorrelation of the centred column, k = 0..max_lag
//     (_autocorrelation, analyze.py:20-30), and
//   * the fraction of spectral energy of the Hann-windowed, centred column in
//     the lowest 5/10/25/50 % of its rfft bins (_spectral_energy, :33-44).
// One workgroup per (slice, dimension).  The column lives in LDS; the rfft is
// a direct DFT in fp64 against an exact twiddle table (bin f, sample t →
// angle index f·t mod N), which matches numpy's fp64 FFT to ~1e-12.  The
// effective rank (:47-58) uses the singular values of nerfhip_svd_rank_metrics.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "nerfhip.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxN = 8192;
constexpr double kPi = 3.14159265358979323846;

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) s += red[w];
  return s;
}

struct DimArgs {
  int32_t n_dims, max_lag;
  int32_t dims[NERFHIP_ANALYSIS_MAX_DIMS];
};

__global__ void __launch_bounds__(kThreads) k_kv_analyze(const float* __restrict__ X, int N,
                                                         int D, DimArgs da,
                                                         double* __restrict__ autocorr,
                                                         double* __restrict__ energy) {
  // LDS: the centred column (fp64), then the windowed column; the twiddle
  // table cos(2πk/N); the |X_f|² bins overwrite the centred column
  __shared__ double col[kMaxN];
  __shared__ double tw[kMaxN];
  __shared__ double red[kThreads / 64];
  const int slice = blockIdx.y, di = blockIdx.x, tid = threadIdx.x;
  const int d = da.dims[di];
  const float* x = X + (int64_t)slice * N * D + d;
  const int NL = da.max_lag + 1;
  double* ac = autocorr + ((int64_t)slice * da.n_dims + di) * NL;
  double* en = energy + ((int64_t)slice * da.n_dims + di) * 4;

  double s = 0.0;
  for (int t = tid; t < N; t += kThreads) {
    const double v = (double)x[(int64_t)t * D];
    col[t] = v;
    s += v;
  }
  // the reference centres the fp32 column in fp32 (signal - signal.mean()):
  // c = fl32(x - fl32(mean)), then works on those values
  const float mean32 = (float)(block_sum(s, red) / N);
  double q = 0.0;
  for (int t = tid; t < N; t += kThreads) {
    const double c = (double)((float)col[t] - mean32);
    col[t] = c;
    q = fma(c, c, q);
  }
  const double var = block_sum(q, red);   // (also makes every col[] visible)
  // ---- autocorrelation, one lag per thread (analyze.py:23-30)
  for (int lag = tid; lag < NL; lag += kThreads) {
    double a = 0.0;
    if (var >= 1e-10 && lag < N) {
      for (int t = 0; t + lag < N; ++t) a = fma(col[t], col[t + lag], a);
      a /= var;
    }
    ac[lag] = a;
  }
  // ---- spectral energy (analyze.py:33-44): w = centred · np.hanning(N)
  for (int k = tid; k < N; k += kThreads) tw[k] = cos(2.0 * kPi * (double)k / (double)N);
  __syncthreads();
  for (int t = tid; t < N; t += kThreads) {
    const double h = N > 1 ? 0.5 - 0.5 * cos(2.0 * kPi * (double)t / (double)(N - 1)) : 1.0;
    col[t] *= h;
  }
  __syncthreads();
  const int nf = N / 2 + 1;
  // |X_f|², f = tid, tid + 256, ...: held in registers, then written over col[]
  constexpr int kMaxPer = (kMaxN / 2 + 1 + kThreads - 1) / kThreads;
  double pw[kMaxPer];
  const int quarter = N / 4;                  // sin(θ_k) = cos(θ_{k − N/4}) when 4 | N
  const bool q4 = (N % 4) == 0;
#pragma unroll
  for (int j = 0; j < kMaxPer; ++j) {
    const int f = tid + kThreads * j;
    double re = 0.0, im = 0.0;
    if (f < nf) {
      int idx = 0;                            // (f·t) mod N, incremented
      for (int t = 0; t < N; ++t) {
        const double c = tw[idx];
        const double sn = q4 ? tw[idx >= quarter ? idx - quarter : idx - quarter + N]
                             : sin(2.0 * kPi * (double)idx / (double)N);
        re = fma(col[t], c, re);
        im = fma(-col[t], sn, im);
        idx += f;
        if (idx >= N) idx -= N;
      }
    }
    pw[j] = re * re + im * im;
  }
  // cumulative energies of the lowest bins: top_{5,10,25,50} %
  const double pct[4] = {0.05, 0.10, 0.25, 0.50};
  int lim[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int m = (int)(nf * pct[p]);
    lim[p] = m > 1 ? m : 1;
  }
  double tot = 0.0, part[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 0; j < kMaxPer; ++j) {
    const int f = tid + kThreads * j;
    if (f < nf) {
      tot += pw[j];
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (f < lim[p]) part[p] += pw[j];
    }
  }
  const double total = block_sum(tot, red);
  double fr[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) fr[p] = block_sum(part[p], red);
  if (tid == 0) {
#pragma unroll
    for (int p = 0; p < 4; ++p) en[p] = total < 1e-10 ? 1.0 : fr[p] / total;
  }
}

}  // namespace

extern "C" int nerfhip_kv_analysis(const nerfhip_kv_analysis_batch* a, void* stream) {
  if (!a) return NERFHIP_ERR_NULL;
  if (a->n_tensors < 1 || a->N < 2 || a->N > 8192 || a->D < 1 || a->n_dims < 1 ||
      a->n_dims > NERFHIP_ANALYSIS_MAX_DIMS || a->max_lag < 0 || a->max_lag > 1023)
    return NERFHIP_ERR_BAD_SHAPE;
  DimArgs da{};
  da.n_dims = a->n_dims;
  da.max_lag = a->max_lag;
  for (int i = 0; i < a->n_dims; ++i) {
    if (a->dims[i] < 0 || a->dims[i] >= a->D) return NERFHIP_ERR_BAD_SHAPE;
    da.dims[i] = a->dims[i];
  }
  if (!a->x || !a->autocorr || !a->energy) return NERFHIP_ERR_NULL;
  hipLaunchKernelGGL(k_kv_analyze, dim3(a->n_dims, a->n_tensors), dim3(kThreads), 0,
                     (hipStream_t)stream, a->x, a->N, a->D, da, a->autocorr, a->energy);
  return hipGetLastError() == hipSuccess ? NERFHIP_OK : NERFHIP_ERR_LAUNCH;
}
