/*
 * nerfhip.h — C ABI of the MI355X (gfx950) SIREN KV-fit engine.
 *
 * Drop-in boundary for the reference hot path `nerf_attention.siren.fit_siren`
 * (reference: nerf_attention/siren.py:70-149) and its sweep driver
 * `nerf_attention.fit.fit_kv_cache` (nerf_attention/fit.py:20-92).  The
 * reference is pure Python and has no FFI; these entry points are what a
 * ctypes / torch.library binding of that path binds.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Every buffer is caller-allocated DEVICE
 *     memory (the caller owns it; the library never allocates, frees or
 *     synchronises).  All work is enqueued on `stream` (a hipStream_t passed
 *     as void*, NULL = default stream) and returns immediately.
 *   - Return value: NERFHIP_OK (0) or a negative nerfhip_status.
 *   - No global mutable state; reentrant across streams and devices.
 *   - fp32 everywhere on the device (the reference trains in fp32,
 *     siren.py:82-105); host-side float64 scalars (LR schedule, Adam bias
 *     corrections) arrive pre-rounded to fp32 in `sched`.
 *
 * One call trains a GROUP of independent fits that share (W, D, N, epochs):
 * each fit f has its own hidden_layers L_f <= L_max and omega_0 (so medium,
 * deep, hifreq and lofreq — all W=256 — share one group).
 */
#ifndef NERFHIP_H
#define NERFHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NERFHIP_ABI_VERSION 5

typedef enum nerfhip_status {
  NERFHIP_OK = 0,
  NERFHIP_ERR_BAD_WIDTH = -1,      /* hidden_features not in {64,128,256,512}      */
  NERFHIP_ERR_BAD_HEAD_DIM = -2,   /* d_head not in {64,128}                       */
  NERFHIP_ERR_BAD_LAYERS = -3,     /* hidden_layers not in [1, NERFHIP_MAX_LAYERS]  */
  NERFHIP_ERR_BAD_SHAPE = -4,      /* seq_len < 2, n_fits < 1, epochs < 0 ...      */
  NERFHIP_ERR_NULL = -5,           /* a required pointer is NULL                   */
  NERFHIP_ERR_LAUNCH = -6,         /* hipGetLastError() after a launch             */
  NERFHIP_ERR_BAD_PRECISION = -7   /* nerfhip_group.precision not a nerfhip_precision */
} nerfhip_status;

/* Arithmetic of the GEMMs (everything else is fp32 in both modes).
 *   FP32    v_mfma_f32_*_f32: an exact k-ordered fp32 fma chain.
 *   BF16X3  fp32 operands split exactly into three bf16 parts (x = h+m+l);
 *           six bf16 MFMA products per operand pair (the three dropped terms
 *           are < 2^-23 of the product: fp32-class accuracy) with fp32
 *           accumulation — 2.7x the matrix-core rate of FP32.  Needs the
 *           `wsplit` workspace. */
typedef enum nerfhip_precision {
  NERFHIP_PRECISION_FP32 = 0,
  NERFHIP_PRECISION_BF16X3 = 1
} nerfhip_precision;

#define NERFHIP_MAX_LAYERS 4

/* Sizes (in fp32 elements, per fit unless noted) of every buffer a group
 * needs.  Filled by nerfhip_group_sizes(); the caller allocates
 * n_fits * <per-fit size> for the per-fit buffers. */
typedef struct nerfhip_sizes {
  int64_t n_pad;           /* seq_len rounded up to 64 rows (row workgroups)  */
  int64_t params;          /* P(L_max) = 2W + L(W^2+W) + W*D + D  (state_dict order) */
  int64_t params_t;        /* transposed weight copies: L_max*W^2 + W*D       */
  int64_t scratch;         /* activations / grads / cos, feature-major        */
  int64_t target;          /* n_pad * D                                       */
  int64_t stats;           /* D (mean) — std has the same size                */
  int64_t loss_partial;    /* epochs * n_pad/16                               */
  int64_t rows;            /* n_pad (row_cos / row_sq)                        */
  int64_t grad_split;      /* row splits of the small-group gradient reduction */
  int64_t grad_partial;    /* grad_split * params: optional split-K workspace  */
  int64_t wsplit;          /* uint16 elements: 6(L_max W^2 + W D), BF16X3 weight planes */
} nerfhip_sizes;

/* One group of fits.  "[n]" = per fit, strided by the matching nerfhip_sizes
 * field; all pointers are device pointers unless marked (host). */
typedef struct nerfhip_group {
  int32_t W;               /* hidden_features                                 */
  int32_t D;               /* d_head = out_features                            */
  int32_t N;               /* seq_len                                         */
  int32_t n_fits;
  int32_t L_max;           /* max hidden_layers over the group.  A one-fit group
                              MUST set it to that fit's hidden_layers: its kernels
                              take the depth from L_max, not from fit_layers */
  int32_t epochs;
  int32_t log_every;       /* probe period (siren.py:107); 0 = no probes       */
  int32_t device;          /* HIP device ordinal the buffers and stream live on */
  int32_t precision;       /* nerfhip_precision (0 = FP32)                     */
  int32_t reserved;

  const int32_t* fit_layers;  /* [n_fits] hidden_layers per fit              */
  const float* fit_omega;     /* [n_fits] omega_0 per fit                    */
  const float* positions;     /* [n_pad] linspace(0,1,N), zero padded (siren.py:82) */
  const float* target;        /* [n] raw KV rows [n_pad][D] (padded rows 0)  */
  float* target_norm;         /* [n] out: (y-mean)/std   (siren.py:85-87)     */
  float* mean;                /* [n] out: column mean [D]                      */
  float* std;                 /* [n] out: column std (unbiased, >=1e-3) [D]    */
  float* params;              /* [n] in: init, out: trained (state_dict order) */
  float* params_t;            /* [n] workspace: transposed weight copies       */
  float* adam_m;              /* [n] workspace (zeroed by the call)            */
  float* adam_v;              /* [n] workspace (zeroed by the call)            */
  float* scratch;             /* [n] workspace                                 */
  const float* sched;         /* [epochs][2]: {lr_e / (1-b1^t), sqrt(1-b2^t)}  */
  float* loss_partial;        /* [n] out: per-epoch partial sum of squared err */
  float* probe_y;             /* [n][epochs/log_every][n_pad][D] out or NULL   */
  float* eval_y;              /* [n] out: final normalised prediction [n_pad][D] */
  float* row_cos;             /* [n] out: final per-row cosine  [n_pad]        */
  float* row_sq;              /* [n] out: final per-row sum (pred-y)^2 [n_pad] */
  float* probe_row_cos;       /* [n][epochs/log_every][n_pad] or NULL          */
  float* probe_row_sq;        /* [n][epochs/log_every][n_pad] or NULL          */
  float* grad_partial;        /* [n] optional workspace or NULL.  When set and
                                 n_fits < 8, each epoch's weight gradient is
                                 reduced in row slices (partial slabs, then a
                                 fixed-order sum + Adam): a small group
                                 otherwise fills only a few workgroups
                                 (nerfhip_group_plan reports the slices).
                                 Deterministic; slices and tiles depend on the
                                 group shape only — not on n_groups or on what
                                 else trains on the device (round 6 lifted the
                                 round-5 single-group rule). */
  void* wsplit;               /* [n] uint16 workspace, BF16X3 only (else NULL):
                                 every weight as exact bf16 split planes, in
                                 the forward and the transposed orientation,
                                 rewritten by each Adam step                 */
} nerfhip_group;

int nerfhip_abi_version(void);
const char* nerfhip_status_string(int status);

/* Validate (W, D, N, L_max, epochs) and fill *out. */
int nerfhip_group_sizes(int32_t W, int32_t D, int32_t N, int32_t L_max, int32_t epochs,
                        nerfhip_sizes* out);

/* Whole fit for every member of `n_groups` groups: prologue (normalise,
 * transposed weights, zero Adam state), `epochs` fused train steps (forward,
 * MSE, backward, Adam, cosine-annealed LR; siren.py:98-105), the log probes
 * (siren.py:107-115) and the final evaluation (siren.py:119-125).
 * Group i runs on streams[i] (a hipStream_t of device groups[i].device).
 * Launches are interleaved epoch by epoch across the groups so that every
 * stream has work queued and the groups run concurrently.  All groups are
 * validated before anything is enqueued. */
int nerfhip_siren_fit(const nerfhip_group* groups, int32_t n_groups, void* const* streams);

/* Per-kernel device time of a group, measured with hipEvents bracketing
 * the launches of its two step kernels in every 4th epoch (bench.py's
 * roofline leg). */
typedef struct nerfhip_timing {
  int32_t launches;        /* out: timed launches per kernel (epochs 3, 7, 11, ...: every 4th, never the cold first);
                              0 when epochs < 4 — callers must check before dividing */
  int32_t reserved;
  double rows_ms;          /* out: Σ duration of the row-step launches        */
  double params_ms;        /* out: Σ duration of the parameter-step launches  */
} nerfhip_timing;

/* nerfhip_siren_fit, with timings[i] (an array of n_groups records) filled
 * for every group.  Unlike the untimed call it synchronises every group's
 * stream before returning. */
int nerfhip_siren_fit_timed(const nerfhip_group* groups, int32_t n_groups,
                            void* const* streams, nerfhip_timing* timings);

/* Forward only with the current params → eval_y (+ row metrics when
 * target/mean/std/row_cos/row_sq are set).  SIREN.forward, siren.py:60-61. */
int nerfhip_siren_forward(const nerfhip_group* g, void* stream);

/* How nerfhip_siren_fit will run a group's epoch (no device work; reads only
 * the group's shape fields, precision and whether grad_partial is set). */
typedef enum nerfhip_rows_variant {
  NERFHIP_ROWS_REGULAR = 0,   /* k_step_rows: 64-row workgroups, one wave per 16 rows     */
  NERFHIP_ROWS_KSPLIT = 1,    /* k_step_rows_ks: four waves split every GEMM's k over one
                                 16-row block (small bf16x3 groups, W >= 128, D = 128)   */
  NERFHIP_ROWS_32 = 2         /* k_step_rows32: 128-row workgroups, one wave per 32 rows,
                                 32x32x16 MFMAs (bf16x3, W = 256, D = 128, n_pad % 128 = 0;
                                 NERFHIP_VARIANTS builds only) */
} nerfhip_rows_variant;

typedef struct nerfhip_plan {
  int32_t rows_variant;       /* nerfhip_rows_variant                                    */
  int32_t grad_split;         /* row slices of the weight-gradient reduction (1 = fused) */
  int32_t rows_workgroups;    /* grid of the row step                                    */
  int32_t params_workgroups;  /* grid of the parameter step                              */
  int32_t launches_per_epoch; /* kernels enqueued per epoch                              */
  int32_t reserved;
} nerfhip_plan;

int nerfhip_group_plan(const nerfhip_group* g, nerfhip_plan* out);

/* Diagnostic compile-time switches this library was built with (0 for a
 * product build): bit 0 any NERFHIP_EXP_* timing/diagnostic macro (such
 * builds may compute wrong results on purpose), bit 1 NERFHIP_STAMPS
 * (in-kernel timestamps), bit 2 NERFHIP_DIAG_* (altered launch sequence),
 * bit 3 NERFHIP_VARIANTS (the opt-in kernels that measured slower than the
 * defaults: the 32-row row kernel, NERFHIP_ROWS32=1, and the fused split-K
 * reduction, NERFHIP_SPLIT_FUSED=1; a product build ignores both switches). */
#define NERFHIP_BUILD_EXP 1
#define NERFHIP_BUILD_STAMPS 2
#define NERFHIP_BUILD_DIAG 4
#define NERFHIP_BUILD_VARIANTS 8
int nerfhip_build_flags(void);

/* ------------------------------------------------------------------------
 * Truncated-SVD baseline (BASELINE config 5).
 * Replaces the per-slice CPU loop of the reference's SVD experiment
 * (nerf_attention/experiments/svd.py:43-75: torch.linalg.svd, rank-r
 * reconstruction U_r diag(S_r) V_rᵀ, F.cosine_similarity per row, mean / min /
 * std) for a batch of KV slices in one call: fp64 Gram, Jacobi
 * eigen-solver, and the per-row cosine of every requested rank as
 * ‖projection onto the top-r right singular vectors‖ / ‖row‖.
 * ------------------------------------------------------------------------ */
#define NERFHIP_SVD_MAX_RANKS 8

typedef struct nerfhip_svd_batch {
  int32_t n_tensors;       /* slices in the batch                              */
  int32_t N;               /* rows per slice (seq_len), >= 2                    */
  int32_t D;               /* columns (head_dim): 64 or 128                     */
  int32_t n_ranks;         /* 1..NERFHIP_SVD_MAX_RANKS                          */
  int32_t ranks[NERFHIP_SVD_MAX_RANKS];   /* (host) each in [1, min(N, D)]      */
  int32_t max_sweeps;      /* Jacobi sweep cap (<= 0: 30)                       */
  int32_t reserved;
  const float* x;          /* [n_tensors][N][D] slices, row-major               */
  double* gram;            /* [n_tensors][D][D] workspace                       */
  double* evec;            /* [n_tensors][D][D] out: row k = k-th right singular
                              vector (eigenvalues descending)                    */
  double* eval;            /* [n_tensors][D] out: σ² descending                  */
  int32_t* order;          /* [n_tensors][D] out: solver index of each σ²        */
  float* row_cos;          /* [n_tensors][n_ranks][N] out: per-row cosine        */
  double* stats;           /* [n_tensors][n_ranks][3] out: mean, min, std (N−1)  */
} nerfhip_svd_batch;

/* Enqueue the whole batch on `stream`; asynchronous like the fit entry points. */
int nerfhip_svd_rank_metrics(const nerfhip_svd_batch* b, void* stream);

/* ------------------------------------------------------------------------
 * KV structure analysis.  Replaces the per-dimension numpy
 * loops of the reference's pre-fit analysis (nerf_attention/analyze.py:20-44,
 * _analyze_tensor :61-71): for every sampled head dimension of every slice,
 * the lag-0..max_lag autocorrelation of the centred column and the fraction
 * of Hann-windowed rfft energy in the lowest 5/10/25/50 % of bins.  fp64.
 * (The effective rank, analyze.py:47-58, uses nerfhip_svd_rank_metrics.)
 * ------------------------------------------------------------------------ */
#define NERFHIP_ANALYSIS_MAX_DIMS 64

typedef struct nerfhip_kv_analysis_batch {
  int32_t n_tensors;       /* slices                                            */
  int32_t N;               /* rows per slice (seq_len), 2..8192                 */
  int32_t D;               /* columns (head_dim)                                */
  int32_t n_dims;          /* sampled dimensions, 1..NERFHIP_ANALYSIS_MAX_DIMS   */
  int32_t max_lag;         /* 0..1023 (reference: 50)                           */
  int32_t reserved;
  int32_t dims[NERFHIP_ANALYSIS_MAX_DIMS];   /* (host) column indices          */
  const float* x;          /* [n_tensors][N][D]                                  */
  double* autocorr;        /* [n_tensors][n_dims][max_lag + 1] out               */
  double* energy;          /* [n_tensors][n_dims][4] out: top 5/10/25/50 %       */
} nerfhip_kv_analysis_batch;

int nerfhip_kv_analysis(const nerfhip_kv_analysis_batch* a, void* stream);

/* ------------------------------------------------------------------------
 * Seeded initialisation replay (host only).  The reference initialises each
 * SIREN with torch's default CPU generator (siren.py:17-67: nn.Linear's own
 * reset, then the SIREN re-draw); a sweep draws ~10^8 floats that way, at
 * ~6 ns each inside torch.  This draws the same sequence at the speed of the
 * bare generator: mt19937 (state[624], left, next exactly as torch's
 * CPUGeneratorImpl state holds them) and the float transform of
 * at::uniform_real_distribution<float> (24 random bits × 2^-24, then
 * x·(hi−lo)+lo in float).  Segment s consumes counts[s] draws from
 * U[lo[s], hi[s]) (the bounds are rounded to float as uniform_ does); it
 * writes them to out + out_off[s], or — out_off[s] < 0 — only advances the
 * generator (nn.Linear's reset values, which the SIREN overwrites).  The state
 * is updated in place.  Host memory only; no device, no stream.
 * ------------------------------------------------------------------------ */
int nerfhip_rng_uniform_segments(uint32_t* state, int32_t* left, uint32_t* next,
                                 int32_t n_segments, const int64_t* counts,
                                 const double* lo, const double* hi,
                                 const int64_t* out_off, float* out);

#ifdef __cplusplus
}
#endif

#endif /* NERFHIP_H */
