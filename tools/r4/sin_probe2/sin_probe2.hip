// Accuracy of candidate fp32 sin/cos pipelines over the argument range a
// SIREN sees (|omega*z| up to a few hundred), against double-precision
// sin/cos of the same fp32 argument.  Diagnostic only (tools/r4).
//   poly : the in-tree sincos_fast (Cody-Waite by pi/2, minimax, quadrant selects)
//   hw2pi: Cody-Waite by 2*pi (exact 3-term), u = r/(2pi) in [-1/2, 1/2],
//          hardware v_sin_f32 / v_cos_f32 (input in revolutions)
//   hwraw: v_sin_f32(x/(2pi)) with no reduction
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ void sc_poly(float x, float* so, float* co) {
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
  const bool swp = q & 1;
  float s = swp ? pc : ps;
  float c = swp ? ps : pc;
  s = (q & 2) ? -s : s;
  c = ((q + 1) & 2) ? -c : c;
  *so = s;
  *co = c;
}
// Cody-Waite by 2*pi: C1, C2 with 12 trailing zero bits (n*C exact for |n| < 2^12)
__device__ __forceinline__ void sc_hw2pi(float x, float* so, float* co) {
  const float n = __builtin_rintf(x * 0.159154936671257019043f);
  float r = fmaf(n, -6.28125000000000000000e+00f, x);
  r = fmaf(n, -1.93500518798828125000e-03f, r);
  r = fmaf(n, -3.01991605056173284538e-07f, r);
  const float u = r * 0.159154936671257019043f;
  *so = __builtin_amdgcn_sinf(u);
  *co = __builtin_amdgcn_cosf(u);
}
// Cody-Waite by pi, u = r/(2pi) in [-1/4, 1/4], sign (-1)^n by a sign-bit xor
__device__ __forceinline__ void sc_hwpi(float x, float* so, float* co) {
  const float n = __builtin_rintf(x * 0.318309873342514038086f);
  float r = fmaf(n, -3.14062500000000000000e+00f, x);
  r = fmaf(n, -9.67502593994140625000e-04f, r);
  r = fmaf(n, -1.50995802528086642269e-07f, r);
  const float u = r * 0.159154936671257019043f;
  const unsigned sg = (unsigned)(int)n << 31;
  *so = __uint_as_float(__float_as_uint(__builtin_amdgcn_sinf(u)) ^ sg);
  *co = __uint_as_float(__float_as_uint(__builtin_amdgcn_cosf(u)) ^ sg);
}
// reduction in revolutions: u = x*(1/2pi) - n with 1/2pi = hi + lo
__device__ __forceinline__ void sc_hwrev(float x, float* so, float* co) {
  const float n = __builtin_rintf(x * 0.159154936671257019043f);
  float u = fmaf(x, 0.159154936671257019043f, -n);
  u = fmaf(x, 6.42063824329852650408e-09f, u);
  *so = __builtin_amdgcn_sinf(u);
  *co = __builtin_amdgcn_cosf(u);
}
__device__ __forceinline__ void sc_hwraw(float x, float* so, float* co) {
  const float u = x * 0.159154936671257019043f;
  *so = __builtin_amdgcn_sinf(u);
  *co = __builtin_amdgcn_cosf(u);
}

constexpr int NV = 10;
__global__ void k(const float* x, float* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s, c;
  sc_poly(x[i], &s, &c); out[NV * (size_t)i + 0] = s; out[NV * (size_t)i + 1] = c;
  sc_hw2pi(x[i], &s, &c); out[NV * (size_t)i + 2] = s; out[NV * (size_t)i + 3] = c;
  sc_hwpi(x[i], &s, &c); out[NV * (size_t)i + 4] = s; out[NV * (size_t)i + 5] = c;
  sc_hwrev(x[i], &s, &c); out[NV * (size_t)i + 6] = s; out[NV * (size_t)i + 7] = c;
  sc_hwraw(x[i], &s, &c); out[NV * (size_t)i + 8] = s; out[NV * (size_t)i + 9] = c;
}

int main(int argc, char** argv) {
  const int n = 1 << 24;
  const double R = argc > 1 ? atof(argv[1]) : 400.0;
  std::vector<float> x(n);
  for (int i = 0; i < n; ++i) x[i] = (float)(-R + 2 * R * (i + 0.5) / n);
  float *dx, *d;
  hipMalloc(&dx, n * 4);
  hipMalloc(&d, (size_t)n * 4 * NV);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, d, n);
  std::vector<float> h((size_t)n * NV);
  hipMemcpy(h.data(), d, (size_t)n * 4 * NV, hipMemcpyDeviceToHost);
  const char* nm[NV] = {"poly_sin", "poly_cos", "hw2pi_sin", "hw2pi_cos", "hwpi_sin", "hwpi_cos", "hwrev_sin", "hwrev_cos", "hwraw_sin", "hwraw_cos"};
  double mabs[NV] = {0}, mulp1[NV] = {0}, rms[NV] = {0};
  for (int i = 0; i < n; ++i) {
    const double s = std::sin((double)x[i]), c = std::cos((double)x[i]);
    for (int j = 0; j < NV; ++j) {
      const double ref = (j & 1) ? c : s;
      const double e = std::fabs((double)h[NV * (size_t)i + j] - ref);
      mabs[j] = std::fmax(mabs[j], e);
      rms[j] += e * e;
    }
  }
  printf("{\"range\": %.1f, \"n\": %d", R, n);
  for (int j = 0; j < NV; ++j)
    printf(", \"%s_max_abs\": %.3e, \"%s_rms\": %.3e", nm[j], mabs[j], nm[j], std::sqrt(rms[j] / n));
  printf(", \"ulp_of_1\": %.3e}\n", (double)(std::nextafter(1.0f, 2.0f) - 1.0f));
  (void)mulp1;
  return 0;
}
