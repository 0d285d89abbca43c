// Accuracy of the hardware v_sin_f32 / v_cos_f32 (input in revolutions) on
// the Cody-Waite-reduced range |r| <= pi/4 that sincos_fast feeds its
// polynomials, against double-precision sin/cos: max error in fp32 ulps of
// the true value, and the same for the in-tree polynomial.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const float* x, float* s_hw, float* c_hw, float* s_po, float* c_po, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float r = x[i];
  const float t = r * 0.15915493667125701904f;   // 1 / (2 pi) in fp32
  s_hw[i] = __builtin_amdgcn_sinf(t);
  c_hw[i] = __builtin_amdgcn_cosf(t);
  const float r2 = r * r;
  float ps = fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f);
  ps = fmaf(r2, ps, -1.6666654611e-1f);
  ps = fmaf(r2 * r, ps, r);
  float pc = fmaf(r2, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = fmaf(r2, pc, 4.166664568298827e-2f);
  pc = fmaf(r2 * r2, pc, fmaf(r2, -0.5f, 1.0f));
  s_po[i] = ps;
  c_po[i] = pc;
}

static double ulp_err(float got, double ref) {
  const float rf = (float)ref;
  const float u = std::nextafter(std::fabs(rf), INFINITY) - std::fabs(rf);
  return std::fabs((double)got - ref) / (double)u;
}

int main() {
  const int n = 1 << 24;
  std::vector<float> x(n);
  for (int i = 0; i < n; ++i) x[i] = (float)(-0.78539816 + 1.5707963 * (i + 0.5) / n);
  float *dx, *d[4];
  hipMalloc(&dx, n * 4);
  for (auto& p : d) hipMalloc(&p, n * 4);
  hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, d[0], d[1], d[2], d[3], n);
  std::vector<float> h[4];
  for (int j = 0; j < 4; ++j) {
    h[j].resize(n);
    hipMemcpy(h[j].data(), d[j], n * 4, hipMemcpyDeviceToHost);
  }
  double m[4] = {0, 0, 0, 0}, mabs[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const double s = std::sin((double)x[i]), c = std::cos((double)x[i]);
    const double ref[4] = {s, c, s, c};
    for (int j = 0; j < 4; ++j) {
      if (std::fabs(ref[j]) > 1e-30) m[j] = std::fmax(m[j], ulp_err(h[j][i], ref[j]));
      mabs[j] = std::fmax(mabs[j], std::fabs(h[j][i] - ref[j]));
    }
  }
  printf("{\"n\": %d, \"sin_hw_max_ulp\": %.3f, \"cos_hw_max_ulp\": %.3f, \"sin_poly_max_ulp\": %.3f, "
         "\"cos_poly_max_ulp\": %.3f, \"sin_hw_max_abs\": %.3e, \"cos_hw_max_abs\": %.3e, "
         "\"sin_poly_max_abs\": %.3e, \"cos_poly_max_abs\": %.3e}\n",
         n, m[0], m[1], m[2], m[3], mabs[0], mabs[1], mabs[2], mabs[3]);
  return 0;
}
