// nc_pdf.hip -- hierarchical (importance) sampling, sample_pdf (src/common.py:19-63),
// as render_batch_ray uses it when N_importance > 0 (src/utils/Renderer.py:244-250).
//
// One wavefront per ray, lane = bin / sample:
//   w_j = weights_j + 1e-5 (float32); pdf_j = w_j / sum(w) (float32)
//   cdf = [0, cumsum(pdf)]: accumulated in float64 and rounded per entry, as ATen's CPU
//         cumsum does for float32 (acc_type<float> = double), sequentially by lane 0
//   u_k = linspace(0, 1, N) (det) or the caller's draw; inds = searchsorted(cdf, u,
//         right=True): the number of cdf entries <= u
//   below = max(inds-1, 0), above = min(inds, nb-1); denom = cdf[above] - cdf[below]
//         (float32, < 1e-5 -> 1); t = (u - cdf[below]) / denom (float32)
//   sample = bins[below] + t * (bins[above] - bins[below])  (float64, t promoted)
#include "nc_internal.h"

namespace nc {

constexpr int PDF_WAVES = 4;

__global__ void __launch_bounds__(64 * PDF_WAVES) k_sample_pdf(const nc_pdf_args a) {
  __shared__ float cdf_s[PDF_WAVES][NC_MAX_SAMPLES + 1];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * PDF_WAVES + wave;
  if (r >= a.n_rays) return;
  const int nb = (int)a.n_bins, nw = nb - 1;
  float* cdf = cdf_s[wave];
  const float w = lane < nw ? a.weights[r * a.weights_stride + lane] + 1e-5f : 0.f;
  if (lane < nw) cdf[lane + 1] = w;  // staged for the sequential sums below
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane == 0) {
    float sum = 0.f;  // torch.sum of <= 63 float32 values
    for (int j = 0; j < nw; ++j) sum += cdf[j + 1];
    double acc = 0.0;
    cdf[0] = 0.f;
    for (int j = 0; j < nw; ++j) {
      acc += (double)(cdf[j + 1] / sum);
      cdf[j + 1] = (float)acc;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane >= a.n_samples) return;
  float u;
  if (a.det) {
    // torch.linspace(0, 1, N) float32: start + k * step for the first half, end - (N-1-k) * step after
    const int n = (int)a.n_samples;
    const float step = n > 1 ? 1.f / (float)(n - 1) : 0.f;
    u = lane < n / 2 ? (float)lane * step : 1.f - (float)(n - 1 - lane) * step;
  } else {
    u = a.u[r * a.u_stride + lane];
  }
  int inds = 0;
  for (int j = 0; j < nb; ++j) inds += cdf[j] <= u ? 1 : 0;  // cdf is non-decreasing
  const int below = inds - 1 > 0 ? inds - 1 : 0;
  const int above = inds < nb - 1 ? inds : nb - 1;
  const float c0 = cdf[below], c1 = cdf[above];
  float denom = c1 - c0;
  denom = denom < 1e-5f ? 1.f : denom;
  const float t = (u - c0) / denom;
  const double* bins = a.bins + r * a.bins_stride;
  const double b0 = bins[below], b1 = bins[above];
  a.samples[r * a.samples_stride + lane] = b0 + (double)t * (b1 - b0);
}

int launch_sample_pdf(const nc_pdf_args& a, hipStream_t s) {
  const int64_t blocks = (a.n_rays + PDF_WAVES - 1) / PDF_WAVES;
  hipLaunchKernelGGL(k_sample_pdf, dim3((unsigned)blocks), dim3(64 * PDF_WAVES), 0, s, a);
  return (int)hipGetLastError();
}

}  // namespace nc
