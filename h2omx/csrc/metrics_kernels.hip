// Model-metric kernels: score histograms for AUC / AUCPR
// / threshold metrics.  Every rank bins its scores into the same 2^16 bins
// over the globally all-reduced [lo, hi] range; the per-class histograms are
// then all-reduced once.  Counts are accumulated as fixed-point int64 (weight
// x 2^24) with global integer atomics, so the histograms - and AUC - are
// bit-identical regardless of row order, grid size or number of GPUs.
#include "common.h"

namespace {

constexpr double WSCALE = 16777216.0;  // 2^24

__global__ __launch_bounds__(256) void auc_hist_kernel(const double* __restrict__ score,
                                                       const double* __restrict__ y,
                                                       const double* __restrict__ w, int64_t n, int nbins,
                                                       double lo, double inv_span,
                                                       unsigned long long* __restrict__ hist) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double yi = y[i];
    if (!(yi == yi)) continue;  // NA response
    const double wi = w ? w[i] : 1.0;
    if (wi == 0.0) continue;
    double f = (score[i] - lo) * inv_span * (nbins - 1);
    int b = (int)rint(f);
    b = b < 0 ? 0 : (b >= nbins ? nbins - 1 : b);
    const unsigned long long q = (unsigned long long)(long long)llrint(wi * WSCALE);
    // y in [0, 1]: positive mass y*w, negative mass (1-y)*w (fractional labels allowed)
    if (yi >= 1.0) atomicAdd(hist + b, q);
    else if (yi <= 0.0) atomicAdd(hist + nbins + b, q);
    else {
      const unsigned long long qp = (unsigned long long)(long long)llrint(wi * yi * WSCALE);
      atomicAdd(hist + b, qp);
      atomicAdd(hist + nbins + b, q - qp);
    }
  }
}

}  // namespace

H2OMX_API int h2omx_auc_hist(const double* score, const double* y, const double* w, int64_t n, int nbins,
                             double lo, double hi, unsigned long long* hist, hipStream_t stream) {
  if (nbins < 2) return kBadArg;
  const double span = hi > lo ? hi - lo : 1e-300;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(auc_hist_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, score, y, w, n, nbins, lo,
                     1.0 / span, hist);
  return launch_status();
}

H2OMX_API double h2omx_auc_weight_scale() { return WSCALE; }
