// Host-side solvers for the small dense sub-problems of the GLM family
// (H2O's GLM does these on the driver node too, hex/glm/ComputationState /
// GramSolver): the IRLS elastic-net step is a (p+1)x(p+1) problem on the
// all-reduced Gram, solved here by covariance-update cyclic coordinate
// descent in double precision.  Called once per IRLS iteration and lambda,
// so it must not be the interpreter-bound loop it would be in Python.
#include <cmath>
#include <cstdint>

#define H2OMX_HOST_API extern "C" __attribute__((visibility("default")))

// Minimise 1/2 b^T A b - r^T b + sum_j pen_j/2 b_j^2 + l1 sum_{j != free} |b_j|
// over b (k coefficients; A is k x k row-major with leading dimension ld).
// `free_idx` (the intercept, or -1) gets neither the L1 nor the L2 penalty
// (pen must be 0 there).  non_negative clamps the penalised coefficients at 0.
// beta holds the warm start on entry and the solution on exit.
// Returns the number of sweeps, or -1 on bad arguments.
H2OMX_HOST_API int h2omx_enet_cd(const double* A, int ld, const double* r, const double* pen, int k, double l1,
                                 int free_idx, int non_negative, double* beta, int max_iter, double tol) {
  if (!A || !r || !pen || !beta || k <= 0 || ld < k) return -1;
  // g = r - A beta (maintained incrementally: O(k) per coordinate update)
  double* g = new double[k];
  for (int i = 0; i < k; ++i) {
    double s = r[i];
    const double* Ai = A + (int64_t)i * ld;
    for (int j = 0; j < k; ++j) s -= Ai[j] * beta[j];
    g[i] = s;
  }
  int it = 0;
  for (; it < max_iter; ++it) {
    double mx = 0.0;
    for (int j = 0; j < k; ++j) {
      const double ajj = A[(int64_t)j * ld + j];
      const double d = ajj + pen[j];
      if (d <= 0.0) continue;
      const double rho = g[j] + ajj * beta[j];          // partial residual correlation
      double nb;
      if (j == free_idx) {
        nb = rho / d;
      } else {
        const double a = std::fabs(rho) - l1;
        nb = a > 0.0 ? std::copysign(a, rho) / d : 0.0;
        if (non_negative && nb < 0.0) nb = 0.0;
      }
      const double delta = nb - beta[j];
      if (delta != 0.0) {
        // A is symmetric: column j == row j
        const double* Aj = A + (int64_t)j * ld;
        for (int i = 0; i < k; ++i) g[i] -= delta * Aj[i];
        beta[j] = nb;
        const double ad = std::fabs(delta);
        if (ad > mx) mx = ad;
      }
    }
    if (mx < tol) { ++it; break; }
  }
  delete[] g;
  return it;
}
