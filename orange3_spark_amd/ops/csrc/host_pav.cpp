// Host-side pool-adjacent-violators (C ABI, libo3s_host.so) for IsotonicRegression.
//
// Spark fits isotonic regression with a parallel PAV: rows are range-partitioned by
// feature, each partition runs PAV, and a final PAV runs over the pooled partition
// outputs.  PAV on a contiguous x-range only ever coarsens, so pooled blocks are exact
// inputs to the final pass.  This routine is both passes: the input is a list of
// x-sorted blocks [xlo, xhi] with mean label y and weight w (raw points have xlo == xhi),
// the output is the coarsened block list.  Equal-x points are pooled first (Spark >= 3
// and scikit-learn do the same), then adjacent violators (y_prev >= y_next, so constant
// runs are compressed too) are merged with a stack -- O(n) amortised.
#include <stdint.h>

extern "C" {

__attribute__((visibility("default"))) int64_t o3s_host_pav(const double* xlo, const double* xhi, const double* y,
                                                            const double* w, int64_t n, double* oxlo, double* oxhi,
                                                            double* oy, double* ow) {
  // Pass 1: pool equal-x runs (must precede PAV: its merges are never undone).
  int64_t u = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (!(w[i] > 0.0)) continue;                      // zero-weight rows carry no information
    if (u > 0 && oxhi[u - 1] == xlo[i]) {
      const double tw = ow[u - 1] + w[i];
      oy[u - 1] = (oy[u - 1] * ow[u - 1] + y[i] * w[i]) / tw;
      ow[u - 1] = tw;
      oxhi[u - 1] = xhi[i];
      continue;
    }
    oxlo[u] = xlo[i];
    oxhi[u] = xhi[i];
    oy[u] = y[i];
    ow[u] = w[i];
    ++u;
  }
  // Pass 2: PAV in place over the u unique-x blocks (stack top = m - 1 <= i).
  int64_t m = 0;
  for (int64_t i = 0; i < u; ++i) {
    double bx0 = oxlo[i], bx1 = oxhi[i], by = oy[i], bw = ow[i];
    while (m > 0 && oy[m - 1] >= by) {                // violator (or equal): merge left
      const double tw = ow[m - 1] + bw;
      by = (oy[m - 1] * ow[m - 1] + by * bw) / tw;
      bw = tw;
      bx0 = oxlo[m - 1];
      --m;
    }
    oxlo[m] = bx0;
    oxhi[m] = bx1;
    oy[m] = by;
    ow[m] = bw;
    ++m;
  }
  return m;
}

}  // extern "C"
