/*
 * nngp_rows.h -- row-major record rows -> R's column-major matrix
 * (records$field, update_Gaussian.R:305-311: one row per saved iteration).
 * Used by nngp_shim.c; a plain C header so the transpose is unit-tested
 * without R (tests/test_capi_and_graph.py).
 */
#ifndef NNGP_ROWS_H
#define NNGP_ROWS_H
#include <stddef.h>

/* dst[i + j * ld] = src[i * n + j] for i < k, j < n: k row-major rows of n
 * into the first k rows of a column-major matrix with leading dimension ld.
 * Cache blocks of 64 x 64 doubles: both sides walk whole 512-B runs. */
static void nngp_rows_to_colmajor(const double* src, double* dst, ptrdiff_t ld, ptrdiff_t k, ptrdiff_t n) {
  enum { B = 64 };
  for (ptrdiff_t j0 = 0; j0 < n; j0 += B) {
    const ptrdiff_t j1 = j0 + B < n ? j0 + B : n;
    for (ptrdiff_t i0 = 0; i0 < k; i0 += B) {
      const ptrdiff_t i1 = i0 + B < k ? i0 + B : k;
      for (ptrdiff_t j = j0; j < j1; ++j)
        for (ptrdiff_t i = i0; i < i1; ++i) dst[i + j * ld] = src[i * n + j];
    }
  }
}
#endif
