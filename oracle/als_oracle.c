/*
 * als_oracle.c — C restatement of Spark ALS's per-row arithmetic.
 * TEST INFRASTRUCTURE ONLY: used by tests/ as an independent cross-check of
 * oracle/als_oracle.py and by bench.py's `cpu_baseline` leg ("port").  The
 * product (libals_hip.so / als_mi355x) never links or calls it.
 *
 * Restated from Apache Spark ml/recommendation/ALS.scala (upstream, version
 * unpinned by the reference — see oracle/als_oracle.py) and the reference
 * BLAS/LAPACK routines it calls through netlib-java:
 *   NormalEquation.add   -> blas.dspr("U", k, c, x, 1, ata) + blas.daxpy(k, b, x, 1, atb, 1)
 *   computeYtY           -> dspr over every src factor (treeAggregate of partials)
 *   CholeskySolver.solve -> ata[diag] += lambda; LAPACK dppsv("U") = dpptrf + dpptrs
 * Packed storage is column-major upper: A(i,j), i <= j, at ap[j*(j+1)/2 + i].
 * The reference call sites reaching this code: RecommenderSystem.py:148-149,
 * :163, :218 (ALS.train).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* BLAS dspr, UPLO = 'U': ap += alpha * x x^T (upper packed). */
static void dspr_u(int n, double alpha, const double* x, double* ap) {
  int kk = 0;
  for (int j = 0; j < n; ++j) {
    if (x[j] != 0.0) {
      const double temp = alpha * x[j];
      for (int i = 0; i <= j; ++i) ap[kk + i] += x[i] * temp;
    }
    kk += j + 1;
  }
}

/* BLAS daxpy: y += a x. */
static void daxpy(int n, double a, const double* x, double* y) {
  if (a == 0.0) return;
  for (int i = 0; i < n; ++i) y[i] += a * x[i];
}

/* BLAS dtpsv, UPLO='U', TRANS='T', DIAG='N': solve U^T x = b in place. */
static void dtpsv_ut(int n, const double* ap, double* x) {
  int kk = 0;
  for (int j = 0; j < n; ++j) {
    double temp = x[j];
    for (int i = 0; i < j; ++i) temp -= ap[kk + i] * x[i];
    x[j] = temp / ap[kk + j];
    kk += j + 1;
  }
}

/* BLAS dtpsv, UPLO='U', TRANS='N', DIAG='N': solve U x = b in place. */
static void dtpsv_un(int n, const double* ap, double* x) {
  int kk = n * (n + 1) / 2 - 1;
  for (int j = n - 1; j >= 0; --j) {
    if (x[j] != 0.0) {
      x[j] /= ap[kk];
      const double temp = x[j];
      int k = kk - 1;
      for (int i = j - 1; i >= 0; --i, --k) x[i] -= temp * ap[k];
    }
    kk -= j + 1;
  }
}

/* LAPACK dpptrf, UPLO='U'.  Returns 0 or the 1-based failing column. */
static int dpptrf_u(int n, double* ap) {
  int jj = -1;
  for (int j = 0; j < n; ++j) {
    const int jc = jj + 1;
    jj += j + 1;
    if (j > 0) dtpsv_ut(j, ap, ap + jc);
    double dot = 0.0;
    for (int i = 0; i < j; ++i) dot += ap[jc + i] * ap[jc + i];
    const double ajj = ap[jj] - dot;
    if (ajj <= 0.0 || isnan(ajj)) {
      ap[jj] = ajj;
      return j + 1;
    }
    ap[jj] = sqrt(ajj);
  }
  return 0;
}

/* YtY of n rows (upper packed, fp64). */
int oracle_yty(const float* Y, int64_t n, int32_t ldy, int32_t k, double* ata_out, int nthreads) {
  const int tri = k * (k + 1) / 2;
  memset(ata_out, 0, sizeof(double) * tri);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
  {
    double* part = (double*)calloc((size_t)tri, sizeof(double));
    double* da = (double*)malloc(sizeof(double) * k);
#pragma omp for schedule(static)
    for (int64_t s = 0; s < n; ++s) {
      for (int i = 0; i < k; ++i) da[i] = (double)Y[s * ldy + i];
      dspr_u(k, 1.0, da, part);
    }
#pragma omp critical
    for (int i = 0; i < tri; ++i) ata_out[i] += part[i];
    free(part);
    free(da);
  }
  return 0;
}

/*
 * One half-sweep (computeFactors) over all rows of a CSR side.
 * X[row*ldx + 0..k) <- solution; status[row] = dpptrf info (0 ok).
 * yty (implicit only): upper-packed YtY from oracle_yty.
 * Returns the number of rows whose Cholesky failed.
 */
int oracle_half_sweep(const int64_t* indptr, const int32_t* indices, const float* vals,
                      int32_t n_rows, const float* Y, int32_t ldy, int32_t k, double reg,
                      int implicit, double alpha, const double* yty, float* X, int32_t ldx,
                      int32_t* status, int nthreads) {
  const int tri = k * (k + 1) / 2;
  int fails = 0;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel reduction(+ : fails)
  {
    double* ata = (double*)malloc(sizeof(double) * tri);
    double* atb = (double*)malloc(sizeof(double) * k);
    double* da = (double*)malloc(sizeof(double) * k);
#pragma omp for schedule(dynamic, 1) /* heavy rows (millions of ratings) spread over threads */
    for (int32_t j = 0; j < n_rows; ++j) {
      memset(ata, 0, sizeof(double) * tri);
      memset(atb, 0, sizeof(double) * k);
      if (implicit) memcpy(ata, yty, sizeof(double) * tri); /* ls.merge(YtY) */
      int64_t n_exp = 0;
      for (int64_t p = indptr[j]; p < indptr[j + 1]; ++p) {
        const float* y = Y + (int64_t)indices[p] * ldy;
        for (int i = 0; i < k; ++i) da[i] = (double)y[i];
        const double rating = (double)vals[p];
        if (implicit) {
          const double c1 = alpha * fabs(rating);
          if (rating > 0.0) n_exp += 1;
          dspr_u(k, c1, da, ata);
          daxpy(k, rating > 0.0 ? 1.0 + c1 : 0.0, da, atb);
        } else {
          dspr_u(k, 1.0, da, ata);
          daxpy(k, rating, da, atb);
          n_exp += 1;
        }
      }
      /* CholeskySolver.solve(ls, numExplicits * regParam) */
      const double lambda = (double)n_exp * reg;
      for (int i = 0, d = 0; i < k; ++i, d += i + 1) ata[d] += lambda;
      const int info = dpptrf_u(k, ata);
      if (info == 0) {
        dtpsv_ut(k, ata, atb);
        dtpsv_un(k, ata, atb);
      } else {
        fails += 1;
      }
      if (status) status[j] = info;
      for (int i = 0; i < k; ++i) X[(int64_t)j * ldx + i] = info == 0 ? (float)atb[i] : 0.0f;
    }
    free(ata);
    free(atb);
    free(da);
  }
  return fails;
}

int oracle_abi_version(void) { return 1; }
