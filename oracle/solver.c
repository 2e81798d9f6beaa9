/*
 * solver.c -- oracle restatement of the 2-D elliptic surface-pressure solve and
 * the steps around it:
 *   INI_CG2D               model/src/ini_cg2d.F:61-237
 *   SOLVE_FOR_PRESSURE     model/src/solve_for_pressure.F:7-468
 *   CALC_DIV_GHAT          model/src/calc_div_ghat.F:6-201
 *   CG2D                   model/src/cg2d.F:13-415
 *   GLOBAL_SUM_TILE_RL     eesupp/src/global_sum_tile.F:161-191 (fixed tile order)
 *   MOMENTUM_CORRECTION_STEP / CORRECTION_STEP / CALC_GRAD_PHI_SURF
 *   INTEGR_CONTINUITY / INTEGRATE_FOR_W
 *   FORWARD_STEP (supported subset), MON_CALC_STATS_RL
 * TEST INFRASTRUCTURE (see oracle.h).
 */
#include "oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* GLOBAL_SUM_TILE_RL: sum = 0; DO bj; DO bi; sum = sum + tile(bi,bj) */
static double gsum_tiles(const double *tile, int nTiles) {
  double s = 0.0;
  for (int t = 0; t < nTiles; t++) s = s + tile[t];
  return s;
}

/* The device CG2D's summation order (include/mitgcm_amd.h, mgcm_cg2d_sum_plan): NG groups
 * (workgroups) of NT threads; thread tid of group g accumulates, from 0.0, the terms at
 * plan[(g*PPT + p)*NT + tid] for p = 0..PPT-1; the group partial is the pairwise tree over
 * its threads in thread order (DPP row sums + row broadcasts + cross-wave row sum,
 * zero-padded to a power of two); the total adds the group partials in group order.
 * Test infrastructure: it lets a device solve be checked bit for bit. */
int oracle_set_sum_plan(OModel *m, const int *plan, int NT, int PPT, int NG) {
  free(m->sumPlan);
  m->sumPlan = NULL;
  if (!plan) return 0;
  if (NT <= 0 || PPT <= 0 || NG <= 0) return -1;
  const size_t n = (size_t)NT * PPT * NG;
  m->sumPlan = malloc(n * sizeof(int));
  memcpy(m->sumPlan, plan, n * sizeof(int));
  m->planNT = NT; m->planPPT = PPT; m->planNG = NG;
  return 0;
}

/* With cg2dUseFMA the device evaluates the CG2D operator rows, dot products and vector
 * updates as fused multiply-adds (kernels_solve.hip k_cg2d_bxy<..., FMA>); the device-order
 * mode then does the same, with C99 fma() (one rounding, as v_fma_f64). */
int oracle_set_cg2d_fma(OModel *m, int on) {
  m->cg2dFMA = on ? 1 : 0;
  return 0;
}

static double pairwise_tree(double *v, int n) {   /* n a power of two; destroys v */
  for (int w = 1; w < n; w *= 2)
    for (int t = 0; t < n; t += 2 * w) v[t] = v[t] + v[t + w];
  return v[0];
}

/* plan_dot: the same order with each thread accumulating fma(a, b, acc) (b = NULL: acc + a) */
static double plan_dot(const OModel *m, const double *a, const double *b);
static double plan_sum(const OModel *m, const double *term) { return plan_dot(m, term, NULL); }
static double plan_dot(const OModel *m, const double *a, const double *b) {
  const double *term = a;
  int np2 = 1;
  while (np2 < m->planNT) np2 *= 2;
  double *th = calloc((size_t)np2, sizeof(double)), lanes[64];
  for (int l = 0; l < 64; l++) lanes[l] = 0.0;
  for (int g = 0; g < m->planNG; g++) {
    for (int t = 0; t < np2; t++) th[t] = 0.0;
    for (int t = 0; t < m->planNT; t++) {
      double e = 0.0;
      for (int p = 0; p < m->planPPT; p++) {
        const int q = m->sumPlan[((size_t)g * m->planPPT + p) * m->planNT + t];
        if (q >= 0) e = b ? fma(term[q], b[q], e) : e + term[q];
      }
      th[t] = e;
    }
    /* workgroup partial g, added into lane g % 64 in workgroup order */
    lanes[g % 64] = lanes[g % 64] + pairwise_tree(th, np2);
  }
  free(th);
  return pairwise_tree(lanes, 64);
}

int oracle_ini_cg2d(OModel *m) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr;
  long N2 = m->n2 * m->nTiles;
  for (long p = 0; p < N2; p++) m->aW2d[p] = m->aS2d[p] = m->aC2d[p] = m->pW[p] = m->pS[p] = m->pC[p] = 0.0;
  double myNorm = 0.0;
  for (int t = 0; t < m->nTiles; t++) {
    for (int k = 1; k <= Nr; k++)
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) {
          long p = O2(m, i, j, t);
          double faceArea = m->dyG[p] * m->drF[k - 1] * m->hFacW[O3(m, i, j, k, t)];
          m->aW2d[p] = m->aW2d[p] + m->implicSurfPress * m->implicDiv2DFlow * faceArea * m->recip_dxC[p];
          faceArea = m->dxG[p] * m->drF[k - 1] * m->hFacS[O3(m, i, j, k, t)];
          m->aS2d[p] = m->aS2d[p] + m->implicSurfPress * m->implicDiv2DFlow * faceArea * m->recip_dyC[p];
        }
    for (int j = 1; j <= sNy; j++)
      for (int i = 1; i <= sNx; i++) {
        myNorm = fmax(fabs(m->aW2d[O2(m, i, j, t)]), myNorm);
        myNorm = fmax(fabs(m->aS2d[O2(m, i, j, t)]), myNorm);
      }
  }
  myNorm = (myNorm != 0.0) ? 1.0 / myNorm : 1.0;
  for (int t = 0; t < m->nTiles; t++)
    for (int j = 1; j <= sNy; j++)
      for (int i = 1; i <= sNx; i++) {
        m->aW2d[O2(m, i, j, t)] = m->aW2d[O2(m, i, j, t)] * myNorm;
        m->aS2d[O2(m, i, j, t)] = m->aS2d[O2(m, i, j, t)] * myNorm;
      }
  oracle_exch_uv_xyz(m, m->aW2d, m->aS2d, 1, 0);   /* EXCH_UV_XY_RS(aW2d,aS2d,.FALSE.) */
  m->cg2dNorm = myNorm;
  m->cg2dNormaliseRHS = (m->cg2dTargetResWunit <= 0.0);
  double tol = m->cg2dNormaliseRHS ? m->cg2dTargetResidual
                                   : m->cg2dNorm * m->cg2dTargetResWunit * m->globalArea / m->deltaTMom;
  m->cg2dTolerance_sq = tol * tol;
  for (int t = 0; t < m->nTiles; t++) {
    for (int j = 0; j <= sNy; j++)
      for (int i = 0; i <= sNx; i++) {
        long p = O2(m, i, j, t);
        m->aC2d[p] = -(m->aW2d[p] + m->aW2d[O2(m, i + 1, j, t)] + m->aS2d[p] + m->aS2d[O2(m, i, j + 1, t)] +
                       m->freeSurfFac * myNorm * m->recip_Bo[p] * m->rA[p] / m->deltaTMom / m->deltaTFreeSurf);
      }
    for (int j = 1; j <= sNy; j++)
      for (int i = 1; i <= sNx; i++) {
        long p = O2(m, i, j, t);
        double aC = m->aC2d[p], aCs = m->aC2d[O2(m, i, j - 1, t)], aCw = m->aC2d[O2(m, i - 1, j, t)];
        m->pC[p] = (aC == 0.0) ? 1.0 : 1.0 / aC;
        if (aC + aCw == 0.0) m->pW[p] = 0.0;
        else { double d = m->cg2dpcOffDFac * (aCw + aC); m->pW[p] = -m->aW2d[p] / (d * d); }
        if (aC + aCs == 0.0) m->pS[p] = 0.0;
        else { double d = m->cg2dpcOffDFac * (aCs + aC); m->pS[p] = -m->aS2d[p] / (d * d); }
      }
  }
  oracle_exch_xy(m, m->pC);
  oracle_exch_uv_xyz(m, m->pW, m->pS, 1, 0);       /* ini_cg2d.F:233-234 */
  (void)OLx; (void)OLy;
  return 0;
}

/* A x at (i,j) as the device's fma chain: aW*w, then + aW(i+1)*e, aS*s, aS(j+1)*n, aC*v */
static double applyA_fma(const OModel *m, const double *v, int i, int j, int t) {
  const double *aW = m->aW2d, *aS = m->aS2d, *aC = m->aC2d;
  const long p = O2(m, i, j, t);
  return fma(aC[p], v[p], fma(aS[O2(m, i, j + 1, t)], v[O2(m, i, j + 1, t)], fma(aS[p], v[O2(m, i, j - 1, t)],
             fma(aW[O2(m, i + 1, j, t)], v[O2(m, i + 1, j, t)], aW[p] * v[O2(m, i - 1, j, t)]))));
}

/* A v and M v at (i,j) in the reference's operand order (cg2d.F:155-161, 212-217), or as the
 * device's fma chains (fmaMode) */
static double cg_applyA(const OModel *m, const double *v, int i, int j, int t, int fmaMode) {
  if (fmaMode) return applyA_fma(m, v, i, j, t);
  const double *aW = m->aW2d, *aS = m->aS2d, *aC = m->aC2d;
  const long p = O2(m, i, j, t);
  return aW[p] * v[O2(m, i - 1, j, t)] + aW[O2(m, i + 1, j, t)] * v[O2(m, i + 1, j, t)] + aS[p] * v[O2(m, i, j - 1, t)] +
         aS[O2(m, i, j + 1, t)] * v[O2(m, i, j + 1, t)] + aC[p] * v[p];
}
static double cg_applyM(const OModel *m, const double *r, int i, int j, int t, int fmaMode) {
  const double *pW = m->pW, *pS = m->pS, *pC = m->pC;
  const long p = O2(m, i, j, t);
  if (fmaMode)
    return fma(pS[O2(m, i, j + 1, t)], r[O2(m, i, j + 1, t)], fma(pS[p], r[O2(m, i, j - 1, t)],
               fma(pW[O2(m, i + 1, j, t)], r[O2(m, i + 1, j, t)], fma(pW[p], r[O2(m, i - 1, j, t)], pC[p] * r[p]))));
  return pC[p] * r[p] + pW[p] * r[O2(m, i - 1, j, t)] + pW[O2(m, i + 1, j, t)] * r[O2(m, i + 1, j, t)] +
         pS[p] * r[O2(m, i, j - 1, t)] + pS[O2(m, i, j + 1, t)] * r[O2(m, i, j + 1, t)];
}
/* sum of a[p]*b[p] over the interior: per-tile sequential partials in tile order
 * (GLOBAL_SUM_TILE_RL / GLOBAL_SUM_VECTOR_RL), or the device's order (sum plan) */
static double cg_dot(const OModel *m, const double *a, const double *b, double *term, int dev, int fmaMode) {
  const int sNx = m->sNx, sNy = m->sNy, nT = m->nTiles;
  double acc = 0.0;
  for (int t = 0; t < nT; t++) {
    double e = 0.0;
    for (int j = 1; j <= sNy; j++)
      for (int i = 1; i <= sNx; i++) {
        const long p = O2(m, i, j, t);
        e = e + a[p] * b[p];
        term[p] = a[p] * b[p];
      }
    acc = acc + e;
  }
  if (dev) return fmaMode ? plan_dot(m, a, b) : plan_sum(m, term);
  return acc;
}

/* CG2D_SR (model/src/cg2d_sr.F:100-440; solve_for_pressure.F:289, useSRCGSolver): the
 * single-reduction conjugate gradient -- one standard step, then per iteration y = M r,
 * v = A y and the three sums (y.r, y.v, r.r) in one GLOBAL_SUM_VECTOR_RL; the residual of the
 * exit test is that of the previous update. */
static void cg2d_sr(OModel *m, double *cg2d_b, double *cg2d_x, double *firstResidual, double *minResidualSq,
                    double *lastResidual, int *numIters, int *nIterMin) {
  const int sNx = m->sNx, sNy = m->sNy, nT = m->nTiles;
  const long N2 = m->n2 * nT;
  double *r = calloc(N2, 8), *s = calloc(N2, 8), *q = calloc(N2, 8), *y = calloc(N2, 8), *v = calloc(N2, 8);
  double *xmin = calloc(N2, 8), *term = calloc(N2, 8);
  const int dev = m->sumPlan != NULL, fmaMode = dev && m->cg2dFMA;
  double rhsMax = 0.0, rhsNorm = 1.0;
  *minResidualSq = -1.0;
#define LOOP for (int t = 0; t < nT; t++) for (int j = 1; j <= sNy; j++) for (int i = 1; i <= sNx; i++)
  LOOP { const long p = O2(m, i, j, t); cg2d_b[p] = cg2d_b[p] * m->cg2dNorm; rhsMax = fmax(fabs(cg2d_b[p]), rhsMax); }
  if (m->cg2dNormaliseRHS) {   /* cg2d_sr.F:113-130 */
    if (rhsMax != 0.0) rhsNorm = 1.0 / rhsMax;
    LOOP { const long p = O2(m, i, j, t); cg2d_b[p] = cg2d_b[p] * rhsNorm; cg2d_x[p] = cg2d_x[p] * rhsNorm; }
  }
  oracle_exch_xy(m, cg2d_x);
  if (*nIterMin >= 0) LOOP xmin[O2(m, i, j, t)] = cg2d_x[O2(m, i, j, t)];
  LOOP { const long p = O2(m, i, j, t); r[p] = cg2d_b[p] - cg_applyA(m, cg2d_x, i, j, t, fmaMode); }
  oracle_exch_xy(m, r);
  {   /* sumRHS, err_sq (cg2d_sr.F:167-170) */
    double *ones = calloc(N2, 8);
    LOOP ones[O2(m, i, j, t)] = 1.0;
    const double sumRHS = dev ? plan_sum(m, cg2d_b) : cg_dot(m, cg2d_b, ones, term, 0, 0);
    m->sumRHS = sumRHS; m->rhsMax = rhsMax;
    free(ones);
  }
  double err_sq = cg_dot(m, r, r, term, dev, fmaMode);
  int it2d = 0;
  *firstResidual = sqrt(err_sq);
  if (*nIterMin >= 0) { *nIterMin = 0; *minResidualSq = err_sq; }
  if (!(err_sq < m->cg2dTolerance_sq)) {
    /* the standard first step (cg2d_sr.F:190-260) */
    LOOP { const long p = O2(m, i, j, t); y[p] = cg_applyM(m, r, i, j, t, fmaMode); s[p] = y[p]; }
    oracle_exch_xy(m, s);
    double eta_qrN = cg_dot(m, y, r, term, dev, fmaMode), eta_qrNM1 = eta_qrN;
    LOOP { const long p = O2(m, i, j, t); q[p] = cg_applyA(m, s, i, j, t, fmaMode); }
    double alpha = cg_dot(m, s, q, term, dev, fmaMode);
    double sigma = eta_qrN / alpha;
    LOOP {
      const long p = O2(m, i, j, t);
      cg2d_x[p] = fmaMode ? fma(sigma, s[p], cg2d_x[p]) : cg2d_x[p] + sigma * s[p];
      r[p] = fmaMode ? fma(-sigma, q[p], r[p]) : r[p] - sigma * q[p];
    }
    oracle_exch_xy(m, r);
    int converged = 0;
    for (it2d = 1; it2d <= *numIters - 1; it2d++) {   /* cg2d_sr.F:262-370 */
      LOOP y[O2(m, i, j, t)] = cg_applyM(m, r, i, j, t, fmaMode);
      oracle_exch_xy(m, y);
      LOOP v[O2(m, i, j, t)] = cg_applyA(m, y, i, j, t, fmaMode);
      eta_qrN = cg_dot(m, y, r, term, dev, fmaMode);
      const double delta = cg_dot(m, y, v, term, dev, fmaMode);
      err_sq = cg_dot(m, r, r, term, dev, fmaMode);
      if (err_sq < m->cg2dTolerance_sq) { converged = 1; break; }
      if (err_sq < *minResidualSq) {
        *minResidualSq = err_sq;
        *nIterMin = it2d;
        LOOP xmin[O2(m, i, j, t)] = cg2d_x[O2(m, i, j, t)];
      }
      const double cgBeta = eta_qrN / eta_qrNM1;
      eta_qrNM1 = eta_qrN;
      alpha = delta - (cgBeta * cgBeta) * alpha;
      sigma = eta_qrN / alpha;
      LOOP {
        const long p = O2(m, i, j, t);
        s[p] = fmaMode ? fma(cgBeta, s[p], y[p]) : y[p] + cgBeta * s[p];
        cg2d_x[p] = fmaMode ? fma(sigma, s[p], cg2d_x[p]) : cg2d_x[p] + sigma * s[p];
        q[p] = fmaMode ? fma(cgBeta, q[p], v[p]) : v[p] + cgBeta * q[p];
        r[p] = fmaMode ? fma(-sigma, q[p], r[p]) : r[p] - sigma * q[p];
      }
      oracle_exch_xy(m, r);
    }
    if (!converged) err_sq = cg_dot(m, r, r, term, dev, fmaMode);   /* cg2d_sr.F:372-382 */
  }
  if (*nIterMin >= 0 && err_sq > *minResidualSq) LOOP cg2d_x[O2(m, i, j, t)] = xmin[O2(m, i, j, t)];
  if (m->cg2dNormaliseRHS) LOOP cg2d_x[O2(m, i, j, t)] = cg2d_x[O2(m, i, j, t)] / rhsNorm;
#undef LOOP
  *lastResidual = sqrt(err_sq);
  *numIters = it2d;   /* cg2d_sr.F:410: the loop index at exit */
  free(r); free(s); free(q); free(y); free(v); free(xmin); free(term);
}

/* CG2D (model/src/cg2d.F:13-415), default branch (no CG2D_SINGLECPU_SUM) */
void oracle_cg2d(OModel *m, double *cg2d_b, double *cg2d_x, double *firstResidual,
                 double *minResidualSq, double *lastResidual, int *numIters, int *nIterMin) {
  if (m->useSRCGSolver) {
    cg2d_sr(m, cg2d_b, cg2d_x, firstResidual, minResidualSq, lastResidual, numIters, nIterMin);
    return;
  }
  const int sNx = m->sNx, sNy = m->sNy, nT = m->nTiles;
  const long N2 = m->n2 * nT;
  double *r = calloc(N2, 8), *s = calloc(N2, 8), *q = calloc(N2, 8), *xmin = calloc(N2, 8);
  double *tile = calloc(nT, 8), *tile2 = calloc(nT, 8);
  double *term = calloc(N2, 8), *term2 = calloc(N2, 8);   /* per-point terms for a device sum plan */
  const int dev = m->sumPlan != NULL, fmaMode = dev && m->cg2dFMA;
  const double *aW = m->aW2d, *aS = m->aS2d, *aC = m->aC2d, *pW = m->pW, *pS = m->pS, *pC = m->pC;
  double err_sq, eta_qrN, eta_qrNM1 = 1.0, cgBeta, alpha, sumRHS, rhsMax = 0.0, rhsNorm = 1.0;
  int actualIts = 0;
  *minResidualSq = -1.0;
  for (int t = 0; t < nT; t++)
    for (int j = 1; j <= sNy; j++)
      for (int i = 1; i <= sNx; i++) {
        long p = O2(m, i, j, t);
        cg2d_b[p] = cg2d_b[p] * m->cg2dNorm;
        rhsMax = fmax(fabs(cg2d_b[p]), rhsMax);
      }
  if (m->cg2dNormaliseRHS) {
    rhsNorm = 1.0;
    if (rhsMax != 0.0) rhsNorm = 1.0 / rhsMax;
    for (int t = 0; t < nT; t++)
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) {
          long p = O2(m, i, j, t);
          cg2d_b[p] = cg2d_b[p] * rhsNorm;
          cg2d_x[p] = cg2d_x[p] * rhsNorm;
        }
  }
  oracle_exch_xy(m, cg2d_x);
  /* OpenMP (bench.py's multi-core baseline): every tile loop below over threads, one tile per
   * iteration; each tile's partial is summed sequentially inside its thread and the partials in
   * tile order by one thread (GLOBAL_SUM_TILE_RL), the halo fills split over destination tiles:
   * bit-identical to one thread.  The scalars are shared, set in `single` blocks (whose barrier
   * publishes them), so every thread takes the same exit. */
  const int minRes = *nIterMin >= 0, maxIts = *numIters;
  int stop = 0;
#pragma omp parallel if (m->nThreads > 1) num_threads(m->nThreads > 1 ? m->nThreads : 1)
  {
#pragma omp for schedule(static)
  for (int t = 0; t < nT; t++) {
    if (minRes)
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) xmin[O2(m, i, j, t)] = cg2d_x[O2(m, i, j, t)];
    double sumT = 0.0, errT = 0.0;
    for (int j = 1; j <= sNy; j++)
      for (int i = 1; i <= sNx; i++) {
        long p = O2(m, i, j, t);
        if (fmaMode)
          r[p] = cg2d_b[p] - applyA_fma(m, cg2d_x, i, j, t);
        else
          r[p] = cg2d_b[p] - (aW[p] * cg2d_x[O2(m, i - 1, j, t)] + aW[O2(m, i + 1, j, t)] * cg2d_x[O2(m, i + 1, j, t)] +
                              aS[p] * cg2d_x[O2(m, i, j - 1, t)] + aS[O2(m, i, j + 1, t)] * cg2d_x[O2(m, i, j + 1, t)] +
                              aC[p] * cg2d_x[p]);
        errT = errT + r[p] * r[p];
        sumT = sumT + cg2d_b[p];
        term[p] = r[p] * r[p];
        term2[p] = cg2d_b[p];
      }
    tile[t] = errT; tile2[t] = sumT;
  }
  /* EXCH_S3D_RL(cg2d_r, 1): halo width 1 fill; the full-halo periodic copy is a superset */
  oracle_exch_xy_for(m, r);
#pragma omp single
  {
  err_sq = dev ? (fmaMode ? plan_dot(m, r, r) : plan_sum(m, term)) : gsum_tiles(tile, nT);
  sumRHS = dev ? plan_sum(m, term2) : gsum_tiles(tile2, nT);
  *firstResidual = sqrt(err_sq);
  if (minRes) { *nIterMin = 0; *minResidualSq = err_sq; }
  m->sumRHS = sumRHS; m->rhsMax = rhsMax;
  stop = !(err_sq < m->cg2dTolerance_sq) ? 0 : 1;
  }
  for (int it2d = 1; !stop && it2d <= maxIts; it2d++) {
#pragma omp for schedule(static)
    for (int t = 0; t < nT; t++) {
      double e = 0.0;
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) {
          long p = O2(m, i, j, t);
          if (fmaMode)
            q[p] = fma(pS[O2(m, i, j + 1, t)], r[O2(m, i, j + 1, t)], fma(pS[p], r[O2(m, i, j - 1, t)],
                   fma(pW[O2(m, i + 1, j, t)], r[O2(m, i + 1, j, t)], fma(pW[p], r[O2(m, i - 1, j, t)], pC[p] * r[p]))));
          else
            q[p] = pC[p] * r[p] + pW[p] * r[O2(m, i - 1, j, t)] + pW[O2(m, i + 1, j, t)] * r[O2(m, i + 1, j, t)] +
                   pS[p] * r[O2(m, i, j - 1, t)] + pS[O2(m, i, j + 1, t)] * r[O2(m, i, j + 1, t)];
          e = e + q[p] * r[p];
          term[p] = q[p] * r[p];
        }
      tile[t] = e;
    }
#pragma omp single
    {
    eta_qrN = dev ? (fmaMode ? plan_dot(m, q, r) : plan_sum(m, term)) : gsum_tiles(tile, nT);
    cgBeta = eta_qrN / eta_qrNM1;
    eta_qrNM1 = eta_qrN;
    }
#pragma omp for schedule(static)
    for (int t = 0; t < nT; t++)
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) {
          long p = O2(m, i, j, t);
          s[p] = fmaMode ? fma(cgBeta, s[p], q[p]) : q[p] + cgBeta * s[p];
        }
    oracle_exch_xy_for(m, s);
#pragma omp for schedule(static)
    for (int t = 0; t < nT; t++) {
      double a = 0.0;
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) {
          long p = O2(m, i, j, t);
          if (fmaMode)
            q[p] = applyA_fma(m, s, i, j, t);
          else
            q[p] = aW[p] * s[O2(m, i - 1, j, t)] + aW[O2(m, i + 1, j, t)] * s[O2(m, i + 1, j, t)] +
                   aS[p] * s[O2(m, i, j - 1, t)] + aS[O2(m, i, j + 1, t)] * s[O2(m, i, j + 1, t)] + aC[p] * s[p];
          a = a + s[p] * q[p];
          term[p] = s[p] * q[p];
        }
      tile[t] = a;
    }
#pragma omp single
    {
    alpha = dev ? (fmaMode ? plan_dot(m, s, q) : plan_sum(m, term)) : gsum_tiles(tile, nT);
    alpha = eta_qrN / alpha;
    }
#pragma omp for schedule(static)
    for (int t = 0; t < nT; t++) {
      double e = 0.0;
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) {
          long p = O2(m, i, j, t);
          cg2d_x[p] = fmaMode ? fma(alpha, s[p], cg2d_x[p]) : cg2d_x[p] + alpha * s[p];
          r[p] = fmaMode ? fma(-alpha, q[p], r[p]) : r[p] - alpha * q[p];
          e = e + r[p] * r[p];
          term[p] = r[p] * r[p];
        }
      tile[t] = e;
    }
    int save = 0;
#pragma omp single copyprivate(save)
    {
    actualIts = it2d;
    err_sq = dev ? (fmaMode ? plan_dot(m, r, r) : plan_sum(m, term)) : gsum_tiles(tile, nT);
    if (err_sq < m->cg2dTolerance_sq) stop = 1;
    else if (err_sq < *minResidualSq) {
      *minResidualSq = err_sq;
      *nIterMin = it2d;
      save = 1;
    }
    }
    if (stop) break;
    if (save) {
#pragma omp for schedule(static)
      for (int t = 0; t < nT; t++)
        for (int j = 1; j <= sNy; j++)
          for (int i = 1; i <= sNx; i++) xmin[O2(m, i, j, t)] = cg2d_x[O2(m, i, j, t)];
    }
    oracle_exch_xy_for(m, r);
  }
  }
  if (*nIterMin >= 0 && err_sq > *minResidualSq)
    for (int t = 0; t < nT; t++)
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) cg2d_x[O2(m, i, j, t)] = xmin[O2(m, i, j, t)];
  if (m->cg2dNormaliseRHS)
    for (int t = 0; t < nT; t++)
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) cg2d_x[O2(m, i, j, t)] = cg2d_x[O2(m, i, j, t)] / rhsNorm;
  *lastResidual = sqrt(err_sq);
  *numIters = actualIts;
  free(r); free(s); free(q); free(xmin); free(tile); free(tile2); free(term); free(term2);
}

/* SOLVE_FOR_PRESSURE (solve_for_pressure.F:122-385), hydrostatic, no OBCS, linear FS */
void oracle_solve_for_pressure(OModel *m) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long N2 = m->n2 * m->nTiles, n2 = m->n2;
  double *cg2d_x = calloc(N2, 8), *cg2d_b = calloc(N2, 8), *pf = calloc(n2, 8);
  for (long p = 0; p < N2; p++) {
    m->etaNm1[p] = m->etaN[p];   /* ALLOW_CD_CODE (solve_for_pressure.F:126-128) */
    cg2d_x[p] = m->Bo_surf[p] * m->etaN[p];
    cg2d_b[p] = 0.0;
  }
  /* solve_for_pressure.F:142-151: fresh-water volume flux */
  if (m->useRealFreshWaterFlux) {
    const double tmpFac = m->freeSurfFac * (1.0 / m->rhoConst) * m->implicDiv2DFlow;
    for (int t = 0; t < m->nTiles; t++)
      for (int j = 1; j <= m->sNy; j++)
        for (int i = 1; i <= m->sNx; i++) {
          const long p = O2(m, i, j, t);
          cg2d_b[p] = tmpFac * m->rA[p] * m->EmPmR[p] / m->deltaTMom * m->maskInC[p];
        }
  }
#define PF(i, j) pf[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx]
  for (int t = 0; t < m->nTiles; t++) {
    for (int k = Nr; k >= 1; k--) {
      /* CALC_DIV_GHAT (calc_div_ghat.F:62-166), implicDiv2DFlow = 1 */
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx + 1; i++) {
          double xA = m->dyG[O2(m, i, j, t)] * m->drF[k - 1] * m->hFacW[O3(m, i, j, k, t)];
          PF(i, j) = xA * m->gU[O3(m, i, j, k, t)] / m->deltaTMom;
        }
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++)
          cg2d_b[O2(m, i, j, t)] = cg2d_b[O2(m, i, j, t)] + PF(i + 1, j) - PF(i, j);
      for (int j = 1; j <= sNy + 1; j++)
        for (int i = 1; i <= sNx; i++) {
          double yA = m->dxG[O2(m, i, j, t)] * m->drF[k - 1] * m->hFacS[O3(m, i, j, k, t)];
          PF(i, j) = yA * m->gV[O3(m, i, j, k, t)] / m->deltaTMom;
        }
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++)
          cg2d_b[O2(m, i, j, t)] = cg2d_b[O2(m, i, j, t)] + PF(i, j + 1) - PF(i, j);
    }
  }
#undef PF
  for (int t = 0; t < m->nTiles; t++)
    for (int j = 1; j <= sNy; j++)
      for (int i = 1; i <= sNx; i++) {
        long p = O2(m, i, j, t);
        /* solve_for_pressure.F:214-236: etaH with exactConserv, else etaN */
        const double eta = m->exactConserv ? m->etaH[p] : m->etaN[p];
        cg2d_b[p] = cg2d_b[p] - m->freeSurfFac * m->rA[p] / m->deltaTMom / m->deltaTFreeSurf * eta;
      }
  int numIters = m->cg2dMaxIters, nIterMin = m->cg2dUseMinResSol - 1;
  double firstRes, minResSq, lastRes;
  oracle_cg2d(m, cg2d_b, cg2d_x, &firstRes, &minResSq, &lastRes, &numIters, &nIterMin);
  oracle_exch_xy(m, cg2d_x);
  m->firstResidual = firstRes; m->lastResidual = lastRes; m->numIters = numIters; m->nIterMin = nIterMin;
  m->minResidualSq = (minResSq >= 0.0) ? sqrt(minResSq) : minResSq;
  for (long p = 0; p < N2; p++) m->etaN[p] = m->recip_Bo[p] * cg2d_x[p];
  free(cg2d_x); free(cg2d_b); free(pf);
}

/* MOMENTUM_CORRECTION_STEP (momentum_correction_step.F:60-91) -> CALC_GRAD_PHI_SURF
 * (calc_grad_phi_surf.F:46-61) -> CORRECTION_STEP (correction_step.F:150-234) */
void oracle_momentum_correction_step(OModel *m) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr;
  const int iMin = 1 - OLx + 1, iMax = sNx + OLx, jMin = 1 - OLy + 1, jMax = sNy + OLy;
  const double psFac = m->pfFacMom * m->implicSurfPress;
  for (int t = 0; t < m->nTiles; t++) {
    for (int k = 1; k <= Nr; k++)
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) {
          long p = O2(m, i, j, t), p3 = O3(m, i, j, k, t);
          double phiSurfX = m->recip_dxC[p] * (m->Bo_surf[p] * m->etaN[p] - m->Bo_surf[O2(m, i - 1, j, t)] * m->etaN[O2(m, i - 1, j, t)]);
          double phiSurfY = m->recip_dyC[p] * (m->Bo_surf[p] * m->etaN[p] - m->Bo_surf[O2(m, i, j - 1, t)] * m->etaN[O2(m, i, j - 1, t)]);
          double gU_dpx = -psFac * phiSurfX * m->maskW[p3];
          double gV_dpy = -psFac * phiSurfY * m->maskS[p3];
          m->uVel[p3] = (m->gU[p3] + m->deltaTMom * gU_dpx) * m->maskW[p3];
          m->vVel[p3] = (m->gV[p3] + m->deltaTMom * gV_dpy) * m->maskS[p3];
        }
  }
}

/* INTEGR_CONTINUITY (integr_continuity.F:66-314) -> INTEGRATE_FOR_W
 * (integrate_for_w.F:61-195) -> UPDATE_ETAH (update_etah.F:55-73).
 * atInit: the call from INITIALISE_VARIA (myIter = nIter0); otherwise the call in
 * FORWARD_STEP, where myIter = nIter0 + iLoop > nIter0.  exactConserv: dEtaHdt
 * from the column divergence (and fresh-water flux), etaN = etaH + dEtaHdt*dtFS;
 * r* (select_rStar > 0): w includes -rStarDhDt*drF*h0FacC. */
static void integr_continuity(OModel *m, int atInit) {
  const int sNx = m->sNx, sNy = m->sNy, Nr = m->Nr, nx = m->nx;
  const long N2 = m->n2 * m->nTiles;
  const int rstar = m->nonlinFreeSurf > 0 && m->select_rStar != 0;
  double *rStarDhDt = calloc(m->n2, 8);
#define RD(i, j) rStarDhDt[O2(m, i, j, 0)]
  for (int t = 0; t < m->nTiles; t++) {
    if (m->exactConserv) {
      double *hDiv = calloc(m->n2, 8);
#define HD(i, j) hDiv[O2(m, i, j, 0)]
      for (int k = 1; k <= Nr; k++)
        for (int j = 1; j <= sNy; j++)
          for (int i = 1; i <= sNx; i++) {
            double uT1 = m->uVel[O3(m, i + 1, j, k, t)] * m->dyG[O2(m, i + 1, j, t)] * m->drF[k - 1] * m->hFacW[O3(m, i + 1, j, k, t)];
            double uT0 = m->uVel[O3(m, i, j, k, t)] * m->dyG[O2(m, i, j, t)] * m->drF[k - 1] * m->hFacW[O3(m, i, j, k, t)];
            double vT1 = m->vVel[O3(m, i, j + 1, k, t)] * m->dxG[O2(m, i, j + 1, t)] * m->drF[k - 1] * m->hFacS[O3(m, i, j + 1, k, t)];
            double vT0 = m->vVel[O3(m, i, j, k, t)] * m->dxG[O2(m, i, j, t)] * m->drF[k - 1] * m->hFacS[O3(m, i, j, k, t)];
            HD(i, j) = HD(i, j) + m->maskC[O3(m, i, j, k, t)] * (uT1 - uT0 + vT1 - vT0);
          }
      const double facEmP = m->useRealFreshWaterFlux ? 1.0 / m->rhoConst : 0.0;   /* mass2rUnit */
      if (atInit && m->nIter0 != 0 && m->useRealFreshWaterFlux) {
        /* integr_continuity.F:117-136: PmEpR consistent with the pickup dEtaHdt */
        for (int j = 1; j <= sNy; j++)
          for (int i = 1; i <= sNx; i++) {
            const long p = O2(m, i, j, t);
            m->PmEpR[p] = m->dEtaHdt[p] + HD(i, j) * m->recip_rA[p];
            m->PmEpR[p] = m->PmEpR[p] * m->rhoConst;                            /* rUnit2mass */
          }
      } else if (atInit) {
        for (int j = 1; j <= sNy; j++)
          for (int i = 1; i <= sNx; i++) {
            const long p = O2(m, i, j, t);
            m->PmEpR[p] = 0.0;
            m->dEtaHdt[p] = -(HD(i, j) * m->recip_rA[p]);
          }
      } else {
        for (long q = 0; q < m->n2; q++) m->PmEpR[t * m->n2 + q] = -m->EmPmR[t * m->n2 + q];
        for (int j = 1; j <= sNy; j++)
          for (int i = 1; i <= sNx; i++) {
            const long p = O2(m, i, j, t);
            m->dEtaHdt[p] = -(HD(i, j) * m->recip_rA[p]) - facEmP * m->EmPmR[p];
          }
      }
      if (!atInit)
        for (int j = 1; j <= sNy; j++)
          for (int i = 1; i <= sNx; i++) {
            const long p = O2(m, i, j, t);
            m->etaN[p] = m->etaH[p] + m->implicDiv2DFlow * m->dEtaHdt[p] * m->deltaTFreeSurf;
          }
#undef HD
      free(hDiv);
      if (rstar)   /* integr_continuity.F:171-183 (deepFac2F = rhoFacF = 1) */
        for (int j = 1; j <= sNy; j++)
          for (int i = 1; i <= sNx; i++) RD(i, j) = m->dEtaHdt[O2(m, i, j, t)] * m->recip_Rcol[O2(m, i, j, t)];
    }
    for (int k = Nr; k >= 1; k--)
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) {
          long p = O2(m, i, j, t);
          double uT1 = m->uVel[O3(m, i + 1, j, k, t)] * m->dyG[O2(m, i + 1, j, t)] * m->drF[k - 1] * m->hFacW[O3(m, i + 1, j, k, t)];
          double uT0 = m->uVel[O3(m, i, j, k, t)] * m->dyG[p] * m->drF[k - 1] * m->hFacW[O3(m, i, j, k, t)];
          double vT1 = m->vVel[O3(m, i, j + 1, k, t)] * m->dxG[O2(m, i, j + 1, t)] * m->drF[k - 1] * m->hFacS[O3(m, i, j + 1, k, t)];
          double vT0 = m->vVel[O3(m, i, j, k, t)] * m->dxG[p] * m->drF[k - 1] * m->hFacS[O3(m, i, j, k, t)];
          double conv2d = -(uT1 - uT0 + vT1 - vT0);
          if (rstar) {   /* integrate_for_w.F:117-140 */
            const double dh = RD(i, j) * m->drF[k - 1] * m->h0FacC[O3(m, i, j, k, t)];
            if (k == Nr)
              m->wVel[O3(m, i, j, k, t)] = (conv2d * m->recip_rA[p] - dh) * m->maskC[O3(m, i, j, k, t)];
            else
              m->wVel[O3(m, i, j, k, t)] =
                  (m->wVel[O3(m, i, j, k + 1, t)] + conv2d * m->recip_rA[p] - dh) * m->maskC[O3(m, i, j, k, t)];
          } else if (k == Nr) {
            m->wVel[O3(m, i, j, k, t)] = conv2d * m->recip_rA[p] * m->maskC[O3(m, i, j, k, t)];
          } else {
            m->wVel[O3(m, i, j, k, t)] = (m->wVel[O3(m, i, j, k + 1, t)] + conv2d * m->recip_rA[p]) * m->maskC[O3(m, i, j, k, t)];
          }
        }
  }
#undef RD
  free(rStarDhDt);
  if (m->exactConserv && !atInit) oracle_exch_xy(m, m->etaN);
  if (atInit) oracle_exch_xyz(m, m->wVel, Nr);
  if (m->exactConserv)
    for (long p = 0; p < N2; p++) m->etaH[p] = m->etaN[p];   /* UPDATE_ETAH, implicDiv2Dflow = 1 */
  (void)nx;
}

void oracle_integr_continuity(OModel *m) { integr_continuity(m, 0); }
void oracle_integr_continuity_init(OModel *m) { integr_continuity(m, 1); }

/* FORWARD_STEP (model/src/forward_step.F:64-1256) for the supported subset:
 * EXTERNAL_FORCING_SURF (momentum part) -> DYNAMICS -> SOLVE_FOR_PRESSURE ->
 * MOMENTUM_CORRECTION_STEP -> INTEGR_CONTINUITY -> DO_FIELDS_BLOCKING_EXCHANGES */
void oracle_forward_step(OModel *m) {
  /* forward_step.F:542 LOAD_FIELDS_DRIVER -> EXTERNAL_FIELDS_LOAD (periodic forcing) */
  oracle_fields_load(m);
  /* forward_step.F:656 DO_OCEANIC_PHYS (always called: surface forcing, rhoInSitu, ...) */
  oracle_oceanic_phys(m);
  if ((m->tempStepping || m->saltStepping) && !m->staggerTimeStep) {
    /* forward_step.F:732 THERMODYNAMICS (staggerTimeStep = F) */
    oracle_thermodynamics(m);
  }
  const int rstar = m->nonlinFreeSurf > 0 && m->select_rStar > 0;
  if (m->momStepping) {
    oracle_dynamics(m);
    /* forward_step.F:806: myIter/myTime advance before SOLVE_FOR_PRESSURE;
     * :829-877 UPDATE_R_STAR(.TRUE.) + UPDATE_CG2D (nonlinFreeSurf > 2) */
    if (rstar) {
      oracle_update_r_star(m, 1);
      if (m->nonlinFreeSurf > 2) oracle_update_cg2d(m);
    }
    oracle_solve_for_pressure(m);
    oracle_momentum_correction_step(m);
  }
  oracle_integr_continuity(m);
  /* forward_step.F:965-977 CALC_R_STAR(etaH(n+1)) */
  if (rstar) oracle_calc_r_star(m);
  if ((m->tempStepping || m->saltStepping) && m->staggerTimeStep) {
    /* forward_step.F:1003-1036: DO_STAGGER_FIELDS_EXCHANGES (u, v, w;
     * do_stagger_fields_exchanges.F:37-43), then THERMODYNAMICS with the new velocities */
    oracle_exch_uv_xyz(m, m->uVel, m->vVel, m->Nr, 1);
    oracle_exch_xyz(m, m->wVel, m->Nr);
    oracle_thermodynamics(m);
  }
  /* do_fields_blocking_exchanges.F:54-97 */
  oracle_exch_uv_xyz(m, m->uVel, m->vVel, m->Nr, 1);
  oracle_exch_xyz(m, m->wVel, m->Nr);
  oracle_exch_xyz(m, m->theta, m->Nr);
  oracle_exch_xyz(m, m->salt, m->Nr);
  if (m->useCDscheme) {   /* EXCH_UV_DGRID_3D_RL(uVelD, vVelD): lat-lon = scalar copies */
    if (m->exchS) { fprintf(stderr, "oracle: CD scheme on an exch2 topology not restated\n"); abort(); }
    oracle_exch_xyz(m, m->uVelD, m->Nr);
    oracle_exch_xyz(m, m->vVelD, m->Nr);
  }
  if (m->storePhiHyd4Phys) oracle_exch_xyz(m, m->totPhiHyd, m->Nr);
  /* next step's RESET_NLFS_VARS + UPDATE_R_STAR(.FALSE.) (forward_step.F:463-498)
   * restore hFac = h0Fac*rStarFacNm1, the values UPDATE_R_STAR(.TRUE.) set above */
  if (rstar) oracle_update_r_star(m, 0);
  m->myIter = m->myIter + 1;
  m->myTime = m->myTime + m->deltaTClock;
}

/* MON_CALC_STATS_RL (pkg/monitor/mon_calc_stats_rl.F). arrhFac is 3-D
 * (myNr levels) when hfac3d, else a 2-D mask reused for every level. */
void oracle_mon_stats(OModel *m, const double *arr, int myNr, const double *arrhFac, int hfac3d,
                      const double *arrMask, const double *arrArea, const double *arrDr, double out[6]) {
  const int sNx = m->sNx, sNy = m->sNy, nT = m->nTiles;
  const long n2 = m->n2, nz = (long)myNr * n2;
  double theMin = 0, theMax = 0, theMean = 0, theSD = 0, theDel2 = 0, theVol = 0, theNbPt = 0;
  int noPnts = 1;
  double *tNb = calloc(nT, 8), *tDel2 = calloc(nT, 8), *tVol = calloc(nT, 8), *tMean = calloc(nT, 8), *tSD = calloc(nT, 8);
#define H(i, j, k) (hfac3d ? arrhFac[O2(m, i, j, t) - (long)t * n2 + (long)((k) - 1) * n2 + (long)t * nz] : arrhFac[O2(m, i, j, t)])
#define A(i, j, k) arr[O2(m, i, j, t) - (long)t * n2 + (long)((k) - 1) * n2 + (long)t * nz]
  for (int t = 0; t < nT; t++) {
    for (int k = 1; k <= myNr; k++)
      for (int j = 1; j <= sNy; j++)
        for (int i = 1; i <= sNx; i++) {
          double v = A(i, j, k);
          double msk = arrMask[O2(m, i, j, t)] * H(i, j, k);
          if (msk > 0.0 && noPnts) { theMin = v; theMax = v; noPnts = 0; }
          if (msk > 0.0) {
            theMin = fmin(theMin, v); theMax = fmax(theMax, v);
            double ddx = H(i + 1, j, k) * H(i - 1, j, k);
            if (ddx > 0.0) ddx = (A(i + 1, j, k) - v) + (A(i - 1, j, k) - v);
            double ddy = H(i, j + 1, k) * H(i, j - 1, k);
            if (ddy > 0.0) ddy = (A(i, j + 1, k) - v) + (A(i, j - 1, k) - v);
            tDel2[t] = tDel2[t] + ddx * ddx + ddy * ddy;
            tNb[t] = tNb[t] + 1.0;
            double vol = arrArea[O2(m, i, j, t)] * arrDr[k - 1] * msk;
            tVol[t] = tVol[t] + vol;
            tMean[t] = tMean[t] + vol * v;
          }
        }
  }
  theNbPt = gsum_tiles(tNb, nT); theDel2 = gsum_tiles(tDel2, nT);
  theVol = gsum_tiles(tVol, nT); theMean = gsum_tiles(tMean, nT);
  if (theNbPt > 0.0) theDel2 = sqrt(theDel2) / theNbPt;
  if (theVol > 0.0) {
    theMean = theMean / theVol;
    if (noPnts) { theMin = theMean; theMax = theMean; }
    for (int t = 0; t < nT; t++)
      for (int k = 1; k <= myNr; k++)
        for (int j = 1; j <= sNy; j++)
          for (int i = 1; i <= sNx; i++) {
            double v = A(i, j, k), msk = arrMask[O2(m, i, j, t)] * H(i, j, k);
            if (msk > 0.0) {
              double vol = arrArea[O2(m, i, j, t)] * arrDr[k - 1] * msk;
              tSD[t] = tSD[t] + vol * (v - theMean) * (v - theMean);
            }
          }
    theSD = gsum_tiles(tSD, nT);
    theSD = sqrt(theSD / theVol);
  }
#undef H
#undef A
  out[0] = theMin; out[1] = theMax; out[2] = theMean; out[3] = theSD; out[4] = theDel2; out[5] = theVol;
  free(tNb); free(tDel2); free(tVol); free(tMean); free(tSD);
}
