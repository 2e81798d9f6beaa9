/*
 * thermo.c -- oracle restatement of the tracer half of the step.
 * TEST INFRASTRUCTURE (see oracle.h): never linked into the product.
 *
 *   oracle_oceanic_phys   DO_OCEANIC_PHYS subset (model/src/do_oceanic_phys.F:555-882):
 *                         EXTERNAL_FORCING_SURF (external_forcing_surf.F:95-186) with
 *                         FORCING_SURF_RELAX (forcing_surf_relax.F:52-80),
 *                         FIND_RHO_2D LINEAR (find_rho.F:125-136) for rhoInSitu,
 *                         GRAD_SIGMA sigmaR (grad_sigma.F:103-117) + CALC_IVDC (calc_ivdc.F:60-71)
 *   oracle_thermodynamics THERMODYNAMICS (thermodynamics.F) -> TEMP_INTEGRATE (temp_integrate.F):
 *                         CALC_3D_DIFFUSIVITY (calc_3d_diffusivity.F:99-156),
 *                         CALC_ADV_FLOW (calc_adv_flow.F:60-113), APPLY_FORCING_T
 *                         (apply_forcing.F:687-695), GAD_CALC_RHS (gad_calc_rhs.F) with
 *                         GAD_C2_ADV_X/Y/R and GAD_DIFF_X/Y, ADAMS_BASHFORTH2
 *                         (adams_bashforth2.F:61-88), TIMESTEP_TRACER (timestep_tracer.F),
 *                         GAD_IMPLICIT_R (gad_implicit_r.F:96-140) -> SOLVE_TRIDIAGONAL
 *                         (solve_tridiagonal.F, default branch), CYCLE_TRACER (cycle_tracer.F)
 * Multiplications by deepFac/rhoFac factors (= 1) and additions of identically-zero
 * terms of disabled packages are dropped (bit-exact).
 */
#include "oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define L(a, i, j) (a)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx]
#define W3(a, i, j, k) (a)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx + (long)((k) - 1) * n2]
#define W3I(i, j, k) ((long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx + (long)((k) - 1) * n2)

/* FIND_RHO_2D, equationOfState = 'LINEAR' (find_rho.F:125-136) */

void oracle_oceanic_phys(OModel *m) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long n2 = m->n2;
  /* do_oceanic_phys.F:548-553 FREEZE_SURFACE, :574 EXTERNAL_FORCING_SURF (full halo range) */
  if (m->allowFreezing) oracle_freeze_surface(m);
  oracle_external_forcing_surf(m);
  const int calcConvect = m->ivdc_kappa != 0.0;
#pragma omp parallel for schedule(dynamic, 1) if (m->nThreads > 1) num_threads(m->nThreads > 1 ? m->nThreads : 1)
  for (int t = 0; t < m->nTiles; t++) {
    const double *theta = m->theta + t * m->n3, *salt = m->salt + t * m->n3;
    const double *maskC = m->maskC + t * m->n3, *maskW = m->maskW + t * m->n3, *maskS = m->maskS + t * m->n3;
    const double *recip_dxC = m->recip_dxC + t * n2, *recip_dyC = m->recip_dyC + t * n2;
    double *rhoInSitu = m->rhoInSitu + t * m->n3, *conv = m->IVDConvCount + t * m->n3;
    double *sigmaX = m->sigmaX + t * m->n3, *sigmaY = m->sigmaY + t * m->n3, *sigmaR = m->sigmaR + t * m->n3;
    for (long p = 0; p < m->n3; p++) { sigmaX[p] = 0.0; sigmaY[p] = 0.0; sigmaR[p] = 0.0; conv[p] = 0.0; }
    /* FIND_RHO_2D for every level, kRef = k (do_oceanic_phys.F:753-761) */
    for (int k = 1; k <= Nr; k++)
      for (int j = 1 - OLy; j <= sNy + OLy; j++)
        for (int i = 1 - OLx; i <= sNx + OLx; i++)
          W3(rhoInSitu, i, j, k) = oracle_find_rho_p(m, k, W3(theta, i, j, k), W3(salt, i, j, k),
                                                     oracle_pressure_for_eos(m, k, t * m->n3 + W3I(i, j, k)));
    /* k = Nr..1 (do_oceanic_phys.F:799-882): GRAD_SIGMA with rho(theta(k-1), kRef = k),
     * CALC_IVDC */
    if (m->useGMRedi || calcConvect) {
      for (int k = Nr; k >= 1; k--) {
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx + 1; i <= sNx + OLx; i++)
            W3(sigmaX, i, j, k) = W3(maskW, i, j, k) * L(recip_dxC, i, j) *
                                  (W3(rhoInSitu, i, j, k) - W3(rhoInSitu, i - 1, j, k));
        for (int j = 1 - OLy + 1; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++)
            W3(sigmaY, i, j, k) = W3(maskS, i, j, k) * L(recip_dyC, i, j) *
                                  (W3(rhoInSitu, i, j, k) - W3(rhoInSitu, i, j - 1, k));
        if (k > 1)
          for (int j = 1 - OLy; j <= sNy + OLy; j++)
            for (int i = 1 - OLx; i <= sNx + OLx; i++) {
              const double rhoKp1 = W3(rhoInSitu, i, j, k);
              const double rhoKm1 = oracle_find_rho_p(m, k, W3(theta, i, j, k - 1), W3(salt, i, j, k - 1),
                                                      oracle_pressure_for_eos(m, k, t * m->n3 + W3I(i, j, k)));
              W3(sigmaR, i, j, k) = W3(maskC, i, j, k) * W3(maskC, i, j, k - 1) * m->recip_drC[k - 1] * m->rkSign *
                                    (rhoKp1 - rhoKm1);
              if (calcConvect) W3(conv, i, j, k) = (-W3(sigmaR, i, j, k) * m->gravitySign > 0.0) ? 1.0 : 0.0;
            }
      }
    }
    if (m->useGMRedi) oracle_gmredi_calc_tensor(m, t);
  }
}

/* ---------------------------------------------------------------------------
 * GAD_DST3FL_ADV_X/Y/R (gad_dst3fl_adv_x.F:47-99, _y, _r.F:70-119): face flux
 * of the 3rd-order direct-space-time scheme with flux limiter.  Returns the
 * flux through the face between cells "m1" (upstream for positive transport)
 * and "p0", given the four cells m2, m1, p0, p1 along the transport direction
 * (for R: m2 = km2 .. p1 = kp1 as the reference orders them).
 */
static const double thetaMax = 1.0e+20, oneSixth = 1.0 / 6.0;

static double dst3fl_limit(double d0, double d1, double theta, double cfl) {
  double psi = d0 + d1 * theta;
  return fmax(0.0, fmin(fmin(1.0, psi), theta * (1.0 - cfl) / (cfl + 1.0e-20)));
}
static double dst3fl_theta(double Rj, double Rother) {
  if (fabs(Rj) * thetaMax <= fabs(Rother)) return copysign(thetaMax, Rother * Rj);
  return Rother / Rj;
}
/* horizontal: Rjp = (T(i+1)-T(i))*mW(i+1), Rj = (T(i)-T(i-1))*mW(i), Rjm = (T(i-1)-T(i-2))*mW(i-1) */
/* lim = 0: GAD_DST3_ADV_X/Y (gad_dst3_adv_x.F:71-118, scheme 30; OLD_DST3_FORMULATION undefined) */
static int dst3_lim = 1;   /* set per tracer by gad_advection_dst3fl */
static double dst3fl_h(double uTr, double cfl, double tm2, double tm1, double t0, double tp1,
                       double mWm1, double mW0, double mWp1) {
  const double Rjp = (tp1 - t0) * mWp1, Rj = (t0 - tm1) * mW0, Rjm = (tm1 - tm2) * mWm1;
  const double d0 = (2.0 - cfl) * (1.0 - cfl) * oneSixth, d1 = (1.0 - cfl * cfl) * oneSixth;
  if (!dst3_lim)
    return 0.5 * (uTr + fabs(uTr)) * (tm1 + (d0 * Rj + d1 * Rjm)) + 0.5 * (uTr - fabs(uTr)) * (t0 - (d0 * Rj + d1 * Rjp));
  const double psiP = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjm), cfl);
  const double psiM = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjp), cfl);
  return 0.5 * (uTr + fabs(uTr)) * (tm1 + psiP * Rj) + 0.5 * (uTr - fabs(uTr)) * (t0 - psiM * Rj);
}

/* FILL_CS_CORNER_TR_RL (eesupp/src/fill_cs_corner_tr_rl.F): the halo corners of a cube
 * tile filled from the neighbouring halo strip, for X (dir 1) or Y (dir 2) stencils. */
static void fill_cs_corner_tr(const OModel *m, int dir, double *a, int edges) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, nx = m->nx;
  const int N = edges & 1, S = edges & 2, E = edges & 4, W = edges & 8;
  for (int j = 1; j <= OLy; j++)
    for (int i = 1; i <= OLx; i++) {
      if (W && S) L(a, 1 - i, 1 - j) = dir == 1 ? L(a, 1 - j, i) : L(a, j, 1 - i);
      if (E && S) L(a, sNx + i, 1 - j) = dir == 1 ? L(a, sNx + j, i) : L(a, sNx + 1 - j, 1 - i);
      if (W && N) L(a, 1 - i, sNy + j) = dir == 1 ? L(a, 1 - j, sNy + 1 - i) : L(a, j, sNy + i);
      if (E && N) L(a, sNx + i, sNy + j) = dir == 1 ? L(a, sNx + j, sNy + 1 - i) : L(a, sNx + 1 - j, sNy + i);
    }
}
/* FILL_CS_CORNER_UV_RS(withSigns = .FALSE.) (eesupp/src/fill_cs_corner_uv_rs.F) on the
 * local masks maskLocW (u) and maskLocS (v), corner by corner in the reference's order. */
static void fill_cs_corner_uv(const OModel *m, double *u, double *v, int edges) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, nx = m->nx;
  const int N = edges & 1, S = edges & 2, E = edges & 4, W = edges & 8;
  if (W && S) {
    for (int j = 1; j <= OLy; j++) for (int i = 1; i <= OLx; i++) L(u, 1 - i, 1 - j) = L(v, 1 - j, 1 + i);
    for (int j = 1; j <= OLy; j++) for (int i = 1; i <= OLx; i++) L(v, 1 - i, 1 - j) = L(u, 1 + j, 1 - i);
  }
  if (E && S) {
    for (int j = 1; j <= OLy; j++) for (int i = 2; i <= OLx; i++) L(u, sNx + i, 1 - j) = L(v, sNx + j, i);
    for (int j = 1; j <= OLy; j++) for (int i = 1; i <= OLx; i++) L(v, sNx + i, 1 - j) = L(u, sNx + 1 - j, 1 - i);
  }
  if (W && N) {
    for (int j = 1; j <= OLy; j++) for (int i = 1; i <= OLx; i++) L(u, 1 - i, sNy + j) = L(v, 1 - j, sNy + 1 - i);
    for (int j = 2; j <= OLy; j++) for (int i = 1; i <= OLx; i++) L(v, 1 - i, sNy + j) = L(u, j, sNy + i);
  }
  if (E && N) {
    for (int j = 1; j <= OLy; j++) for (int i = 2; i <= OLx; i++) L(u, sNx + i, sNy + j) = L(v, sNx + j, sNy + 2 - i);
    for (int j = 2; j <= OLy; j++) for (int i = 1; i <= OLx; i++) L(v, sNx + i, sNy + j) = L(u, sNx + 2 - j, sNy + i);
  }
}

/* GAD_ADVECTION (gad_advection.F:292-1097) for one tile, explicit, advectionScheme = 33.
 * Lat-lon: npass = 2 (X then Y).  Cube (EXCH2 tiles, useCubedSphereExchange): npass = 3,
 * the direction of each pass and whether it updates the tile's interior, its overlap only,
 * or both chosen by the tile's face (:339-367), with FILL_CS_CORNER_TR_RL before / after the
 * fluxes of overlap-only passes and FILL_CS_CORNER_UV_RS on the local masks.
 * GAD_MULTIDIM_COMPRESSIBLE (m->multiDimCompressible): the volume-weighted update with the
 * local volume carried through the passes.  Writes the advective tendency into gTr. */
static void gad_advection_dst3fl(const OModel *m, int t, const double *tr, const double *uVel, const double *vVel,
                                 const double *wVel, double *gTr, double dT) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long n2 = m->n2, n3 = m->n3;
  const int cube = m->tileFace != NULL, comp = m->multiDimCompressible;
  const int face = cube ? m->tileFace[t] : 0, edges = cube ? m->tileEdge[t] : 0;
  const int Ned = edges & 1, Sed = edges & 2, Eed = edges & 4, Wed = edges & 8;
  const double *hFacW = m->hFacW + t * n3, *hFacS = m->hFacS + t * n3, *maskW = m->maskW + t * n3;
  const double *maskS = m->maskS + t * n3, *maskC = m->maskC + t * n3, *rhFacC = m->recip_hFacC + t * n3;
  const double *hFacC = m->hFacC + t * n3;
  const double *dxG = m->dxG + t * n2, *dyG = m->dyG + t * n2, *rA = m->rA + t * n2, *recip_rA = m->recip_rA + t * n2;
  const double *recip_dxC = m->recip_dxC + t * n2, *recip_dyC = m->recip_dyC + t * n2, *maskInC = m->maskInC + t * n2;
  double *uTrans = calloc(n2, 8), *vTrans = calloc(n2, 8), *loc = calloc(n2, 8), *af = calloc(n2, 8);
  double *locT3d = calloc(n3, 8), *rTrans = calloc(n2, 8), *rTransKp = calloc(n2, 8), *fV[2];
  double *vol = calloc(n2, 8), *vol3d = calloc(n3, 8), *mLW = calloc(n2, 8), *mLS = calloc(n2, 8);
  fV[0] = calloc(n2, 8); fV[1] = calloc(n2, 8);
  /* one cell's update by the X (dir 0) or Y (dir 1) flux divergence */
#define UPD(i, j, dir)                                                                                         \
  do {                                                                                                         \
    const double dF = dir ? L(af, i, (j) + 1) - L(af, i, j) : L(af, (i) + 1, j) - L(af, i, j);                 \
    const double dU = dir ? L(vTrans, i, (j) + 1) - L(vTrans, i, j) : L(uTrans, (i) + 1, j) - L(uTrans, i, j); \
    if (comp) {                                                                                                \
      const double tmpTrac = L(loc, i, j) * L(vol, i, j) - dT * dF * L(maskInC, i, j);                        \
      L(vol, i, j) = L(vol, i, j) - dT * dU * L(maskInC, i, j);                                                \
      L(loc, i, j) = tmpTrac / L(vol, i, j);                                                                   \
    } else {                                                                                                   \
      L(loc, i, j) = L(loc, i, j) - dT * W3(rhFacC, i, j, k) * m->recip_drF[k - 1] * L(recip_rA, i, j) *      \
                                        (dF - W3(tr, i, j, k) * dU) * L(maskInC, i, j);                        \
    }                                                                                                          \
  } while (0)
  for (int k = 1; k <= Nr; k++) {
    for (int j = 1 - OLy; j <= sNy + OLy; j++)
      for (int i = 1 - OLx; i <= sNx + OLx; i++) {
        const double xA = L(dyG, i, j) * m->drF[k - 1] * W3(hFacW, i, j, k);
        const double yA = L(dxG, i, j) * m->drF[k - 1] * W3(hFacS, i, j, k);
        L(uTrans, i, j) = W3(uVel, i, j, k) * xA;
        L(vTrans, i, j) = W3(vVel, i, j, k) * yA;
        L(loc, i, j) = W3(tr, i, j, k);
        if (comp) L(vol, i, j) = L(rA, i, j) * m->drF[k - 1] * W3(hFacC, i, j, k) + (1.0 - W3(maskC, i, j, k));
        L(mLW, i, j) = W3(maskW, i, j, k);
        L(mLS, i, j) = W3(maskS, i, j, k);
      }
    if (cube) fill_cs_corner_uv(m, mLW, mLS, edges);
    const int npass = cube ? 3 : 2;
    for (int ipass = 1; ipass <= npass; ipass++) {
      int overlapOnly = 0, interiorOnly = 0, calcX, calcY;
      if (cube) {
        if (ipass == 1) {
          overlapOnly = face % 3 == 0; interiorOnly = face % 3 != 0;
          calcX = face == 6 || face == 1 || face == 2; calcY = face == 3 || face == 4 || face == 5;
        } else if (ipass == 2) {
          overlapOnly = face % 3 == 2; interiorOnly = face % 3 == 1;
          calcX = face == 2 || face == 3 || face == 4; calcY = face == 5 || face == 6 || face == 1;
        } else {
          interiorOnly = 1;
          calcX = face == 5 || face == 6; calcY = face == 2 || face == 3;
        }
      } else {
        calcX = ipass % 2 == 1; calcY = !calcX;
      }
      /* X direction: GAD_DST3FL_ADV_X over i = 3-OLx..sNx+OLx-1 (af = 0 elsewhere) */
      if (calcX) {
        if (!overlapOnly || Ned || Sed) {
          if (overlapOnly) fill_cs_corner_tr(m, 1, loc, edges);
          for (long p = 0; p < n2; p++) af[p] = 0.0;
          for (int j = 1 - OLy; j <= sNy + OLy; j++)
            for (int i = 3 - OLx; i <= sNx + OLx - 1; i++) {
              const double cfl = fabs(W3(uVel, i, j, k) * dT * L(recip_dxC, i, j));
              L(af, i, j) = dst3fl_h(L(uTrans, i, j), cfl, L(loc, i - 2, j), L(loc, i - 1, j), L(loc, i, j),
                                     L(loc, i + 1, j), L(mLW, i - 1, j), L(mLW, i, j), L(mLW, i + 1, j));
            }
          if (overlapOnly && ipass == 1) fill_cs_corner_tr(m, 2, loc, edges);
        }
        if (overlapOnly) {
          const int iMin = Wed ? 1 : 2 - OLx, iMax = Eed ? sNx : sNx + OLx - 1;
          if (Sed) for (int j = 1 - OLy; j <= 0; j++) for (int i = iMin; i <= iMax; i++) UPD(i, j, 0);
          if (Ned) for (int j = sNy + 1; j <= sNy + OLy; j++) for (int i = iMin; i <= iMax; i++) UPD(i, j, 0);
        } else {
          const int jMin = (interiorOnly && Sed) ? 1 : 1 - OLy, jMax = (interiorOnly && Ned) ? sNy : sNy + OLy;
          for (int j = jMin; j <= jMax; j++) for (int i = 2 - OLx; i <= sNx + OLx - 1; i++) UPD(i, j, 0);
        }
      }
      /* Y direction: GAD_DST3FL_ADV_Y over j = 3-OLy..sNy+OLy-1 */
      for (long p = 0; p < n2; p++) af[p] = 0.0;
      if (calcY) {
        if (!overlapOnly || Eed || Wed) {
          if (overlapOnly) fill_cs_corner_tr(m, 2, loc, edges);
          for (long p = 0; p < n2; p++) af[p] = 0.0;
          for (int j = 3 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 1 - OLx; i <= sNx + OLx; i++) {
              const double cfl = fabs(W3(vVel, i, j, k) * dT * L(recip_dyC, i, j));
              L(af, i, j) = dst3fl_h(L(vTrans, i, j), cfl, L(loc, i, j - 2), L(loc, i, j - 1), L(loc, i, j),
                                     L(loc, i, j + 1), L(mLS, i, j - 1), L(mLS, i, j), L(mLS, i, j + 1));
            }
          if (overlapOnly && ipass == 1) fill_cs_corner_tr(m, 1, loc, edges);
        }
        if (overlapOnly) {
          const int jMin = Sed ? 1 : 2 - OLy, jMax = Ned ? sNy : sNy + OLy - 1;
          if (Wed) for (int j = jMin; j <= jMax; j++) for (int i = 1 - OLx; i <= 0; i++) UPD(i, j, 1);
          if (Eed) for (int j = jMin; j <= jMax; j++) for (int i = sNx + 1; i <= sNx + OLx; i++) UPD(i, j, 1);
        } else {
          const int iMin = (interiorOnly && Wed) ? 1 : 1 - OLx, iMax = (interiorOnly && Eed) ? sNx : sNx + OLx;
          for (int j = 2 - OLy; j <= sNy + OLy - 1; j++) for (int i = iMin; i <= iMax; i++) UPD(i, j, 1);
        }
      }
    }
#undef UPD
    for (int j = 1 - OLy; j <= sNy + OLy; j++)
      for (int i = 1 - OLx; i <= sNx + OLx; i++) {
        W3(locT3d, i, j, k) = L(loc, i, j);
        if (comp) W3(vol3d, i, j, k) = L(vol, i, j);
      }
  }
  /* vertical: k = Nr..1, GAD_DST3FL_ADV_R on the horizontally-updated tracer */
  for (long p = 0; p < n2; p++) { rTrans[p] = 0.0; fV[0][p] = fV[1][p] = 0.0; }
  for (int k = Nr; k >= 1; k--) {
    const int kUp = 1 + (k + 1) % 2, kDown = 1 + k % 2;
    const double kp1Msk = (k == Nr) ? 0.0 : 1.0;
    double *fUp = fV[kUp - 1], *fDn = fV[kDown - 1];
    const int km2 = k - 2 > 1 ? k - 2 : 1, km1 = k - 1 > 1 ? k - 1 : 1, kp1 = k + 1 < Nr ? k + 1 : Nr;
    for (int j = 1 - OLy; j <= sNy + OLy; j++)
      for (int i = 1 - OLx; i <= sNx + OLx; i++) {
        L(rTransKp, i, j) = kp1Msk * L(rTrans, i, j);
        if (k == 1) {
          L(rTrans, i, j) = 0.0;
          L(fUp, i, j) = 0.0;
        } else {
          L(rTrans, i, j) = W3(wVel, i, j, k) * L(rA, i, j) * W3(maskC, i, j, k - 1);
          L(fUp, i, j) = 0.0;
          const double Rjp = (W3(locT3d, i, j, k) - W3(locT3d, i, j, kp1)) * W3(maskC, i, j, kp1);
          const double Rj = (W3(locT3d, i, j, km1) - W3(locT3d, i, j, k)) * W3(maskC, i, j, k) * W3(maskC, i, j, km1);
          const double Rjm = (W3(locT3d, i, j, km2) - W3(locT3d, i, j, km1)) * W3(maskC, i, j, km1);
          const double cfl = fabs(W3(wVel, i, j, k) * dT * m->recip_drC[k - 1]);
          const double d0 = (2.0 - cfl) * (1.0 - cfl) * oneSixth, d1 = (1.0 - cfl * cfl) * oneSixth;
          const double rT = L(rTrans, i, j);
          if (!dst3_lim) {   /* GAD_DST3_ADV_R (gad_dst3_adv_r.F:70-119) */
            L(fUp, i, j) = 0.5 * (rT + fabs(rT)) * (W3(locT3d, i, j, k) + (d0 * Rj + d1 * Rjp)) +
                           0.5 * (rT - fabs(rT)) * (W3(locT3d, i, j, km1) - (d0 * Rj + d1 * Rjm));
            continue;
          }
          const double psiP = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjm), cfl);
          const double psiM = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjp), cfl);
          L(fUp, i, j) = 0.5 * (rT + fabs(rT)) * (W3(locT3d, i, j, k) + psiM * Rj) +
                         0.5 * (rT - fabs(rT)) * (W3(locT3d, i, j, km1) - psiP * Rj);
        }
      }
    for (int j = 1 - OLy; j <= sNy + OLy; j++)
      for (int i = 1 - OLx; i <= sNx + OLx; i++) {
        if (comp) {   /* gad_advection.F:1036-1057 */
          const double tmpTrac = W3(locT3d, i, j, k) * W3(vol3d, i, j, k) -
                                 dT * (L(fDn, i, j) - L(fUp, i, j)) * m->rkSign * L(maskInC, i, j);
          const double lv = W3(vol3d, i, j, k) - dT * (L(rTransKp, i, j) - L(rTrans, i, j)) * m->rkSign * L(maskInC, i, j);
          W3(gTr, i, j, k) = (tmpTrac - W3(tr, i, j, k) * lv) * L(recip_rA, i, j) * m->recip_drF[k - 1] *
                             W3(rhFacC, i, j, k) / dT;
          continue;
        }
        const double lt = W3(locT3d, i, j, k) -
                          dT * W3(rhFacC, i, j, k) * m->recip_drF[k - 1] * L(recip_rA, i, j) *
                              (L(fDn, i, j) - L(fUp, i, j) - W3(tr, i, j, k) * (L(rTransKp, i, j) - L(rTrans, i, j))) *
                              m->rkSign * L(maskInC, i, j);
        W3(gTr, i, j, k) = (lt - W3(tr, i, j, k)) / dT;
      }
  }
  free(uTrans); free(vTrans); free(loc); free(af); free(locT3d); free(rTrans); free(rTransKp); free(fV[0]); free(fV[1]);
  free(vol); free(vol3d); free(mLW); free(mLS);
}

/* One tracer through TEMP_INTEGRATE / SALT_INTEGRATE (temp_integrate.F, salt_integrate.F). */
typedef struct {
  double *tr, *gNm1;        /* tracer, its AB2 tendency history (AB3: gtNm(:,:,:,1)) */
  double *gNm2;             /* AB3: gtNm(:,:,:,2) */
  const double *sfc;        /* surface forcing (surfaceForcingT/S), may be NULL */
  double diffKh, diffKr;
  int advScheme, vAdvScheme, advection, forcing;
} TracerSpec;

static void tracer_integrate(OModel *m, const TracerSpec *c) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long n2 = m->n2, n3 = m->n3;
  const int multiDim = m->multiDimAdvection && c->advection && c->advScheme != 2 && c->advScheme != 3 && c->advScheme != 4;
  const int useAB = (c->advScheme == 2 || c->advScheme == 3 || c->advScheme == 4);   /* gad_init_fixed.F:144-162 */
  if (!(c->advScheme == 2 || c->advScheme == 3 || c->advScheme == 4 ||
        ((c->advScheme == 30 || c->advScheme == 33) && multiDim)) || c->vAdvScheme != c->advScheme) {
    fprintf(stderr, "oracle tracer_integrate: advection scheme %d/%d not restated\n", c->advScheme, c->vAdvScheme); abort();
  }
#pragma omp parallel if (m->nThreads > 1) num_threads(m->nThreads > 1 ? m->nThreads : 1)
  {
  double *gT = calloc(n3, 8), *kappaRT = calloc(n3, 8);
  double *a3 = calloc(n3, 8), *b3 = calloc(n3, 8), *c3 = calloc(n3, 8), *cp = calloc(n3, 8), *yp = calloc(n3, 8);
  double *fVer[2], *xA = calloc(n2, 8), *yA = calloc(n2, 8), *uTrans = calloc(n2, 8), *vTrans = calloc(n2, 8);
  double *rTrans = calloc(n2, 8), *rTransKp = calloc(n2, 8), *maskUp = calloc(n2, 8), *gtForc = calloc(n2, 8);
  double *fZon = calloc(n2, 8), *fMer = calloc(n2, 8), *af = calloc(n2, 8), *df = calloc(n2, 8);
  fVer[0] = calloc(n2, 8); fVer[1] = calloc(n2, 8);
  double *uRes = calloc(n3, 8), *vRes = calloc(n3, 8), *wRes = calloc(n3, 8), *dTdz = calloc(n2, 8);
  const int calcAdvection = c->advection && !multiDim;
  const double advFac = calcAdvection ? 1.0 : 0.0, rAdvFac = m->rkSign * advFac;
  const double abFac = (m->myIter == m->nIter0 && m->nIter0 == 0) ? 0.0 : 0.5 + m->abEps; /* startAB = nIter0 */
  /* ADAMS_BASHFORTH3 (adams_bashforth3.F:60-78): startAB = nIter0 (ini_model_io.F:117), history
   * slots m1 = 1 + MOD(iter+1,2), m2 = 1 + MOD(iter,2) of gtNm(:,:,:,1:2) = (gNm1, gNm2) */
  double ab0 = 0.0, ab1 = 0.0, ab2 = 0.0;
  {
    const int it = m->myIter, n0 = m->nIter0, startAB = m->nIter0;
    if (it == n0 && startAB == 0) { ab0 = 0.0; ab1 = 0.0; ab2 = 0.0; }
    else if ((it == n0 && startAB == 1) || (it == 1 + n0 && startAB == 0)) { ab0 = m->alph_AB; ab1 = -m->alph_AB; ab2 = 0.0; }
    else { ab0 = m->alph_AB + m->beta_AB; ab1 = -m->alph_AB - 2. * m->beta_AB; ab2 = m->beta_AB; }
  }
  const int abM1 = 1 + (m->myIter + 1) % 2;
  const int rstar = m->nonlinFreeSurf > 0 && m->select_rStar > 0;

#pragma omp for schedule(dynamic, 1)
  for (int t = 0; t < m->nTiles; t++) {
    double *theta = c->tr + t * n3, *gtNm1 = c->gNm1 + t * n3;
    double *gtA = m->useAB3 ? (abM1 == 1 ? gtNm1 : c->gNm2 + t * n3) : NULL;   /* gtNm(m1) */
    double *gtB = m->useAB3 ? (abM1 == 1 ? c->gNm2 + t * n3 : gtNm1) : NULL;   /* gtNm(m2) */
    const double *dxG = m->dxG + t * n2, *dyG = m->dyG + t * n2, *rA = m->rA + t * n2;
    const double *recip_rA = m->recip_rA + t * n2, *recip_dxC = m->recip_dxC + t * n2;
    const double *uVel = m->uVel + t * n3, *vVel = m->vVel + t * n3, *wVel = m->wVel + t * n3;
    const double *hFacW = m->hFacW + t * n3, *hFacS = m->hFacS + t * n3, *maskC = m->maskC + t * n3;
    if (m->useGMRedi && m->GM_AdvForm) {
      /* thermodynamics.F:252-268: uFld = uVel (+ GMREDI_RESIDUAL_FLOW's bolus velocity,
       * gmredi_residual_flow.F:58-97, z-coordinates: flipSign4LHCoord = -gravitySign = 1) */
      const double *PsiX = m->GM_PsiX + t * n3, *PsiY = m->GM_PsiY + t * n3;
      const double *rhW = m->recip_hFacW + t * n3, *rhS = m->recip_hFacS + t * n3;
      const double flip = -m->gravitySign;
      for (long p = 0; p < n3; p++) { uRes[p] = uVel[p]; vRes[p] = vVel[p]; wRes[p] = wVel[p]; }
      for (int k = 1; k <= Nr; k++) {
        const int kp1 = k + 1 < Nr ? k + 1 : Nr;
        const double maskp1 = k >= Nr ? 0.0 : 1.0;
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) {
            double delPsi = W3(PsiX, i, j, kp1) * 1.0 * maskp1 - W3(PsiX, i, j, k) * 1.0;
            W3(uRes, i, j, k) = W3(uRes, i, j, k) + delPsi * m->recip_drF[k - 1] * W3(rhW, i, j, k) * 1.0 * flip;
            delPsi = W3(PsiY, i, j, kp1) * 1.0 * maskp1 - W3(PsiY, i, j, k) * 1.0;
            W3(vRes, i, j, k) = W3(vRes, i, j, k) + delPsi * m->recip_drF[k - 1] * W3(rhS, i, j, k) * 1.0 * flip;
          }
        for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
          for (int i = 1 - OLx; i <= sNx + OLx - 1; i++) {
            const double delPsi = (L(dyG, i + 1, j) * W3(PsiX, i + 1, j, k) - L(dyG, i, j) * W3(PsiX, i, j, k) +
                                   L(dxG, i, j + 1) * W3(PsiY, i, j + 1, k) - L(dxG, i, j) * W3(PsiY, i, j, k));
            W3(wRes, i, j, k) = W3(wRes, i, j, k) + delPsi * L(recip_rA, i, j) * 1.0 * flip;
          }
      }
      uVel = uRes; vVel = vRes; wVel = wRes;
    }
    const double *rhFacC = m->recip_hFacC + t * n3, *conv = m->IVDConvCount + t * n3;

    const double *recip_dyC = m->recip_dyC + t * n2, *maskInC = m->maskInC + t * n2;
    const double *sfT = c->sfc ? c->sfc + t * n2 : NULL;
    const double *Kwx = m->Kwx + t * n3, *Kwy = m->Kwy + t * n3, *Kwz = m->Kwz + t * n3;
    const double *Kux = m->Kux + t * n3, *Kvy = m->Kvy + t * n3, *maskW = m->maskW + t * n3;
    const double *maskS = m->maskS + t * n3;
    const double *rStarExpC = m->rStarExpC + t * n2;

    /* CALC_3D_DIFFUSIVITY: KappaR = IVDConvCount*ivdc_kappa + KbryanLewis79(=0) + diffKrNr(k) */
    for (int k = 1; k <= Nr; k++)
      for (int j = 1 - OLy; j <= sNy + OLy; j++)
        for (int i = 1 - OLx; i <= sNx + OLx; i++)
          W3(kappaRT, i, j, k) = (W3(conv, i, j, k) * m->ivdc_kappa + 0.0) + c->diffKr;
    /* GMREDI_CALC_DIFF (gmredi_calc_diff.F:57-70) over iMin..iMax = 0..sNx+1 */
    if (m->useGMRedi)
      for (int k = 1; k <= Nr; k++)
        for (int j = 0; j <= sNy + 1; j++)
          for (int i = 0; i <= sNx + 1; i++)
            W3(kappaRT, i, j, k) = W3(kappaRT, i, j, k) + W3(Kwz, i, j, k) * L(maskInC, i, j);
    for (long p = 0; p < n3; p++) gT[p] = 0.0;
    dst3_lim = c->advScheme == 33;
    if (multiDim) gad_advection_dst3fl(m, t, theta, uVel, vVel, wVel, gT, m->deltaTtracer);
    for (long p = 0; p < n2; p++) { fVer[0][p] = fVer[1][p] = 0.0; rTrans[p] = 0.0; }

    for (int k = Nr; k >= 1; k--) {
      const int kM1 = k > 1 ? k - 1 : 1, kUp = 1 + (k + 1) % 2, kDown = 1 + k % 2;
      double *fVerUp = fVer[kUp - 1], *fVerDn = fVer[kDown - 1];
      /* CALC_ADV_FLOW */
      for (int j = 1 - OLy; j <= sNy + OLy; j++)
        for (int i = 1 - OLx; i <= sNx + OLx; i++) {
          L(xA, i, j) = L(dyG, i, j) * m->drF[k - 1] * W3(hFacW, i, j, k);
          L(yA, i, j) = L(dxG, i, j) * m->drF[k - 1] * W3(hFacS, i, j, k);
          L(rTransKp, i, j) = (k == Nr) ? 0.0 : L(rTrans, i, j);
          L(uTrans, i, j) = W3(uVel, i, j, k) * L(xA, i, j);
          L(vTrans, i, j) = W3(vVel, i, j, k) * L(yA, i, j);
          if (k == 1) {
            L(maskUp, i, j) = 0.0; L(rTrans, i, j) = 0.0;
          } else {
            L(maskUp, i, j) = W3(maskC, i, j, k - 1) * W3(maskC, i, j, k);
            L(rTrans, i, j) = W3(wVel, i, j, k) * L(rA, i, j) * L(maskUp, i, j);
          }
        }
      /* APPLY_FORCING_T/S: surface flux at k = kSurface = 1 over 0..sNx+1 */
      for (long p = 0; p < n2; p++) gtForc[p] = 0.0;
      if (c->forcing && sfT && k == 1)
        for (int j = 0; j <= sNy + 1; j++)
          for (int i = 0; i <= sNx + 1; i++)
            L(gtForc, i, j) = L(gtForc, i, j) + L(sfT, i, j) * m->recip_drF[k - 1] * W3(rhFacC, i, j, k);
      /* GAD_CALC_RHS */
      for (long p = 0; p < n2; p++) { fZon[p] = 0.0; fMer[p] = 0.0; fVerUp[p] = 0.0; df[p] = 0.0; }
      if (calcAdvection && c->advScheme == 2) { /* GAD_C2_ADV_X */
        for (int j = 1 - OLy; j <= sNy + OLy; j++) {
          L(af, 1 - OLx, j) = 0.0;
          for (int i = 2 - OLx; i <= sNx + OLx; i++)
            L(af, i, j) = L(uTrans, i, j) * (W3(theta, i, j, k) + W3(theta, i - 1, j, k)) * 0.5;
        }
        for (long p = 0; p < n2; p++) fZon[p] = fZon[p] + af[p];
      } else if (calcAdvection) {
        /* GAD_U3_ADV_X (gad_u3_adv_x.F:70-92) / GAD_C4_ADV_X (gad_c4_adv_x.F:70-93); maskLocW =
         * maskW(k) (gad_calc_rhs.F:262-268, no OBCS) */
        const double oneSixth = 1.0 / 6.0;
        for (int j = 1 - OLy; j <= sNy + OLy; j++) {
          L(af, 1 - OLx, j) = 0.0; L(af, 2 - OLx, j) = 0.0; L(af, sNx + OLx, j) = 0.0;
          for (int i = 1 - OLx + 2; i <= sNx + OLx - 1; i++) {
            const double Rjp = (W3(theta, i + 1, j, k) - W3(theta, i, j, k)) * W3(maskW, i + 1, j, k);
            const double Rj = (W3(theta, i, j, k) - W3(theta, i - 1, j, k)) * W3(maskW, i, j, k);
            const double Rjm = (W3(theta, i - 1, j, k) - W3(theta, i - 2, j, k)) * W3(maskW, i - 1, j, k);
            const double Rjjp = Rjp - Rj, Rjjm = Rj - Rjm;
            const double uTr = L(uTrans, i, j);
            double v = uTr * (W3(theta, i, j, k) + W3(theta, i - 1, j, k) - oneSixth * (Rjjp + Rjjm)) * 0.5;
            if (c->advScheme == 3) v = v + fabs(uTr) * 0.5 * oneSixth * (Rjjp - Rjjm);
            else v = v + fabs(uTr) * 0.5 * oneSixth * (Rjjp - Rjjm) *
                             (1.0 - W3(maskW, i - 1, j, k) * W3(maskW, i + 1, j, k));
            L(af, i, j) = v;
          }
        }
        for (long p = 0; p < n2; p++) fZon[p] = fZon[p] + af[p];
      }
      if (c->diffKh != 0.0) { /* GAD_DIFF_X, cosFacU = 1 */
        for (int j = 1 - OLy; j <= sNy + OLy; j++) {
          L(df, 1 - OLx, j) = 0.0;
          for (int i = 2 - OLx; i <= sNx + OLx; i++)
            L(df, i, j) = -c->diffKh * L(xA, i, j) * L(recip_dxC, i, j) * (W3(theta, i, j, k) - W3(theta, i - 1, j, k));
        }
      } else {
        for (long p = 0; p < n2; p++) df[p] = 0.0;
      }
      if (m->useGMRedi) /* GMREDI_XTRANSPORT (gmredi_xtransport.F:94-101), i = iMin..iMax+1 */
        for (int j = 0; j <= sNy + 1; j++)
          for (int i = 0; i <= sNx + 2; i++)
            L(df, i, j) = L(df, i, j) - L(xA, i, j) * W3(Kux, i, j, k) * L(recip_dxC, i, j) *
                                            (W3(theta, i, j, k) - W3(theta, i - 1, j, k));
      if (m->useGMRedi && m->GM_ExtraDiag) { /* gmredi_xtransport.F:117-146 (maskFk = maskUp) */
        const int km1 = k > 1 ? k - 1 : 1, kp1 = k + 1 < Nr ? k + 1 : Nr;
        const double maskp1 = k >= Nr ? 0.0 : 1.0;
        for (int j = 0; j <= sNy + 1; j++)
          for (int i = 0; i <= sNx + 2; i++) {
            L(dTdz, i, j) = 0.5 * (+0.5 * m->recip_drC[k - 1] *
                                       (L(maskUp, i - 1, j) * (W3(theta, i - 1, j, km1) - W3(theta, i - 1, j, k)) +
                                        L(maskUp, i, j) * (W3(theta, i, j, km1) - W3(theta, i, j, k))) +
                                   0.5 * m->recip_drC[kp1 - 1] *
                                       (W3(maskC, i - 1, j, k) * W3(maskC, i - 1, j, kp1) * maskp1 *
                                            (W3(theta, i - 1, j, k) - W3(theta, i - 1, j, kp1)) +
                                        W3(maskC, i, j, k) * W3(maskC, i, j, kp1) * maskp1 *
                                            (W3(theta, i, j, k) - W3(theta, i, j, kp1))));
            L(df, i, j) = L(df, i, j) - L(xA, i, j) * W3(m->Kuz + t * n3, i, j, k) * L(dTdz, i, j);
          }
      }
      for (long p = 0; p < n2; p++) fZon[p] = fZon[p] + df[p];
      if (calcAdvection && c->advScheme == 2) { /* GAD_C2_ADV_Y */
        for (int i = 1 - OLx; i <= sNx + OLx; i++) L(af, i, 1 - OLy) = 0.0;
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++)
            L(af, i, j) = L(vTrans, i, j) * (W3(theta, i, j, k) + W3(theta, i, j - 1, k)) * 0.5;
        for (long p = 0; p < n2; p++) fMer[p] = fMer[p] + af[p];
      } else if (calcAdvection) {   /* GAD_U3_ADV_Y / GAD_C4_ADV_Y (maskLocS = maskS(k)) */
        const double oneSixth = 1.0 / 6.0;
        for (int i = 1 - OLx; i <= sNx + OLx; i++) {
          L(af, i, 1 - OLy) = 0.0; L(af, i, 2 - OLy) = 0.0; L(af, i, sNy + OLy) = 0.0;
        }
        for (int j = 1 - OLy + 2; j <= sNy + OLy - 1; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) {
            const double Rjp = (W3(theta, i, j + 1, k) - W3(theta, i, j, k)) * W3(maskS, i, j + 1, k);
            const double Rj = (W3(theta, i, j, k) - W3(theta, i, j - 1, k)) * W3(maskS, i, j, k);
            const double Rjm = (W3(theta, i, j - 1, k) - W3(theta, i, j - 2, k)) * W3(maskS, i, j - 1, k);
            const double Rjjp = Rjp - Rj, Rjjm = Rj - Rjm;
            const double vTr = L(vTrans, i, j);
            double v = vTr * (W3(theta, i, j, k) + W3(theta, i, j - 1, k) - oneSixth * (Rjjp + Rjjm)) * 0.5;
            if (c->advScheme == 3) v = v + fabs(vTr) * 0.5 * oneSixth * (Rjjp - Rjjm);
            else v = v + fabs(vTr) * 0.5 * oneSixth * (Rjjp - Rjjm) *
                             (1.0 - W3(maskS, i, j - 1, k) * W3(maskS, i, j + 1, k));
            L(af, i, j) = v;
          }
        for (long p = 0; p < n2; p++) fMer[p] = fMer[p] + af[p];
      }
      if (c->diffKh != 0.0) { /* GAD_DIFF_Y */
        for (int i = 1 - OLx; i <= sNx + OLx; i++) L(df, i, 1 - OLy) = 0.0;
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++)
            L(df, i, j) = -c->diffKh * L(yA, i, j) * L(recip_dyC, i, j) * (W3(theta, i, j, k) - W3(theta, i, j - 1, k));
      } else {
        for (long p = 0; p < n2; p++) df[p] = 0.0;
      }
      if (m->useGMRedi) /* GMREDI_YTRANSPORT, j = jMin..jMax+1 */
        for (int j = 0; j <= sNy + 2; j++)
          for (int i = 0; i <= sNx + 1; i++)
            L(df, i, j) = L(df, i, j) - L(yA, i, j) * W3(Kvy, i, j, k) * L(recip_dyC, i, j) *
                                            (W3(theta, i, j, k) - W3(theta, i, j - 1, k));
      if (m->useGMRedi && m->GM_ExtraDiag) { /* gmredi_ytransport.F:117-146 */
        const int km1 = k > 1 ? k - 1 : 1, kp1 = k + 1 < Nr ? k + 1 : Nr;
        const double maskp1 = k >= Nr ? 0.0 : 1.0;
        for (int j = 0; j <= sNy + 2; j++)
          for (int i = 0; i <= sNx + 1; i++) {
            L(dTdz, i, j) = 0.5 * (+0.5 * m->recip_drC[k - 1] *
                                       (L(maskUp, i, j - 1) * (W3(theta, i, j - 1, km1) - W3(theta, i, j - 1, k)) +
                                        L(maskUp, i, j) * (W3(theta, i, j, km1) - W3(theta, i, j, k))) +
                                   0.5 * m->recip_drC[kp1 - 1] *
                                       (W3(maskC, i, j - 1, k) * W3(maskC, i, j - 1, kp1) * maskp1 *
                                            (W3(theta, i, j - 1, k) - W3(theta, i, j - 1, kp1)) +
                                        W3(maskC, i, j, k) * W3(maskC, i, j, kp1) * maskp1 *
                                            (W3(theta, i, j, k) - W3(theta, i, j, kp1))));
            L(df, i, j) = L(df, i, j) - L(yA, i, j) * W3(m->Kvz + t * n3, i, j, k) * L(dTdz, i, j);
          }
      }
      for (long p = 0; p < n2; p++) fMer[p] = fMer[p] + df[p];
      if (calcAdvection && k >= 2 && c->advScheme == 2) { /* GAD_C2_ADV_R */
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) {
            double wT = W3(maskC, i, j, kM1) * L(rTrans, i, j) * (W3(theta, i, j, k) + W3(theta, i, j, kM1)) * 0.5;
            L(fVerUp, i, j) = L(fVerUp, i, j) + wT * L(maskInC, i, j);
          }
      } else if (calcAdvection && k >= 2) {
        /* GAD_U3_ADV_R (gad_u3_adv_r.F:58-88) / GAD_C4_ADV_R (gad_c4_adv_r.F:58-92): km2 = max(1,k-2),
         * kp1 = min(Nr,k+1); U3's Rjm masked at km2, C4's at km1 with C4's boundary term */
        const double oneSixth = 1.0 / 6.0;
        const int km2 = k - 2 > 1 ? k - 2 : 1, km1 = kM1, kp1 = k + 1 < Nr ? k + 1 : Nr;
        const double maskPM = (k <= 2 || k >= Nr) ? 0.0 : 1.0;
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) {
            const double Rjp = (W3(theta, i, j, kp1) - W3(theta, i, j, k)) * W3(maskC, i, j, kp1);
            const double Rj = (W3(theta, i, j, k) - W3(theta, i, j, km1));
            const double Rjm = (W3(theta, i, j, km1) - W3(theta, i, j, km2)) *
                               (c->advScheme == 3 ? W3(maskC, i, j, km2) : W3(maskC, i, j, km1));
            const double Rjjp = Rjp - Rj, Rjjm = Rj - Rjm, rTr = L(rTrans, i, j);
            double wT;
            if (c->advScheme == 3)
              wT = W3(maskC, i, j, km1) * (rTr * ((W3(theta, i, j, k) + W3(theta, i, j, km1)) * 0.5 -
                                                  oneSixth * (Rjjm + Rjjp) * 0.5) +
                                           fabs(rTr) * oneSixth * (Rjjm - Rjjp) * 0.5);
            else {
              const double maskBound = maskPM * W3(maskC, i, j, km2) * W3(maskC, i, j, kp1);
              wT = W3(maskC, i, j, km1) * (rTr * ((W3(theta, i, j, k) + W3(theta, i, j, km1)) * 0.5 -
                                                  oneSixth * (Rjjm + Rjjp) * 0.5) +
                                           fabs(rTr) * oneSixth * (Rjjm - Rjjp) * 0.5 * (1.0 - maskBound));
            }
            L(fVerUp, i, j) = L(fVerUp, i, j) + wT * L(maskInC, i, j);
          }
      }
      /* vertical diffusive flux: 0 with implicitDiffusion, else GAD_DIFF_R */
      for (int j = 1 - OLy; j <= sNy + OLy; j++)
        for (int i = 1 - OLx; i <= sNx + OLx; i++) {
          double dfr = 0.0;
          if (!m->implicitDiffusion && k >= 2)
            dfr = -W3(kappaRT, i, j, k) * L(maskUp, i, j) * L(rA, i, j) * m->recip_drC[k - 1] *
                  (W3(theta, i, j, k) - W3(theta, i, j, kM1)) * m->rkSign;
          L(df, i, j) = dfr;
        }
      if (m->useGMRedi && k > 1) /* GMREDI_RTRANSPORT (gmredi_rtransport.F:75-130), iMin..iMax */
        for (int j = 0; j <= sNy + 1; j++)
          for (int i = 0; i <= sNx + 1; i++) {
            const double dTdx = 0.5 * (0.5 * (W3(maskW, i + 1, j, k) * L(recip_dxC, i + 1, j) *
                                                  (W3(theta, i + 1, j, k) - W3(theta, i, j, k)) +
                                              W3(maskW, i, j, k) * L(recip_dxC, i, j) *
                                                  (W3(theta, i, j, k) - W3(theta, i - 1, j, k))) +
                                       0.5 * (W3(maskW, i + 1, j, k - 1) * L(recip_dxC, i + 1, j) *
                                                  (W3(theta, i + 1, j, k - 1) - W3(theta, i, j, k - 1)) +
                                              W3(maskW, i, j, k - 1) * L(recip_dxC, i, j) *
                                                  (W3(theta, i, j, k - 1) - W3(theta, i - 1, j, k - 1))));
            const double dTdy = 0.5 * (0.5 * (W3(maskS, i, j + 1, k) * L(recip_dyC, i, j + 1) *
                                                  (W3(theta, i, j + 1, k) - W3(theta, i, j, k)) +
                                              W3(maskS, i, j, k) * L(recip_dyC, i, j) *
                                                  (W3(theta, i, j, k) - W3(theta, i, j - 1, k))) +
                                       0.5 * (W3(maskS, i, j + 1, k - 1) * L(recip_dyC, i, j + 1) *
                                                  (W3(theta, i, j + 1, k - 1) - W3(theta, i, j, k - 1)) +
                                              W3(maskS, i, j, k - 1) * L(recip_dyC, i, j) *
                                                  (W3(theta, i, j, k - 1) - W3(theta, i, j - 1, k - 1))));
            L(df, i, j) = L(df, i, j) - L(rA, i, j) * L(maskInC, i, j) *
                                            (W3(Kwx, i, j, k) * dTdx + W3(Kwy, i, j, k) * dTdy) * L(maskUp, i, j);
          }
      for (long p = 0; p < n2; p++) fVerUp[p] = fVerUp[p] + df[p];
      for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
        for (int i = 1 - OLx; i <= sNx + OLx - 1; i++) {
          double T = W3(theta, i, j, k);
          W3(gT, i, j, k) = W3(gT, i, j, k) -
              W3(rhFacC, i, j, k) * m->recip_drF[k - 1] * L(recip_rA, i, j) *
              ((L(fZon, i + 1, j) - L(fZon, i, j)) * L(maskInC, i, j) +
               (L(fMer, i, j + 1) - L(fMer, i, j)) * L(maskInC, i, j) +
               (L(fVerDn, i, j) - L(fVerUp, i, j)) * m->rkSign -
               T * ((L(uTrans, i + 1, j) - L(uTrans, i, j)) * advFac + (L(vTrans, i, j + 1) - L(vTrans, i, j)) * advFac +
                    (L(rTransKp, i, j) - L(rTrans, i, j)) * rAdvFac) * L(maskInC, i, j));
        }
      /* gT += gtForc inside (tracForcingOutAB = 0) or after (= 1) ADAMS_BASHFORTH2(k)
       * (temp_integrate.F:373-410) */
      for (int j = 1 - OLy; j <= sNy + OLy; j++)
        for (int i = 1 - OLx; i <= sNx + OLx; i++) {
          if (!m->tracForcingOutAB) W3(gT, i, j, k) = W3(gT, i, j, k) + L(gtForc, i, j);
          if (useAB && m->useAB3) {   /* ADAMS_BASHFORTH3(k) (adams_bashforth3.F:91-103) */
            const double g = W3(gT, i, j, k);
            const double abG = ab0 * g + ab1 * W3(gtA, i, j, k) + ab2 * W3(gtB, i, j, k);
            W3(gtB, i, j, k) = g;
            W3(gT, i, j, k) = g + abG;
          } else if (useAB) {
            double ab = abFac * (W3(gT, i, j, k) - W3(gtNm1, i, j, k));
            W3(gtNm1, i, j, k) = W3(gT, i, j, k);
            W3(gT, i, j, k) = W3(gT, i, j, k) + ab;
          }
          if (m->tracForcingOutAB) W3(gT, i, j, k) = W3(gT, i, j, k) + L(gtForc, i, j);
        }
      if (rstar)   /* FREESURF_RESCALE_G (freesurf_rescale_g.F:52-62) of gT and gtNm1 (temp_integrate.F:412-446) */
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) {
            W3(gT, i, j, k) = W3(gT, i, j, k) / L(rStarExpC, i, j);
            if (useAB) W3(gtNm1, i, j, k) = W3(gtNm1, i, j, k) / L(rStarExpC, i, j);
          }
    }
    /* TIMESTEP_TRACER: gT = tracer + dTtracerLev(k)*gT */
    for (long p = 0; p < n3; p++) gT[p] = theta[p] + m->deltaTtracer * gT[p];
    if (m->implicitDiffusion) {
      /* GAD_IMPLICIT_R: b5d (sub), c5d (diag), d5d (super) on 1..sNx, 1..sNy */
      for (long p = 0; p < n3; p++) { a3[p] = 0.0; b3[p] = 1.0; c3[p] = 0.0; }
      for (int k = 1; k <= Nr; k++)
        for (int j = 1; j <= sNy; j++)
          for (int i = 1; i <= sNx; i++) {
            double sub = 0.0, sup = 0.0;
            /* recip_hFacNew (thermodynamics.F:198-210): recip_hFacC/rStarExpC under r* */
            const double rhN = rstar ? W3(rhFacC, i, j, k) / L(rStarExpC, i, j) : W3(rhFacC, i, j, k);
            if (k >= 2)
              sub = -(m->deltaTtracer * W3(maskC, i, j, k - 1) * rhN * m->recip_drF[k - 1] *
                      W3(kappaRT, i, j, k) * m->recip_drC[k - 1]);
            if (k <= Nr - 1)
              sup = -(m->deltaTtracer * W3(maskC, i, j, k + 1) * rhN * m->recip_drF[k - 1] *
                      W3(kappaRT, i, j, k + 1) * m->recip_drC[k]);
            W3(a3, i, j, k) = sub; W3(c3, i, j, k) = sup;
            W3(b3, i, j, k) = 1.0 - (sub + sup);
          }
      /* SOLVE_TRIDIAGONAL (default: neither LOWMEMORY nor KINNER), whole tile */
      for (int k = 1; k <= Nr; k++)
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) {
            double y = W3(gT, i, j, k);
            if (k == 1) {
              if (W3(b3, i, j, 1) != 0.0) {
                double rec = 1.0 / W3(b3, i, j, 1);
                W3(cp, i, j, 1) = W3(c3, i, j, 1) * rec;
                W3(yp, i, j, 1) = y * rec;
              } else { W3(cp, i, j, 1) = 0.0; W3(yp, i, j, 1) = 0.0; }
            } else {
              double tmp = W3(b3, i, j, k) - W3(a3, i, j, k) * W3(cp, i, j, k - 1);
              if (tmp != 0.0) {
                double rec = 1.0 / tmp;
                W3(cp, i, j, k) = W3(c3, i, j, k) * rec;
                W3(yp, i, j, k) = (y - W3(a3, i, j, k) * W3(yp, i, j, k - 1)) * rec;
              } else { W3(cp, i, j, k) = 0.0; W3(yp, i, j, k) = 0.0; }
            }
          }
      for (int k = Nr; k >= 1; k--)
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++)
            W3(gT, i, j, k) = (k == Nr) ? W3(yp, i, j, k) : W3(yp, i, j, k) - W3(cp, i, j, k) * W3(gT, i, j, k + 1);
    }
    /* CYCLE_TRACER */
    for (long p = 0; p < n3; p++) theta[p] = gT[p];
  }
  free(gT); free(kappaRT); free(a3); free(b3); free(c3); free(cp); free(yp);
  free(fVer[0]); free(fVer[1]); free(xA); free(yA); free(uTrans); free(vTrans); free(rTrans); free(rTransKp);
  free(maskUp); free(gtForc); free(fZon); free(fMer); free(af); free(df);
  free(uRes); free(vRes); free(wRes); free(dTdz);
  }   /* omp parallel */
}

void oracle_thermodynamics(OModel *m) {
  if (m->tempStepping) {
    TracerSpec c = {m->theta, m->gtNm1, m->gtNm2, m->surfaceForcingT, m->diffKhT, m->diffKrT,
                    m->tempAdvScheme, m->tempVertAdvScheme, m->tempAdvection, m->tempForcing};
    tracer_integrate(m, &c);
  }
  if (m->saltStepping) {
    TracerSpec c = {m->salt, m->gsNm1, m->gsNm2, m->surfaceForcingS, m->diffKhS, m->diffKrS,
                    m->saltAdvScheme, m->saltVertAdvScheme, m->saltAdvection, m->saltForcing};
    tracer_integrate(m, &c);
  }
}
