/*
 * dynamics.c -- oracle restatement of DYNAMICS (model/src/dynamics.F:21-739):
 * MOM_FLUXFORM (pkg/mom_fluxform/mom_fluxform.F:42-1064) and TIMESTEP
 * (model/src/timestep.F:10-429) with ADAMS_BASHFORTH2
 * (model/src/adams_bashforth2.F:6-92), per tile and per level k.
 * TEST INFRASTRUCTURE (see oracle.h).
 */
#include "oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* tile-local 2-D scratch, Fortran indexing (i,j) */
#define L(a, i, j) (a)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx]

static void check_supported(const OModel *m) {
  if ((m->viscA4D != 0.0 || m->viscA4Z != 0.0) && m->OLx < 3) {
    fprintf(stderr, "oracle_dynamics: biharmonic viscosity needs OLx, OLy >= 3\n"); abort();
  }
  if (!m->usingCartesianGrid && !m->usingSphericalPolarGrid &&
      !(m->usingCurvilinearGrid && m->vectorInvariantMomentum)) {
    fprintf(stderr, "oracle_dynamics: grid/momentum-scheme combination not restated\n"); abort();
  }
  if (m->integr_GeoPot != 2) { fprintf(stderr, "oracle_dynamics: integr_GeoPot=%d not restated\n", m->integr_GeoPot); abort(); }
}

/* MOM_U_IMPLICIT_R / MOM_V_IMPLICIT_R (pkg/mom_common/mom_u_implicit_r.F:118-160,
 * mom_v_implicit_r.F), implicitViscosity only (momImplVertAdv = F, selectImplicitDrag = 0;
 * deepFac = rhoFac = 1): tri-diagonal coefficients on i0..i1 x j0..j1 (U: 1..sNx+1 x 1..sNy,
 * V: 1..sNx x 1..sNy+1), identity elsewhere, then SOLVE_TRIDIAGONAL's default branch
 * (solve_tridiagonal.F:224-297) over the whole tile, in place on g (= u* or v*). */
static void mom_implicit_r(const OModel *m, double *g, const double *mask, const double *rhFac,
                           const double *kappa, int i0, int i1, int j0, int j1) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long n2 = m->n2;
  double *sub = malloc(sizeof(double) * Nr), *sup = malloc(sizeof(double) * Nr);
  double *cp = malloc(sizeof(double) * Nr), *yp = malloc(sizeof(double) * Nr);
#define W3(a, i, j, k) (a)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx + (long)((k) - 1) * n2]
#define KAP(i, j, k) kappa[(long)((k) - 1) * n2 + ((i) + OLx - 1) + (long)((j) + OLy - 1) * nx]
  for (int j = 1 - OLy; j <= sNy + OLy; j++)
    for (int i = 1 - OLx; i <= sNx + OLx; i++) {
      const int in = i >= i0 && i <= i1 && j >= j0 && j <= j1;
      for (int k = 1; k <= Nr; k++) {
        double b = 0.0, dd = 0.0;
        if (in && k >= 2 && W3(mask, i, j, k - 1) == 1.0)   /* 1rst lower diagonal (:123-133) */
          b = -(m->deltaTMom * W3(rhFac, i, j, k) * m->recip_drF[k - 1] * KAP(i, j, k) * m->recip_drC[k - 1]);
        if (in && k <= Nr - 1 && W3(mask, i, j, k + 1) == 1.0)   /* 1rst upper diagonal (:135-145) */
          dd = -(m->deltaTMom * W3(rhFac, i, j, k) * m->recip_drF[k - 1] * KAP(i, j, k + 1) * m->recip_drC[k]);
        sub[k - 1] = b; sup[k - 1] = dd;
      }
      for (int k = 1; k <= Nr; k++) {
        const double c = 1.0 - (sub[k - 1] + sup[k - 1]);   /* main diagonal (:147-153) */
        const double y = W3(g, i, j, k);
        if (k == 1) {
          if (c != 0.0) { const double rec = 1.0 / c; cp[0] = sup[0] * rec; yp[0] = y * rec; }
          else { cp[0] = 0.0; yp[0] = 0.0; }
        } else {
          const double tmp = c - sub[k - 1] * cp[k - 2];
          if (tmp != 0.0) {
            const double rec = 1.0 / tmp;
            cp[k - 1] = sup[k - 1] * rec;
            yp[k - 1] = (y - sub[k - 1] * yp[k - 2]) * rec;
          } else { cp[k - 1] = 0.0; yp[k - 1] = 0.0; }
        }
      }
      for (int k = Nr; k >= 1; k--)
        W3(g, i, j, k) = (k == Nr) ? yp[k - 1] : yp[k - 1] - cp[k - 1] * W3(g, i, j, k + 1);
    }
#undef W3
#undef KAP
  free(sub); free(sup); free(cp); free(yp);
}

/* IMPLDIFF (model/src/impldiff.F:24-245) with tracerId = 0 (deltaTX = deltaTMom; deepFac =
 * rhoFac = 1): the implicit vertical viscosity DYNAMICS applies to the CD scheme's D-grid
 * velocities (dynamics.F:614-634) on i0..i1 x j0..j1, in place on g -- its own recurrence
 * (bet, gam), not SOLVE_TRIDIAGONAL's: a(k) and c(k) vanish where recip_hFac of the level
 * above / below is 0 (impldiff.F:109-145), bet = 1 / gam = 0 where a pivot is 0 (:147-201). */
static void impldiff(const OModel *m, double *g, const double *rhFac, const double *kappa, int i0, int i1, int j0, int j1) {
  const int OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long n2 = m->n2;
  double *a = malloc(sizeof(double) * Nr), *c = malloc(sizeof(double) * Nr), *b = malloc(sizeof(double) * Nr);
  double *bet = malloc(sizeof(double) * Nr), *gam = malloc(sizeof(double) * Nr), *lt = malloc(sizeof(double) * Nr);
#define W3(a_, i, j, k) (a_)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx + (long)((k) - 1) * n2]
#define KAP(i, j, k) kappa[(long)((k) - 1) * n2 + ((i) + OLx - 1) + (long)((j) + OLy - 1) * nx]
  for (int j = j0; j <= j1; j++)
    for (int i = i0; i <= i1; i++) {
      a[0] = 0.0;
      for (int k = 2; k <= Nr; k++) {
        a[k - 1] = -(m->deltaTMom * W3(rhFac, i, j, k) * m->recip_drF[k - 1] * KAP(i, j, k) * m->recip_drC[k - 1]);
        if (W3(rhFac, i, j, k - 1) == 0.0) a[k - 1] = 0.0;
      }
      for (int k = 1; k <= Nr - 1; k++) {
        c[k - 1] = -(m->deltaTMom * W3(rhFac, i, j, k) * m->recip_drF[k - 1] * KAP(i, j, k + 1) * m->recip_drC[k]);
        if (W3(rhFac, i, j, k + 1) == 0.0) c[k - 1] = 0.0;
      }
      c[Nr - 1] = 0.0;
      for (int k = 1; k <= Nr; k++) { b[k - 1] = 1.0 - (a[k - 1] + c[k - 1]); bet[k - 1] = 1.0; gam[k - 1] = 0.0; }
      if (Nr > 1) {
        if (b[0] != 0.0) bet[0] = 1.0 / b[0];
        for (int k = 2; k <= Nr; k++) {
          gam[k - 1] = c[k - 2] * bet[k - 2];
          if ((b[k - 1] - a[k - 1] * gam[k - 1]) != 0.0) bet[k - 1] = 1.0 / (b[k - 1] - a[k - 1] * gam[k - 1]);
        }
      }
      lt[0] = W3(g, i, j, 1) * bet[0];
      for (int k = 2; k <= Nr; k++) lt[k - 1] = bet[k - 1] * (W3(g, i, j, k) - a[k - 1] * lt[k - 2]);
      for (int k = Nr - 1; k >= 1; k--) lt[k - 1] = lt[k - 1] - gam[k] * lt[k];
      for (int k = 1; k <= Nr; k++) W3(g, i, j, k) = lt[k - 1];
    }
#undef W3
#undef KAP
  free(a); free(c); free(b); free(bet); free(gam); free(lt);
}

void oracle_dynamics(OModel *m) {
  check_supported(m);
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long n2 = m->n2;
  const int iMin = 0, iMax = sNx + 1, jMin = 0, jMax = sNy + 1; /* dynamics.F:191-192 */
  /* tiles in parallel (OpenMP; one thread = the sequential restatement): every tile's work
     reads and writes its own slabs only, each thread keeps its own scratch */
#pragma omp parallel if (m->nThreads > 1) num_threads(m->nThreads > 1 ? m->nThreads : 1)
  {
  double *fVerU[2], *fVerV[2];
  for (int q = 0; q < 2; q++) { fVerU[q] = calloc(n2, 8); fVerV[q] = calloc(n2, 8); }
  double *hFacZ = calloc(n2, 8), *r_hFacZ = calloc(n2, 8), *xA = calloc(n2, 8), *yA = calloc(n2, 8);
  double *uTrans = calloc(n2, 8), *vTrans = calloc(n2, 8), *rTransU = calloc(n2, 8), *rTransV = calloc(n2, 8);
  double *fZon = calloc(n2, 8), *fMer = calloc(n2, 8), *fVrUp = calloc(n2, 8), *fVrDw = calloc(n2, 8);
  double *uCf = calloc(n2, 8), *vCf = calloc(n2, 8), *vF = calloc(n2, 8), *cDrag = calloc(n2, 8);
  double *guDiss = calloc(n2, 8), *gvDiss = calloc(n2, 8), *guExt = calloc(n2, 8), *gvExt = calloc(n2, 8);
  double *gUtmp = calloc(n2, 8), *gVtmp = calloc(n2, 8), *ab = calloc(n2, 8);
  double *kappaRU = calloc(n2 * (Nr + 1), 8), *kappaRV = calloc(n2 * (Nr + 1), 8);
  double *phiHydF = calloc(n2, 8), *phiHydC = calloc(n2, 8), *dPhiHydX = calloc(n2, 8), *dPhiHydY = calloc(n2, 8);
  double *mT = calloc(n2, 8), *h0FacZ = calloc(n2, 8), *v4F = calloc(n2, 8), *d2Z = calloc(n2, 8), *d2M = calloc(n2, 8);
  double *alphaRho = calloc(n2, 8), *varLoc = calloc(n2, 8);
  double *dWtransC = calloc(n2, 8), *dWtransU = calloc(n2, 8), *dWtransV = calloc(n2, 8);
  const int rstar = m->nonlinFreeSurf > 0 && m->select_rStar > 0;
  const int biharm = m->viscA4D != 0.0 || m->viscA4Z != 0.0;   /* useBiharmonicVisc (set_parms.F:141) */
  const int qh3d = m->quasiHydrostatic && (m->select3dCoriScheme >= 1 || m->useNHMTerms);
  const int metricSphere = m->usingSphericalPolarGrid && m->selectMetricTerms >= 1;
  const double recip_rSphere = m->usingSphericalPolarGrid ? 1.0 / m->rSphere : 0.0; /* ini_parms.F:1334 */
  const double recip_rhoConst = 1.0 / m->rhoConst;

  /* MOM_FLUXFORM factors (mom_fluxform.F:236-277) */
  const double uDudxFac = m->afFacMom, vDudyFac = m->afFacMom, rVelDudrFac = m->afFacMom;
  const double AhDudxFac = m->vfFacMom, AhDudyFac = m->vfFacMom;
  const double ArDudrFac = m->implicitViscosity ? 0.0 : m->vfFacMom;
  const double fuFac = m->cfFacMom, fvFac = m->cfFacMom;
  const int bottomDragTerms = m->no_slip_bottom; /* selectBotDragQuadr=-1, bottomDragLinear=0 */

#pragma omp for schedule(dynamic, 1)
  for (int t = 0; t < m->nTiles; t++) {
    double *gU = m->gU + t * m->n3, *gV = m->gV + t * m->n3;
    double *uVel = m->uVel + t * m->n3, *vVel = m->vVel + t * m->n3, *wVel = m->wVel + t * m->n3;
    double *guNm1 = m->guNm1 + t * m->n3, *gvNm1 = m->gvNm1 + t * m->n3;
    const double *hFacW = m->hFacW + t * m->n3, *hFacS = m->hFacS + t * m->n3, *hFacC = m->hFacC + t * m->n3;
    const double *maskW = m->maskW + t * m->n3, *maskS = m->maskS + t * m->n3, *maskC = m->maskC + t * m->n3;
    const double *rhFacW = m->recip_hFacW + t * m->n3, *rhFacS = m->recip_hFacS + t * m->n3;
    const double *dxG = m->dxG + t * n2, *dyG = m->dyG + t * n2, *dxF = m->dxF + t * n2, *dyF = m->dyF + t * n2;
    const double *dxV = m->dxV + t * n2, *dyU = m->dyU + t * n2, *rA = m->rA + t * n2, *rAw = m->rAw + t * n2;
    const double *rAs = m->rAs + t * n2;
    const double *recip_dxF = m->recip_dxF + t * n2, *recip_dyF = m->recip_dyF + t * n2;
    const double *recip_dxV = m->recip_dxV + t * n2, *recip_dyU = m->recip_dyU + t * n2;
    const double *recip_rAw = m->recip_rAw + t * n2, *recip_rAs = m->recip_rAs + t * n2;
    const double *fCori = m->fCori + t * n2;
    const double *tanPhiAtU = m->tanPhiAtU + t * n2, *tanPhiAtV = m->tanPhiAtV + t * n2;
    const double *recip_dxC = m->recip_dxC + t * n2, *recip_dyC = m->recip_dyC + t * n2;
    const double *rhoInSitu = m->rhoInSitu + t * m->n3;
    const double *sfU = m->surfaceForcingU + t * n2, *sfV = m->surfaceForcingV + t * n2;
    const double *h0FacW = m->h0FacW + t * m->n3, *h0FacS = m->h0FacS + t * m->n3, *h0FacC = m->h0FacC + t * m->n3;
    const double *rStarFacC = m->rStarFacC + t * n2, *rStarExpW = m->rStarExpW + t * n2, *rStarExpS = m->rStarExpS + t * n2;
    const double *rStarDhCDt = m->rStarDhCDt + t * n2, *rStarDhWDt = m->rStarDhWDt + t * n2, *rStarDhSDt = m->rStarDhSDt + t * n2;
    const double *etaH = m->etaH + t * n2, *recip_Rcol = m->recip_Rcol + t * n2, *Ro_surf = m->Ro_surf + t * n2;
    const double *R_low = m->R_low + t * n2, *fCoriCos = m->fCoriCos + t * n2;
    double *totPhiHyd = m->totPhiHyd + t * m->n3;
#define W3(a, i, j, k) (a)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx + (long)((k) - 1) * n2]

    /* dynamics.F:288-343: zero gU/gV and the ping-pong flux buffers */
    for (long p = 0; p < m->n3; p++) { gU[p] = 0.0; gV[p] = 0.0; }
    for (long p = 0; p < n2; p++) { fVerU[0][p] = fVerU[1][p] = fVerV[0][p] = fVerV[1][p] = 0.0; }
    /* CALC_VISCOSITY (model/src/calc_viscosity.F): kappaRU = viscArNr(k) */
    for (long p = 0; p < n2 * (Nr + 1); p++) { kappaRU[p] = m->viscAr; kappaRV[p] = m->viscAr; }
    /* CALC_PHI_HYD (calc_phi_hyd.F:167-172): phiHydF = 0 at k = 1 */
    for (long p = 0; p < n2; p++) phiHydF[p] = 0.0;

    for (int k = 1; k <= Nr; k++) {
      const int kUp = 1 + (k + 1) % 2, kDown = 1 + k % 2; /* dynamics.F:425-426 */
      double *fVerUkm = fVerU[kUp - 1], *fVerVkm = fVerV[kUp - 1];
      double *fVerUkp = fVerU[kDown - 1], *fVerVkp = fVerV[kDown - 1];
      /* CALC_PHI_HYD (calc_phi_hyd.F:175-327), OCEANIC, integr_GeoPot = 2, uniformFreeSurfLev,
       * alphaRho = rhoInSitu from DO_OCEANIC_PHYS; gravFac* = 1; iMin..iMax = 0..sNx+1 */
      {
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) L(alphaRho, i, j) = W3(rhoInSitu, i, j, k);
        if (qh3d) {
          /* MOM_QUASIHYDROSTATIC (pkg/mom_common/mom_quasihydrostatic.F:76-147), z-coords:
           * scalingFactor = rhoConst*gravitySign/gravity; angleCosC = 1, angleSinC = 0 */
          const double scalingFactor = m->rhoConst * m->gravitySign * (1.0 / m->gravity);
          for (int j = jMin; j <= jMax; j++)
            for (int i = iMin; i <= iMax; i++) {
              double gW = 0.0;
              if (m->select3dCoriScheme >= 1)
                gW = L(fCoriCos, i, j) * (1.0 * 0.5 * (W3(uVel, i, j, k) + W3(uVel, i + 1, j, k)) -
                                          0.0 * 0.5 * (W3(vVel, i, j, k) + W3(vVel, i, j + 1, k)));
              if (m->useNHMTerms)
                gW = gW + ((W3(uVel, i, j, k) * W3(uVel, i, j, k) + W3(uVel, i + 1, j, k) * W3(uVel, i + 1, j, k)) +
                           (W3(vVel, i, j, k) * W3(vVel, i, j, k) + W3(vVel, i, j + 1, k) * W3(vVel, i, j + 1, k))) *
                              0.5 * recip_rSphere;
              L(alphaRho, i, j) = L(alphaRho, i, j) + scalingFactor * gW;
            }
        }
        double dRlocM = 0.5 * m->drC[k - 1];
        if (k == 1) dRlocM = m->rF[0] - m->rC[0];
        double dRlocP = (k == Nr) ? (m->rC[k - 1] - m->rF[k]) : 0.5 * m->drC[k];
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            double a = L(alphaRho, i, j);
            L(phiHydC, i, j) = L(phiHydF, i, j) + dRlocM * m->gravity * a * recip_rhoConst;
            L(phiHydF, i, j) = L(phiHydC, i, j) + dRlocP * m->gravity * a * recip_rhoConst;
          }
        /* CALC_GRAD_PHI_HYD (calc_grad_phi_hyd.F:92-171), phi0surf = 0 */
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++)
            L(varLoc, i, j) = (rstar && m->select_rStar >= 2 && m->nonlinFreeSurf >= 4)
                                  ? L(phiHydC, i, j) * L(rStarFacC, i, j) + 0.0
                                  : L(phiHydC, i, j) + 0.0;
        for (long p = 0; p < n2; p++) dPhiHydX[p] = dPhiHydY[p] = 0.0;
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin + 1; i <= iMax; i++)
            L(dPhiHydX, i, j) = L(recip_dxC, i, j) * (L(varLoc, i, j) - L(varLoc, i - 1, j));
        for (int j = jMin + 1; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++)
            L(dPhiHydY, i, j) = L(recip_dyC, i, j) * (L(varLoc, i, j) - L(varLoc, i, j - 1));
        if (rstar && m->select_rStar >= 2) {
          /* calc_grad_phi_hyd.F:173-214: fluidIsWater, z-coords, generalForm = F */
          const double factorP = m->gravity * recip_rhoConst * 0.5;
          for (int j = jMin; j <= jMax; j++)
            for (int i = iMin; i <= iMax; i++)
              L(varLoc, i, j) = L(etaH, i, j) * (1.0 + m->rC[k - 1] * L(recip_Rcol, i, j));
          for (int j = jMin; j <= jMax; j++)
            for (int i = iMin + 1; i <= iMax; i++)
              L(dPhiHydX, i, j) = L(dPhiHydX, i, j) + factorP * (L(alphaRho, i - 1, j) + L(alphaRho, i, j)) *
                                                          (L(varLoc, i, j) - L(varLoc, i - 1, j)) * L(recip_dxC, i, j);
          for (int j = jMin + 1; j <= jMax; j++)
            for (int i = iMin; i <= iMax; i++)
              L(dPhiHydY, i, j) = L(dPhiHydY, i, j) + factorP * (L(alphaRho, i, j - 1) + L(alphaRho, i, j)) *
                                                          (L(varLoc, i, j) - L(varLoc, i, j - 1)) * L(recip_dyC, i, j);
        }
        /* DIAGS_PHI_HYD (diags_phi_hyd.F:60-120): totPhiHyd, phi0surf = 0 */
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            if (rstar && m->nonlinFreeSurf >= 4) {
              const double dPhiRef = (L(Ro_surf, i, j) - m->rC[k - 1]) * m->gravity;
              W3(totPhiHyd, i, j, k) = L(phiHydC, i, j) * L(rStarFacC, i, j) +
                                       fmax(dPhiRef, 0.0) * (L(rStarFacC, i, j) - 1.0) + 0.0;
            } else {
              W3(totPhiHyd, i, j, k) = L(phiHydC, i, j) + L(m->Bo_surf + t * n2, i, j) * L(m->etaN + t * n2, i, j) + 0.0;
            }
          }
      }
      for (long p = 0; p < n2; p++) {
        guDiss[p] = gvDiss[p] = 0.0; fZon[p] = fMer[p] = fVrUp[p] = fVrDw[p] = 0.0;
        uCf[p] = vCf[p] = vF[p] = 0.0; rTransU[p] = rTransV[p] = 0.0;
      }
      /* MOM_CALC_HFACZ (pkg/mom_common/mom_calc_hfacz.F:158-371, hZoption=0) */
      for (int i = 1 - OLx; i <= sNx + OLx; i++) L(hFacZ, i, 1 - OLy) = 0.0;
      for (int j = 2 - OLy; j <= sNy + OLy; j++) L(hFacZ, 1 - OLx, j) = 0.0;
      for (int j = 2 - OLy; j <= sNy + OLy; j++)
        for (int i = 2 - OLx; i <= sNx + OLx; i++) {
          double h = fmin(W3(hFacW, i, j, k), W3(hFacW, i, j - 1, k));
          h = fmin(W3(hFacS, i, j, k), h);
          h = fmin(W3(hFacS, i - 1, j, k), h);
          L(hFacZ, i, j) = h;
        }
      for (int j = 1 - OLy; j <= sNy + OLy; j++)
        for (int i = 1 - OLx; i <= sNx + OLx; i++)
          L(r_hFacZ, i, j) = (L(hFacZ, i, j) == 0.0) ? 0.0 : 1.0 / L(hFacZ, i, j);
      /* h0FacZ (mom_fluxform.F:290-307) */
      for (long p = 0; p < n2; p++) h0FacZ[p] = hFacZ[p];
      if (m->momViscosity && m->no_slip_sides && m->nonlinFreeSurf > 0)
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 2 - OLx; i <= sNx + OLx; i++)
            L(h0FacZ, i, j) = fmin(fmin(W3(h0FacW, i, j, k), W3(h0FacW, i, j - 1, k)),
                                   fmin(W3(h0FacS, i, j, k), W3(h0FacS, i - 1, j, k)));
      if (m->vectorInvariantMomentum) {
        /* MOM_VECINV (dynamics.F:517-530) replaces MOM_FLUXFORM; the ping-pong buffers carry
         * the vertical viscous fluxes there */
        oracle_mom_vecinv(m, t, k, hFacZ, r_hFacZ, h0FacZ, kappaRU, kappaRV, fVerUkm, fVerVkm,
                          fVerUkp, fVerVkp, guDiss, gvDiss);
      } else {
      for (long p = 0; p < n2; p++) v4F[p] = 0.0;
      /* xA, yA, uTrans, vTrans (mom_fluxform.F:287-327) */
      for (int j = 1 - OLy; j <= sNy + OLy; j++)
        for (int i = 1 - OLx; i <= sNx + OLx; i++) {
          L(xA, i, j) = L(dyG, i, j) * m->drF[k - 1] * W3(hFacW, i, j, k);
          L(yA, i, j) = L(dxG, i, j) * m->drF[k - 1] * W3(hFacS, i, j, k);
          L(uTrans, i, j) = W3(uVel, i, j, k) * L(xA, i, j);
          L(vTrans, i, j) = W3(vVel, i, j, k) * L(yA, i, j);
        }
      if (m->momAdvection && k == 1) {
        /* MOM_CALC_RTRANS(k=1) (mom_calc_rtrans.F:92-105), MOM_U/V_ADV_WU/WV(k=1) surface flux */
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 2 - OLx; i <= sNx + OLx; i++) {
            L(rTransU, i, j) = 0.5 * (W3(wVel, i - 1, j, 1) * L(rA, i - 1, j) + W3(wVel, i, j, 1) * L(rA, i, j));
            L(rTransV, i, j) = 0.5 * (W3(wVel, i, j - 1, 1) * L(rA, i, j - 1) + W3(wVel, i, j, 1) * L(rA, i, j));
          }
        if (rstar) {   /* mom_calc_rtrans.F:91-106 */
          for (int j = 1 - OLy; j <= sNy + OLy; j++)
            for (int i = 1 - OLx; i <= sNx + OLx; i++)
              L(dWtransC, i, j) = L(rStarDhCDt, i, j) * (L(Ro_surf, i, j) - L(R_low, i, j)) * L(rA, i, j);
          for (int j = 2 - OLy; j <= sNy + OLy; j++)
            for (int i = 2 - OLx; i <= sNx + OLx; i++) {
              L(dWtransU, i, j) = 0.5 * (L(dWtransC, i - 1, j) + L(dWtransC, i, j));
              L(dWtransV, i, j) = 0.5 * (L(dWtransC, i, j - 1) + L(dWtransC, i, j));
            }
        }
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 2 - OLx; i <= sNx + OLx; i++) {
            L(fVerUkm, i, j) = L(rTransU, i, j) * W3(uVel, i, j, 1); /* mom_u_adv_wu.F:65-72 */
            L(fVerVkm, i, j) = L(rTransV, i, j) * W3(vVel, i, j, 1);
          }
      }
      if (m->momAdvection) {
        /* MOM_CALC_RTRANS(k+1) */
        if (k + 1 > Nr) {
          for (int j = 2 - OLy; j <= sNy + OLy; j++)
            for (int i = 2 - OLx; i <= sNx + OLx; i++) L(rTransU, i, j) = L(rTransV, i, j) = 0.0;
        } else {
          for (int j = 2 - OLy; j <= sNy + OLy; j++)
            for (int i = 2 - OLx; i <= sNx + OLx; i++) {
              L(rTransU, i, j) = 0.5 * (W3(wVel, i - 1, j, k + 1) * L(rA, i - 1, j) + W3(wVel, i, j, k + 1) * L(rA, i, j));
              L(rTransV, i, j) = 0.5 * (W3(wVel, i, j - 1, k + 1) * L(rA, i, j - 1) + W3(wVel, i, j, k + 1) * L(rA, i, j));
            }
          if (rstar) {   /* mom_calc_rtrans.F:107-137, kk = k+1 <= Nr */
            const int kk = k + 1;
            for (int j = 1 - OLy; j <= sNy + OLy; j++)
              for (int i = 1 - OLx; i <= sNx + OLx; i++)
                L(dWtransC, i, j) = L(dWtransC, i, j) - L(rStarDhCDt, i, j) * m->drF[kk - 2] * W3(h0FacC, i, j, kk - 1) * L(rA, i, j);
            for (int j = 2 - OLy; j <= sNy + OLy; j++)
              for (int i = 2 - OLx; i <= sNx + OLx; i++) {
                L(dWtransU, i, j) = L(dWtransU, i, j) - L(rStarDhWDt, i, j) * m->drF[kk - 2] * W3(h0FacW, i, j, kk - 1) * L(rAw, i, j);
                L(dWtransV, i, j) = L(dWtransV, i, j) - L(rStarDhSDt, i, j) * m->drF[kk - 2] * W3(h0FacS, i, j, kk - 1) * L(rAs, i, j);
              }
            for (int j = 2 - OLy; j <= sNy + OLy; j++)
              for (int i = 2 - OLx; i <= sNx + OLx; i++) {
                L(rTransU, i, j) = L(rTransU, i, j) - L(dWtransU, i, j) + (L(dWtransC, i - 1, j) + L(dWtransC, i, j)) * 0.5;
                L(rTransV, i, j) = L(rTransV, i, j) - L(dWtransV, i, j) + (L(dWtransC, i, j - 1) + L(dWtransC, i, j)) * 0.5;
              }
          }
        }
      }
      /* ================= U component ================= */
      if (m->momAdvection) {
        /* MOM_U_ADV_UU (mom_u_adv_uu.F:46-57) */
        for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
          for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
            L(fZon, i, j) = 0.25 * (L(uTrans, i, j) + L(uTrans, i + 1, j)) * (W3(uVel, i, j, k) + W3(uVel, i + 1, j, k));
        /* MOM_U_ADV_VU (mom_u_adv_vu.F:46-61) */
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 2 - OLx; i <= sNx + OLx; i++)
            L(fMer, i, j) = 0.25 * (L(vTrans, i, j) + L(vTrans, i - 1, j)) * (W3(uVel, i, j, k) + W3(uVel, i, j - 1, k));
        /* MOM_U_ADV_WU(k+1) (mom_u_adv_wu.F:56-105), select_rStar=0 branch */
        if (k + 1 > Nr) {
          for (int j = 1 - OLy; j <= sNy + OLy; j++)
            for (int i = 1 - OLx; i <= sNx + OLx; i++) L(fVerUkp, i, j) = 0.0;
        } else {
          const int kk = k + 1;
          for (int j = 2 - OLy; j <= sNy + OLy; j++)
            for (int i = 2 - OLx; i <= sNx + OLx; i++) {
              double f = L(rTransU, i, j) * (0.5 * (W3(uVel, i, j, kk) + W3(uVel, i, j, kk - 1)));
              if (m->select_rStar == 0) f = f + 0.25 * (W3(wVel, i, j, kk) * L(rA, i, j) * (W3(maskC, i, j, kk) - W3(maskC, i, j, kk - 1)) +
                              W3(wVel, i - 1, j, kk) * L(rA, i - 1, j) * (W3(maskC, i - 1, j, kk) - W3(maskC, i - 1, j, kk - 1))) *
                          W3(uVel, i, j, kk);
              L(fVerUkp, i, j) = f;
            }
        }
        /* gU (mom_fluxform.F:502-517) */
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++)
            W3(gU, i, j, k) = -W3(rhFacW, i, j, k) * m->recip_drF[k - 1] * L(recip_rAw, i, j) *
                              ((L(fZon, i, j) - L(fZon, i - 1, j)) * uDudxFac +
                               (L(fMer, i, j + 1) - L(fMer, i, j)) * vDudyFac +
                               (L(fVerUkp, i, j) - L(fVerUkm, i, j)) * m->rkSign * rVelDudrFac);
        if (rstar)   /* mom_fluxform.F:527-548 */
          for (int j = jMin; j <= jMax; j++)
            for (int i = iMin; i <= iMax; i++)
              W3(gU, i, j, k) = W3(gU, i, j, k) - (L(rStarExpW, i, j) - 1.0) / m->deltaTFreeSurf * W3(uVel, i, j, k);
      } else {
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) W3(gU, i, j, k) = 0.0;
      }
      if (m->momViscosity) {
        if (biharm) {
          /* MOM_U_DEL2U (pkg/mom_fluxform/mom_u_del2u.F:59-117), cosFac = 1, no OBCS */
          for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
              L(d2Z, i, j) = m->drF[k - 1] * W3(hFacC, i, j, k) * L(dyF, i, j) * L(recip_dxF, i, j) *
                             (W3(uVel, i + 1, j, k) - W3(uVel, i, j, k)) * 1.0;
          for (int j = 2 - OLy; j <= sNy + OLy; j++)
            for (int i = 2 - OLx; i <= sNx + OLx - 1; i++)
              L(d2M, i, j) = m->drF[k - 1] * L(hFacZ, i, j) * L(dxV, i, j) * L(recip_dyU, i, j) *
                             (W3(uVel, i, j, k) - W3(uVel, i, j - 1, k));
          for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 2 - OLx; i <= sNx + OLx - 1; i++)
              L(v4F, i, j) = m->recip_drF[k - 1] * W3(rhFacW, i, j, k) * L(recip_rAw, i, j) *
                             (L(d2Z, i, j) - L(d2Z, i - 1, j) + L(d2M, i, j + 1) - L(d2M, i, j)) * W3(maskW, i, j, k);
          if (m->no_slip_sides)
            for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
              for (int i = 2 - OLx; i <= sNx + OLx - 1; i++) {
                const double hS = W3(h0FacW, i, j, k) - L(h0FacZ, i, j);
                const double hN = W3(h0FacW, i, j, k) - L(h0FacZ, i, j + 1);
                L(v4F, i, j) = L(v4F, i, j) - W3(rhFacW, i, j, k) * L(recip_rAw, i, j) *
                                                  (hS * L(dxV, i, j) * L(recip_dyU, i, j) +
                                                   hN * L(dxV, i, j + 1) * L(recip_dyU, i, j + 1)) *
                                                  W3(uVel, i, j, k) * m->sideDragFactor * W3(maskW, i, j, k);
              }
        }
        /* MOM_U_XVISCFLUX (mom_u_xviscflux.F:51-68), cosFacU = sqCosFacU = 1 */
        for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
          for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
            L(fZon, i, j) = L(dyF, i, j) * m->drF[k - 1] * W3(hFacC, i, j, k) *
                            (-m->viscAhD * (W3(uVel, i + 1, j, k) - W3(uVel, i, j, k)) * 1.0 +
                             m->viscA4D * (L(v4F, i + 1, j) - L(v4F, i, j)) * 1.0) *
                            L(recip_dxF, i, j);
        /* MOM_U_YVISCFLUX (mom_u_yviscflux.F:52-73) */
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++)
            L(fMer, i, j) = L(dxV, i, j) * m->drF[k - 1] * L(hFacZ, i, j) *
                            (-m->viscAhZ * (W3(uVel, i, j, k) - W3(uVel, i, j - 1, k)) +
                             m->viscA4Z * (L(v4F, i, j) - L(v4F, i, j - 1))) *
                            L(recip_dyU, i, j);
        /* MOM_U_RVISCFLUX(k) and (k+1) (mom_u_rviscflux.F) */
        for (int q = 0; q < 2; q++) {
          int kk = k + q; double *fl = q ? fVrDw : fVrUp;
          if (kk <= 1 || kk > Nr) {
            for (long p = 0; p < n2; p++) fl[p] = 0.0;
          } else {
            for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
              for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
                L(fl, i, j) = -kappaRU[(long)(kk - 1) * n2 + (i + OLx - 1) + (long)(j + OLy - 1) * nx] * L(rAw, i, j) *
                              (W3(uVel, i, j, kk) - W3(uVel, i, j, kk - 1)) * m->rkSign * m->recip_drC[kk - 1] *
                              W3(maskW, i, j, kk) * W3(maskW, i, j, kk - 1);
          }
        }
        /* guDiss (mom_fluxform.F:602-618) */
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++)
            L(guDiss, i, j) = -W3(rhFacW, i, j, k) * m->recip_drF[k - 1] * L(recip_rAw, i, j) *
                              ((L(fZon, i, j) - L(fZon, i - 1, j)) * AhDudxFac +
                               (L(fMer, i, j + 1) - L(fMer, i, j)) * AhDudyFac +
                               (L(fVrDw, i, j) - L(fVrUp, i, j)) * m->rkSign * ArDudrFac);
        if (m->no_slip_sides) {
          /* MOM_U_SIDEDRAG (pkg/mom_common/mom_u_sidedrag.F:100-145), variable-viscosity form */
          for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 2 - OLx; i <= sNx + OLx - 1; i++) {
              /* NONLIN_FRSURF: h0FacW - h0FacZ (h0Fac = hFac for a linear free surface) */
              double hS = W3(h0FacW, i, j, k) - L(h0FacZ, i, j);
              double hN = W3(h0FacW, i, j, k) - L(h0FacZ, i, j + 1);
              L(vF, i, j) = -W3(rhFacW, i, j, k) * m->recip_drF[k - 1] * L(recip_rAw, i, j) *
                            (hS * L(dxV, i, j) * L(recip_dyU, i, j) * (m->viscAhZ * W3(uVel, i, j, k) - m->viscA4Z * L(v4F, i, j)) +
                             hN * L(dxV, i, j + 1) * L(recip_dyU, i, j + 1) * (m->viscAhZ * W3(uVel, i, j, k) - m->viscA4Z * L(v4F, i, j))) *
                            m->drF[k - 1] * m->sideDragFactor;
            }
          for (int j = jMin; j <= jMax; j++)
            for (int i = iMin; i <= iMax; i++) L(guDiss, i, j) = L(guDiss, i, j) + L(vF, i, j);
        }
        if (bottomDragTerms) {
          /* MOM_U_BOTDRAG_COEFF (pkg/mom_common/mom_u_botdrag_coeff.F), z-coords, no quadratic drag */
          const int kBottom = Nr, kDn = (k + 1 < Nr) ? k + 1 : Nr, kLowF = k + 1;
          const double recDrC = (k == kBottom) ? m->recip_drF[k - 1] : m->recip_drC[kLowF - 1];
          const double viscFac = m->no_slip_bottom ? 2.0 : 0.0;
          for (int j = 1 - OLy; j <= sNy + OLy; j++)
            for (int i = 2 - OLx; i <= sNx + OLx; i++) L(cDrag, i, j) = 0.0 * 1.0;
          for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 2 - OLx; i <= sNx + OLx - 1; i++)
              L(cDrag, i, j) = L(cDrag, i, j) + kappaRU[(long)(kLowF - 1) * n2 + (i + OLx - 1) + (long)(j + OLy - 1) * nx] * recDrC * viscFac;
          for (int j = 1 - OLy; j <= sNy + OLy; j++)
            for (int i = 2 - OLx; i <= sNx + OLx; i++)
              L(cDrag, i, j) = (k == kBottom) ? L(cDrag, i, j) * W3(maskW, i, j, k)
                                              : L(cDrag, i, j) * W3(maskW, i, j, k) * (1.0 - W3(maskW, i, j, kDn));
          for (int j = jMin; j <= jMax; j++)
            for (int i = iMin; i <= iMax; i++)
              L(guDiss, i, j) = L(guDiss, i, j) - L(cDrag, i, j) * W3(uVel, i, j, k) * W3(rhFacW, i, j, k) * m->recip_drF[k - 1];
        }
      }
      if (m->useNHMTerms) {
        /* MOM_U_METRIC_NH (pkg/mom_common/mom_u_metric_nh.F:56-68), rVel2wUnit = 1, mtNHFacU = 1 */
        const int kp1 = k + 1 < Nr ? k + 1 : Nr;
        const double ov = (k == Nr) ? 0.0 : 1.0;
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++)
            W3(gU, i, j, k) = W3(gU, i, j, k) +
                1.0 * (W3(uVel, i, j, k) * recip_rSphere * 0.25 *
                       ((W3(wVel, i - 1, j, kp1) + W3(wVel, i, j, kp1)) * ov + (W3(wVel, i - 1, j, k) + W3(wVel, i, j, k))) *
                       m->gravitySign);
      }
      if (metricSphere) {
        /* MOM_U_METRIC_SPHERE (pkg/mom_fluxform/mom_u_metric_sphere.F), mom_fluxform.F:714-721 */
        for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
          for (int i = 2 - OLx; i <= sNx + OLx; i++)
            L(mT, i, j) = W3(uVel, i, j, k) * recip_rSphere * 0.25 *
                          (W3(vVel, i, j, k) + W3(vVel, i - 1, j, k) + W3(vVel, i, j + 1, k) + W3(vVel, i - 1, j + 1, k)) *
                          L(tanPhiAtU, i, j);
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) W3(gU, i, j, k) = W3(gU, i, j, k) + m->mtFacMom * L(mT, i, j);
      }
      /* ================= V component ================= */
      if (m->momAdvection) {
        /* MOM_V_ADV_UV (mom_v_adv_uv.F:45-60) */
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 2 - OLx; i <= sNx + OLx; i++)
            L(fZon, i, j) = 0.25 * (L(uTrans, i, j) + L(uTrans, i, j - 1)) * (W3(vVel, i, j, k) + W3(vVel, i - 1, j, k));
        /* MOM_V_ADV_VV (mom_v_adv_vv.F:46-57) */
        for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
          for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
            L(fMer, i, j) = 0.25 * (L(vTrans, i, j) + L(vTrans, i, j + 1)) * (W3(vVel, i, j, k) + W3(vVel, i, j + 1, k));
        /* MOM_V_ADV_WV(k+1) */
        if (k + 1 > Nr) {
          for (int j = 1 - OLy; j <= sNy + OLy; j++)
            for (int i = 1 - OLx; i <= sNx + OLx; i++) L(fVerVkp, i, j) = 0.0;
        } else {
          const int kk = k + 1;
          for (int j = 2 - OLy; j <= sNy + OLy; j++)
            for (int i = 2 - OLx; i <= sNx + OLx; i++) {
              double f = L(rTransV, i, j) * (0.5 * (W3(vVel, i, j, kk) + W3(vVel, i, j, kk - 1)));
              if (m->select_rStar == 0) f = f + 0.25 * (W3(wVel, i, j, kk) * L(rA, i, j) * (W3(maskC, i, j, kk) - W3(maskC, i, j, kk - 1)) +
                              W3(wVel, i, j - 1, kk) * L(rA, i, j - 1) * (W3(maskC, i, j - 1, kk) - W3(maskC, i, j - 1, kk - 1))) *
                          W3(vVel, i, j, kk);
              L(fVerVkp, i, j) = f;
            }
        }
        /* gV (mom_fluxform.F:762-777) */
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++)
            W3(gV, i, j, k) = -W3(rhFacS, i, j, k) * m->recip_drF[k - 1] * L(recip_rAs, i, j) *
                              ((L(fZon, i + 1, j) - L(fZon, i, j)) * uDudxFac +
                               (L(fMer, i, j) - L(fMer, i, j - 1)) * vDudyFac +
                               (L(fVerVkp, i, j) - L(fVerVkm, i, j)) * m->rkSign * rVelDudrFac);
        if (rstar)   /* mom_fluxform.F:787-808 */
          for (int j = jMin; j <= jMax; j++)
            for (int i = iMin; i <= iMax; i++)
              W3(gV, i, j, k) = W3(gV, i, j, k) - (L(rStarExpS, i, j) - 1.0) / m->deltaTFreeSurf * W3(vVel, i, j, k);
      } else {
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) W3(gV, i, j, k) = 0.0;
      }
      if (m->momViscosity) {
        if (biharm) {
          /* MOM_V_DEL2V (pkg/mom_fluxform/mom_v_del2v.F:59-117) */
          for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 2 - OLx; i <= sNx + OLx; i++)
              L(d2Z, i, j) = m->drF[k - 1] * L(hFacZ, i, j) * L(dyU, i, j) * L(recip_dxV, i, j) *
                             (W3(vVel, i, j, k) - W3(vVel, i - 1, j, k)) * 1.0;
          for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 2 - OLx; i <= sNx + OLx - 1; i++)
              L(d2M, i, j) = m->drF[k - 1] * W3(hFacC, i, j, k) * L(dxF, i, j) * L(recip_dyF, i, j) *
                             (W3(vVel, i, j + 1, k) - W3(vVel, i, j, k));
          for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 2 - OLx; i <= sNx + OLx - 1; i++)
              L(v4F, i, j) = m->recip_drF[k - 1] * W3(rhFacS, i, j, k) * L(recip_rAs, i, j) *
                             (L(d2Z, i + 1, j) - L(d2Z, i, j) + L(d2M, i, j) - L(d2M, i, j - 1)) * W3(maskS, i, j, k);
          if (m->no_slip_sides)
            for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
              for (int i = 2 - OLx; i <= sNx + OLx - 1; i++) {
                const double hW = W3(h0FacS, i, j, k) - L(h0FacZ, i, j);
                const double hE = W3(h0FacS, i, j, k) - L(h0FacZ, i + 1, j);
                L(v4F, i, j) = L(v4F, i, j) - W3(rhFacS, i, j, k) * L(recip_rAs, i, j) *
                                                  (hW * L(dyU, i, j) * L(recip_dxV, i, j) +
                                                   hE * L(dyU, i + 1, j) * L(recip_dxV, i + 1, j)) *
                                                  W3(vVel, i, j, k) * m->sideDragFactor * W3(maskS, i, j, k);
              }
        }
        /* MOM_V_XVISCFLUX (mom_v_xviscflux.F:52-69) */
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 2 - OLx; i <= sNx + OLx; i++)
            L(fZon, i, j) = L(dyU, i, j) * m->drF[k - 1] * L(hFacZ, i, j) *
                            (-m->viscAhZ * (W3(vVel, i, j, k) - W3(vVel, i - 1, j, k)) * 1.0 +
                             m->viscA4Z * (L(v4F, i, j) - L(v4F, i - 1, j)) * 1.0) *
                            L(recip_dxV, i, j);
        /* MOM_V_YVISCFLUX (mom_v_yviscflux.F:51-73) */
        for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
          for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
            L(fMer, i, j) = L(dxF, i, j) * m->drF[k - 1] * W3(hFacC, i, j, k) *
                            (-m->viscAhD * (W3(vVel, i, j + 1, k) - W3(vVel, i, j, k)) +
                             m->viscA4D * (L(v4F, i, j + 1) - L(v4F, i, j))) *
                            L(recip_dyF, i, j);
        for (int q = 0; q < 2; q++) {
          int kk = k + q; double *fl = q ? fVrDw : fVrUp;
          if (kk <= 1 || kk > Nr) {
            for (long p = 0; p < n2; p++) fl[p] = 0.0;
          } else {
            for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
              for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
                L(fl, i, j) = -kappaRV[(long)(kk - 1) * n2 + (i + OLx - 1) + (long)(j + OLy - 1) * nx] * L(rAs, i, j) *
                              (W3(vVel, i, j, kk) - W3(vVel, i, j, kk - 1)) * m->rkSign * m->recip_drC[kk - 1] *
                              W3(maskS, i, j, kk) * W3(maskS, i, j, kk - 1);
          }
        }
        /* gvDiss (mom_fluxform.F:861-877) */
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++)
            L(gvDiss, i, j) = -W3(rhFacS, i, j, k) * m->recip_drF[k - 1] * L(recip_rAs, i, j) *
                              ((L(fZon, i + 1, j) - L(fZon, i, j)) * AhDudxFac +
                               (L(fMer, i, j) - L(fMer, i, j - 1)) * AhDudyFac +
                               (L(fVrDw, i, j) - L(fVrUp, i, j)) * m->rkSign * ArDudrFac);
        if (m->no_slip_sides) {
          /* MOM_V_SIDEDRAG (pkg/mom_common/mom_v_sidedrag.F) */
          for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 2 - OLx; i <= sNx + OLx - 1; i++) {
              double hW = W3(h0FacS, i, j, k) - L(h0FacZ, i, j);
              double hE = W3(h0FacS, i, j, k) - L(h0FacZ, i + 1, j);
              L(vF, i, j) = -W3(rhFacS, i, j, k) * m->recip_drF[k - 1] * L(recip_rAs, i, j) *
                            (hW * L(dyU, i, j) * L(recip_dxV, i, j) * (m->viscAhZ * W3(vVel, i, j, k) - m->viscA4Z * L(v4F, i, j)) +
                             hE * L(dyU, i + 1, j) * L(recip_dxV, i + 1, j) * (m->viscAhZ * W3(vVel, i, j, k) - m->viscA4Z * L(v4F, i, j))) *
                            m->drF[k - 1] * m->sideDragFactor;
            }
          for (int j = jMin; j <= jMax; j++)
            for (int i = iMin; i <= iMax; i++) L(gvDiss, i, j) = L(gvDiss, i, j) + L(vF, i, j);
        }
        if (bottomDragTerms) {
          const int kBottom = Nr, kDn = (k + 1 < Nr) ? k + 1 : Nr, kLowF = k + 1;
          const double recDrC = (k == kBottom) ? m->recip_drF[k - 1] : m->recip_drC[kLowF - 1];
          const double viscFac = m->no_slip_bottom ? 2.0 : 0.0;
          for (int j = 2 - OLy; j <= sNy + OLy; j++)
            for (int i = 1 - OLx; i <= sNx + OLx; i++) L(cDrag, i, j) = 0.0 * 1.0;
          for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
            for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
              L(cDrag, i, j) = L(cDrag, i, j) + kappaRV[(long)(kLowF - 1) * n2 + (i + OLx - 1) + (long)(j + OLy - 1) * nx] * recDrC * viscFac;
          for (int j = 2 - OLy; j <= sNy + OLy; j++)
            for (int i = 1 - OLx; i <= sNx + OLx; i++)
              L(cDrag, i, j) = (k == kBottom) ? L(cDrag, i, j) * W3(maskS, i, j, k)
                                              : L(cDrag, i, j) * W3(maskS, i, j, k) * (1.0 - W3(maskS, i, j, kDn));
          for (int j = jMin; j <= jMax; j++)
            for (int i = iMin; i <= iMax; i++)
              L(gvDiss, i, j) = L(gvDiss, i, j) - L(cDrag, i, j) * W3(vVel, i, j, k) * W3(rhFacS, i, j, k) * m->recip_drF[k - 1];
        }
      }
      if (m->useNHMTerms) {
        /* MOM_V_METRIC_NH (pkg/mom_common/mom_v_metric_nh.F:56-68) */
        const int kp1 = k + 1 < Nr ? k + 1 : Nr;
        const double ov = (k == Nr) ? 0.0 : 1.0;
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++)
            W3(gV, i, j, k) = W3(gV, i, j, k) +
                1.0 * (W3(vVel, i, j, k) * recip_rSphere * 0.25 *
                       ((W3(wVel, i, j - 1, kp1) + W3(wVel, i, j, kp1)) * ov + (W3(wVel, i, j - 1, k) + W3(wVel, i, j, k))) *
                       m->gravitySign);
      }
      if (metricSphere) {
        /* MOM_V_METRIC_SPHERE (pkg/mom_fluxform/mom_v_metric_sphere.F), mom_fluxform.F:973-980 */
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx - 1; i++) {
            double ub = W3(uVel, i, j, k) + W3(uVel, i + 1, j, k) + W3(uVel, i, j - 1, k) + W3(uVel, i + 1, j - 1, k);
            L(mT, i, j) = -(recip_rSphere * 0.25 * ub * 0.25 * ub * L(tanPhiAtV, i, j));
          }
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) W3(gV, i, j, k) = W3(gV, i, j, k) + m->mtFacMom * L(mT, i, j);
      }
      /* Coriolis (mom_fluxform.F:995-1022; mom_u_coriolis.F, mom_v_coriolis.F) */
      if (m->useCoriolis && !m->useCDscheme) {   /* CD scheme: Coriolis in timestep.F */
        const int sc = m->selectCoriScheme;
        for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
          for (int i = 2 - OLx; i <= sNx + OLx; i++) {
            double c;
            if (sc >= 2)
              c = 0.5 * (L(fCori, i, j) * 0.5 * (W3(vVel, i, j, k) + W3(vVel, i, j + 1, k)) +
                         L(fCori, i - 1, j) * 0.5 * (W3(vVel, i - 1, j, k) + W3(vVel, i - 1, j + 1, k)));
            else
              c = 0.5 * (L(fCori, i, j) + L(fCori, i - 1, j)) *
                  0.25 * (W3(vVel, i, j, k) + W3(vVel, i, j + 1, k) + W3(vVel, i - 1, j, k) + W3(vVel, i - 1, j + 1, k));
            if (sc == 1 || sc == 3)
              c = c * 4.0 / fmax(1.0, W3(maskS, i, j, k) + W3(maskS, i, j + 1, k) + W3(maskS, i - 1, j, k) + W3(maskS, i - 1, j + 1, k));
            L(uCf, i, j) = c;
          }
        for (int j = 2 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx - 1; i++) {
            double c;
            if (sc >= 2)
              c = -0.5 * (L(fCori, i, j) * 0.5 * (W3(uVel, i, j, k) + W3(uVel, i + 1, j, k)) +
                          L(fCori, i, j - 1) * 0.5 * (W3(uVel, i, j - 1, k) + W3(uVel, i + 1, j - 1, k)));
            else
              c = -0.5 * (L(fCori, i, j) + L(fCori, i, j - 1)) *
                  0.25 * (W3(uVel, i, j, k) + W3(uVel, i + 1, j, k) + W3(uVel, i, j - 1, k) + W3(uVel, i + 1, j - 1, k));
            if (sc == 1 || sc == 3)
              c = c * 4.0 / fmax(1.0, W3(maskW, i, j, k) + W3(maskW, i + 1, j, k) + W3(maskW, i, j - 1, k) + W3(maskW, i + 1, j - 1, k));
            L(vCf, i, j) = c;
          }
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            W3(gU, i, j, k) = W3(gU, i, j, k) + fuFac * L(uCf, i, j);
            W3(gV, i, j, k) = W3(gV, i, j, k) + fvFac * L(vCf, i, j);
          }
      }
      if (m->select3dCoriScheme >= 1) {
        /* MOM_U_CORIOLIS_NH (pkg/mom_common/mom_u_coriolis_nh.F:60-76), angleCosC = 1, rVel2wUnit = 1;
         * MOM_V_CORIOLIS_NH only on curvilinear / rotated grids (mom_fluxform.F:1031-1040) */
        const int kp1 = k + 1 < Nr ? k + 1 : Nr;
        const double wMsk = (k == Nr) ? 0.0 : 1.0;
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            const double c = 0.5 * (L(fCoriCos, i, j) * 1.0 * 0.5 * (W3(wVel, i, j, k) + W3(wVel, i, j, kp1) * wMsk) +
                                    L(fCoriCos, i - 1, j) * 1.0 * 0.5 * (W3(wVel, i - 1, j, k) + W3(wVel, i - 1, j, kp1) * wMsk)) *
                             m->gravitySign;
            W3(gU, i, j, k) = W3(gU, i, j, k) + fuFac * c;
          }
      }
      /* masks (mom_fluxform.F:1044-1051) */
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) {
          W3(gU, i, j, k) = W3(gU, i, j, k) * W3(maskW, i, j, k);
          L(guDiss, i, j) = L(guDiss, i, j) * W3(maskW, i, j, k);
          W3(gV, i, j, k) = W3(gV, i, j, k) * W3(maskS, i, j, k);
          L(gvDiss, i, j) = L(gvDiss, i, j) * W3(maskS, i, j, k);
        }

      }   /* vectorInvariantMomentum */
      /* ======================== TIMESTEP (timestep.F) ======================== */
      for (long p = 0; p < n2; p++) guExt[p] = gvExt[p] = gUtmp[p] = gVtmp[p] = 0.0;
      if (m->momForcing) {
        /* APPLY_FORCING_U/V (model/src/apply_forcing.F:81-88), kSurface=1 */
        if (k == 1) {
          for (int j = 0; j <= sNy + 1; j++)
            for (int i = 1; i <= sNx + 1; i++)
              L(guExt, i, j) = L(guExt, i, j) + m->foFacMom * L(sfU, i, j) * m->recip_drF[k - 1] * W3(rhFacW, i, j, k);
          for (int j = 1; j <= sNy + 1; j++)
            for (int i = 0; i <= sNx + 1; i++)
              L(gvExt, i, j) = L(gvExt, i, j) + m->foFacMom * L(sfV, i, j) * m->recip_drF[k - 1] * W3(rhFacS, i, j, k);
        }
      }
      /* timestep.F:116-126: synchronous time step, gU -= phFac*dPhiHydX */
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) {
          W3(gU, i, j, k) = W3(gU, i, j, k) - m->pfFacMom * L(dPhiHydX, i, j);
          W3(gV, i, j, k) = W3(gV, i, j, k) - m->pfFacMom * L(dPhiHydY, i, j);
        }
      if (m->momViscosity && m->momDissip_In_AB)
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            W3(gU, i, j, k) = W3(gU, i, j, k) + L(guDiss, i, j);
            W3(gV, i, j, k) = W3(gV, i, j, k) + L(gvDiss, i, j);
          }
      if (m->momForcing && m->momForcingOutAB != 1)
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            W3(gU, i, j, k) = W3(gU, i, j, k) + L(guExt, i, j);
            W3(gV, i, j, k) = W3(gV, i, j, k) + L(gvExt, i, j);
          }
      /* ADAMS_BASHFORTH2 (adams_bashforth2.F:61-88), kArg = k */
      {
        const double abFac = (m->myIter == m->nIter0 && m->nIter0 == 0) ? 0.0 : 0.5 + m->abEps;
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) {
            double a = abFac * (W3(gU, i, j, k) - W3(guNm1, i, j, k));
            W3(guNm1, i, j, k) = W3(gU, i, j, k);
            W3(gU, i, j, k) = W3(gU, i, j, k) + a;
            a = abFac * (W3(gV, i, j, k) - W3(gvNm1, i, j, k));
            W3(gvNm1, i, j, k) = W3(gV, i, j, k);
            W3(gV, i, j, k) = W3(gV, i, j, k) + a;
          }
      }
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) { L(gUtmp, i, j) = W3(gU, i, j, k); L(gVtmp, i, j) = W3(gV, i, j, k); }
      if (m->momForcing && m->momForcingOutAB == 1)
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            L(gUtmp, i, j) = L(gUtmp, i, j) + L(guExt, i, j);
            L(gVtmp, i, j) = L(gVtmp, i, j) + L(gvExt, i, j);
          }
      if (m->momViscosity && !m->momDissip_In_AB)
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            L(gUtmp, i, j) = L(gUtmp, i, j) + L(guDiss, i, j);
            L(gVtmp, i, j) = L(gVtmp, i, j) + L(gvDiss, i, j);
          }
      if (m->useCDscheme) {
        /* CD_CODE_SCHEME (pkg/cd_code/cd_code_scheme.F:85-236), staggerTimeStep = F: phxFac = 0 */
        const int ci0 = 1 - OLx + 1, ci1 = sNx + OLx - 1, cj0 = 1 - OLy + 1, cj1 = sNy + OLy - 1;
        double *uVelD = m->uVelD + t * m->n3, *vVelD = m->vVelD + t * m->n3;
        double *uNM1 = m->uNM1 + t * m->n3, *vNM1 = m->vNM1 + t * m->n3;
        const double *etaNm1 = m->etaNm1 + t * n2, *etaN = m->etaN + t * n2, *Bo = m->Bo_surf + t * n2;
        const double *fC = m->fCori + t * n2, *rdxC = m->recip_dxC + t * n2, *rdyC = m->recip_dyC + t * n2;
        const double ab15 = m->myIter == 0 ? 1.0 : 1.5 + m->epsAB_CD;
        const double ab05 = m->myIter == 0 ? -0.0 : -0.5 - m->epsAB_CD;
        const double phxFac = 0.0, phyFac = 0.0;
        double *pf = fZon, *af = fMer, *vfl = vF;     /* scratch (free at this point) */
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++)
            L(pf, i, j) = L(Bo, i, j) * (ab15 * L(etaN, i, j) + ab05 * L(etaNm1, i, j));
        for (int j = 1 - OLy + 1; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++)
            L(af, i, j) = (L(gVtmp, i, j) - (L(rdyC, i, j) * (L(pf, i, j) - L(pf, i, j - 1)) +
                                              phyFac * L(dPhiHydY, i, j))) * W3(maskS, i, j, k);
        for (int j = cj0; j <= cj1; j++)
          for (int i = ci0; i <= ci1; i++)
            L(vfl, i, j) = ((L(af, i, j) + L(af, i - 1, j + 1)) + (L(af, i - 1, j) + L(af, i, j + 1))) * 0.25 *
                               W3(maskW, i, j, k) -
                           (L(fC, i, j) + L(fC, i - 1, j)) * 0.5 * (ab15 * W3(uVel, i, j, k) + ab05 * W3(uNM1, i, j, k));
        for (int j = cj0; j <= cj1; j++)
          for (int i = ci0; i <= ci1; i++) W3(vVelD, i, j, k) = W3(vVelD, i, j, k) + m->deltaTMom * L(vfl, i, j);
        for (int j = cj0; j <= cj1; j++)
          for (int i = ci0; i <= ci1; i++)
            W3(vVelD, i, j, k) =
                (m->rCD * W3(vVelD, i, j, k) +
                 (1.0 - m->rCD) *
                     (ab15 * ((W3(vVel, i, j, k) + W3(vVel, i - 1, j + 1, k)) + (W3(vVel, i - 1, j, k) + W3(vVel, i, j + 1, k))) * 0.25 +
                      ab05 * ((W3(vNM1, i, j, k) + W3(vNM1, i - 1, j + 1, k)) + (W3(vNM1, i - 1, j, k) + W3(vNM1, i, j + 1, k))) * 0.25)) *
                W3(maskW, i, j, k);
        for (int j = cj0; j <= cj1; j++)
          for (int i = ci0; i <= ci1; i++)
            L(uCf, i, j) = (L(fC, i, j) + L(fC, i - 1, j)) * 0.5 * W3(vVelD, i, j, k) * m->cfFacMom;   /* guCor */
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx + 1; i <= sNx + OLx; i++)
            L(af, i, j) = (L(gUtmp, i, j) - (L(rdxC, i, j) * (L(pf, i, j) - L(pf, i - 1, j)) +
                                              phxFac * L(dPhiHydX, i, j))) * W3(maskW, i, j, k);
        for (int j = cj0; j <= cj1; j++)
          for (int i = ci0; i <= ci1; i++)
            L(vfl, i, j) = ((L(af, i, j) + L(af, i + 1, j - 1)) + (L(af, i + 1, j) + L(af, i, j - 1))) * 0.25 *
                               W3(maskS, i, j, k) +
                           (L(fC, i, j) + L(fC, i, j - 1)) * 0.5 * (ab15 * W3(vVel, i, j, k) + ab05 * W3(vNM1, i, j, k));
        for (int j = cj0; j <= cj1; j++)
          for (int i = ci0; i <= ci1; i++) W3(uVelD, i, j, k) = W3(uVelD, i, j, k) + m->deltaTMom * L(vfl, i, j);
        for (int j = cj0; j <= cj1; j++)
          for (int i = ci0; i <= ci1; i++)
            W3(uVelD, i, j, k) =
                (m->rCD * W3(uVelD, i, j, k) +
                 (1.0 - m->rCD) *
                     (ab15 * ((W3(uVel, i, j, k) + W3(uVel, i + 1, j - 1, k)) + (W3(uVel, i, j - 1, k) + W3(uVel, i + 1, j, k))) * 0.25 +
                      ab05 * ((W3(uNM1, i, j, k) + W3(uNM1, i + 1, j - 1, k)) + (W3(uNM1, i, j - 1, k) + W3(uNM1, i + 1, j, k))) * 0.25)) *
                W3(maskS, i, j, k);
        for (int j = cj0; j <= cj1; j++)
          for (int i = ci0; i <= ci1; i++)
            L(vCf, i, j) = -(L(fC, i, j) + L(fC, i, j - 1)) * 0.5 * W3(uVelD, i, j, k) * m->cfFacMom;  /* gvCor */
        for (int j = 1 - OLy; j <= sNy + OLy; j++)
          for (int i = 1 - OLx; i <= sNx + OLx; i++) {
            W3(uNM1, i, j, k) = W3(uVel, i, j, k);
            W3(vNM1, i, j, k) = W3(vVel, i, j, k);
          }
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            L(gUtmp, i, j) = L(gUtmp, i, j) + L(uCf, i, j);
            L(gVtmp, i, j) = L(gVtmp, i, j) + L(vCf, i, j);
          }
      }
      if (rstar && m->nonlinFreeSurf > 1)   /* timestep.F:274-284 */
        for (int j = jMin; j <= jMax; j++)
          for (int i = iMin; i <= iMax; i++) {
            L(gUtmp, i, j) = L(gUtmp, i, j) / L(rStarExpW, i, j);
            L(gVtmp, i, j) = L(gVtmp, i, j) / L(rStarExpS, i, j);
          }
      /* u* = u + dt*(gUtmp + gUdPx)*maskW, gUdPx = 0 for implicSurfPress = 1 (timestep.F:373-388) */
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) {
          W3(gU, i, j, k) = W3(uVel, i, j, k) + m->deltaTMom * (L(gUtmp, i, j) + 0.0) * W3(maskW, i, j, k);
          W3(gV, i, j, k) = W3(vVel, i, j, k) + m->deltaTMom * (L(gVtmp, i, j) + 0.0) * W3(maskS, i, j, k);
        }
    }
#undef W3
    if (m->implicitViscosity && Nr > 1) {   /* dynamics.F:568-580 */
      mom_implicit_r(m, gU, maskW, rhFacW, kappaRU, 1, sNx + 1, 1, sNy);
      mom_implicit_r(m, gV, maskS, rhFacS, kappaRV, 1, sNx, 1, sNy + 1);
    }
    if (m->implicitViscosity && m->useCDscheme) {   /* dynamics.F:614-634: D-grid velocities */
      impldiff(m, m->vVelD + t * m->n3, rhFacW, kappaRU, iMin, iMax, jMin, jMax);
      impldiff(m, m->uVelD + t * m->n3, rhFacS, kappaRV, iMin, iMax, jMin, jMax);
    }
  }
  (void)ab;
  for (int q = 0; q < 2; q++) { free(fVerU[q]); free(fVerV[q]); }
  free(hFacZ); free(r_hFacZ); free(xA); free(yA); free(uTrans); free(vTrans); free(rTransU); free(rTransV);
  free(fZon); free(fMer); free(fVrUp); free(fVrDw); free(uCf); free(vCf); free(vF); free(cDrag);
  free(guDiss); free(gvDiss); free(guExt); free(gvExt); free(gUtmp); free(gVtmp); free(ab);
  free(kappaRU); free(kappaRV);
  free(phiHydF); free(phiHydC); free(dPhiHydX); free(dPhiHydY); free(mT);
  free(h0FacZ); free(v4F); free(d2Z); free(d2M); free(alphaRho); free(varLoc); free(dWtransC); free(dWtransU); free(dWtransV);
  }   /* omp parallel */
}
