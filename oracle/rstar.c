/*
 * rstar.c -- oracle restatement of the non-linear free surface in the r*
 * coordinate (nonlinFreeSurf = 4, select_rStar = 2; global_ocean.90x40x15):
 *   CALC_R_STAR            model/src/calc_r_star.F:55-283
 *   UPDATE_R_STAR          model/src/update_r_star.F:48-131
 *   UPDATE_CG2D            model/src/update_cg2d.F:49-199
 *   INITIALISE_VARIA       model/src/initialise_varia.F:299-349 (r* sequence after a pickup)
 * TEST INFRASTRUCTURE (see oracle.h).
 */
#include "oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

/* CALC_R_STAR(etaH): rStarFac at t+1 from etaH, previous factors kept in
 * rStarFacNm1, expansion ratio rStarExp = Fac/Fac_old and rStarDh*Dt.
 * rStarAreaWeight = .TRUE. (flux-form momentum). */
void oracle_calc_r_star(OModel *m) {
  const int sNx = m->sNx, sNy = m->sNy, Nr = m->Nr;
  const long N2 = m->n2 * m->nTiles;
  const double *eta = m->etaH;
  int bad = 0;
  for (long p = 0; p < N2; p++) {                     /* calc_r_star.F:95-109 */
    m->rStarFacNm1C[p] = m->rStarFacC[p];
    m->rStarFacNm1S[p] = m->rStarFacS[p];
    m->rStarFacNm1W[p] = m->rStarFacW[p];
    m->rStarExpC[p] = m->rStarFacC[p];
    m->rStarExpW[p] = m->rStarFacW[p];
    m->rStarExpS[p] = m->rStarFacS[p];
  }
  for (int t = 0; t < m->nTiles; t++) {
    for (int j = 0; j <= sNy + 1; j++)                /* :111-122 */
      for (int i = 0; i <= sNx + 1; i++) {
        const long p = O2(m, i, j, t);
        if (m->kSurfC[p] <= Nr)
          m->rStarFacC[p] = (eta[p] + m->Ro_surf[p] - m->R_low[p]) * m->recip_Rcol[p];
        else
          m->rStarFacC[p] = 1.0;
      }
    for (int j = 1; j <= sNy; j++)                    /* :123-136 */
      for (int i = 1; i <= sNx + 1; i++) {
        const long p = O2(m, i, j, t), pw = O2(m, i - 1, j, t);
        if (m->kSurfW[p] <= Nr) {
          const double tmp = m->rSurfW[p] - m->rLowW[p];
          m->rStarFacW[p] = (0.5 * (eta[pw] * m->rA[pw] + eta[p] * m->rA[p]) * m->recip_rAw[p] + tmp) / tmp;
        } else {
          m->rStarFacW[p] = 1.0;
        }
      }
    for (int j = 1; j <= sNy + 1; j++)                /* :137-150 */
      for (int i = 1; i <= sNx; i++) {
        const long p = O2(m, i, j, t), ps = O2(m, i, j - 1, t);
        if (m->kSurfS[p] <= Nr) {
          const double tmp = m->rSurfS[p] - m->rLowS[p];
          m->rStarFacS[p] = (0.5 * (eta[ps] * m->rA[ps] + eta[p] * m->rA[p]) * m->recip_rAs[p] + tmp) / tmp;
        } else {
          m->rStarFacS[p] = 1.0;
        }
      }
    for (int j = 1; j <= sNy + 1; j++)                /* :192-211: hFacInf check */
      for (int i = 1; i <= sNx + 1; i++) {
        const long p = O2(m, i, j, t);
        if (m->rStarFacC[p] < m->hFacInf || m->rStarFacW[p] < m->hFacInf || m->rStarFacS[p] < m->hFacInf) bad++;
      }
  }
  if (bad) { fprintf(stderr, "STOP in CALC_R_STAR : too SMALL rStarFac[C,W,S] !\n"); abort(); }
  oracle_exch_xy(m, m->rStarFacC);                    /* :256-257 */
  oracle_exch_uv_xyz(m, m->rStarFacW, m->rStarFacS, 1, 0);   /* EXCH_UV_XY_RL(.FALSE.) */
  for (long p = 0; p < N2; p++) {                     /* :283-298 */
    m->rStarDhCDt[p] = (m->rStarFacC[p] - m->rStarExpC[p]) / m->deltaTFreeSurf;
    m->rStarDhWDt[p] = (m->rStarFacW[p] - m->rStarExpW[p]) / m->deltaTFreeSurf;
    m->rStarDhSDt[p] = (m->rStarFacS[p] - m->rStarExpS[p]) / m->deltaTFreeSurf;
    m->rStarExpC[p] = m->rStarFacC[p] / m->rStarExpC[p];
    m->rStarExpW[p] = m->rStarFacW[p] / m->rStarExpW[p];
    m->rStarExpS[p] = m->rStarFacS[p] / m->rStarExpS[p];
  }
}

/* UPDATE_R_STAR: hFac = h0Fac * rStarFac (useLatest) or * rStarFacNm1, and the
 * reciprocals where the mask is wet (USE_MASK_AND_NO_IF undefined). */
void oracle_update_r_star(OModel *m, int useLatest) {
  const double *fC = useLatest ? m->rStarFacC : m->rStarFacNm1C;
  const double *fW = useLatest ? m->rStarFacW : m->rStarFacNm1W;
  const double *fS = useLatest ? m->rStarFacS : m->rStarFacNm1S;
  for (int t = 0; t < m->nTiles; t++)
    for (int k = 1; k <= m->Nr; k++)
      for (long q = 0; q < m->n2; q++) {
        const long p = t * m->n3 + (long)(k - 1) * m->n2 + q, p2 = t * m->n2 + q;
        m->hFacC[p] = m->h0FacC[p] * fC[p2];
        m->hFacW[p] = m->h0FacW[p] * fW[p2];
        m->hFacS[p] = m->h0FacS[p] * fS[p2];
        if (m->maskC[p] != 0.0) m->recip_hFacC[p] = 1.0 / m->hFacC[p];
        if (m->maskW[p] != 0.0) m->recip_hFacW[p] = 1.0 / m->hFacW[p];
        if (m->maskS[p] != 0.0) m->recip_hFacS[p] = 1.0 / m->hFacS[p];
      }
}

/* UPDATE_CG2D: the 2-D operator from the current hFacW/S, cg2dNorm kept from
 * INI_CG2D; preconditioner refreshed (cg2dPreCondFreq = 1). */
void oracle_update_cg2d(OModel *m) {
  const int sNx = m->sNx, sNy = m->sNy, Nr = m->Nr;
  for (int t = 0; t < m->nTiles; t++) {
    for (long q = 0; q < m->n2; q++) { m->aW2d[t * m->n2 + q] = 0.0; m->aS2d[t * m->n2 + q] = 0.0; }
    for (int k = 1; k <= Nr; k++)
      for (int j = 1; j <= sNy + 1; j++)
        for (int i = 1; i <= sNx + 1; i++) {
          const long p = O2(m, i, j, t), p3 = O3(m, i, j, k, t);
          double faceArea = m->dyG[p] * m->drF[k - 1] * m->hFacW[p3];
          m->aW2d[p] = m->aW2d[p] + faceArea * m->recip_dxC[p];
          faceArea = m->dxG[p] * m->drF[k - 1] * m->hFacS[p3];
          m->aS2d[p] = m->aS2d[p] + faceArea * m->recip_dyC[p];
        }
    for (int j = 1; j <= sNy + 1; j++)
      for (int i = 1; i <= sNx + 1; i++) {
        const long p = O2(m, i, j, t);
        m->aW2d[p] = m->aW2d[p] * m->cg2dNorm * m->implicSurfPress * m->implicDiv2DFlow;
        m->aS2d[p] = m->aS2d[p] * m->cg2dNorm * m->implicSurfPress * m->implicDiv2DFlow;
      }
    for (int j = 1; j <= sNy; j++)
      for (int i = 1; i <= sNx; i++) {
        const long p = O2(m, i, j, t);
        m->aC2d[p] = -(m->aW2d[p] + m->aW2d[O2(m, i + 1, j, t)] + m->aS2d[p] + m->aS2d[O2(m, i, j + 1, t)] +
                       m->freeSurfFac * m->cg2dNorm * m->recip_Bo[p] * m->rA[p] / m->deltaTMom / m->deltaTFreeSurf);
      }
  }
  if (m->cg2dPreCondFreq == 0) return;
  oracle_exch_xy(m, m->aC2d);
  for (int t = 0; t < m->nTiles; t++)
    for (int j = 1; j <= sNy + 1; j++)
      for (int i = 1; i <= sNx + 1; i++) {
        const long p = O2(m, i, j, t);
        const double aC = m->aC2d[p], aCw = m->aC2d[O2(m, i - 1, j, t)], aCs = m->aC2d[O2(m, i, j - 1, t)];
        m->pC[p] = (aC == 0.0) ? 1.0 : 1.0 / aC;
        const double pWt = aC + aCw;
        if (pWt == 0.0) m->pW[p] = 0.0;
        else { const double d = m->cg2dpcOffDFac * pWt; m->pW[p] = -m->aW2d[p] / (d * d); }
        const double pSt = aC + aCs;
        if (pSt == 0.0) m->pS[p] = 0.0;
        else { const double d = m->cg2dpcOffDFac * pSt; m->pS[p] = -m->aS2d[p] / (d * d); }
      }
}

/* INITIALISE_VARIA after READ_PICKUP (initialise_varia.F:299-349):
 * CALC_R_STAR(etaH) -> UPDATE_R_STAR(.TRUE.) -> UPDATE_CG2D ->
 * INTEGR_CONTINUITY(myIter = nIter0) -> CALC_R_STAR(etaH). */
void oracle_ini_nlfs_pickup(OModel *m) {
  oracle_calc_r_star(m);
  oracle_update_r_star(m, 1);
  oracle_update_cg2d(m);
  oracle_integr_continuity_init(m);
  oracle_calc_r_star(m);
}
