/*
 * vecinv.c -- oracle restatement of MOM_VECINV (pkg/mom_vecinv/mom_vecinv.F:42-1064)
 * for one tile and level: vector-invariant momentum tendencies with the cubed-sphere
 * corner treatment of the relative vorticity.  TEST INFRASTRUCTURE (see oracle.h).
 *
 * Supported subset (anything else aborts): useAbsVorticity = F, highOrderVorticity =
 * upwindVorticity = F, useJamartMomAdv = F, selectVortScheme 0..3, selectCoriScheme
 * 0..3, selectKEscheme 0..3, harmonic constant viscosity (useVariableVisc = F,
 * useStrainTensionVisc = F), no biharmonic viscosity, explicit vertical viscosity,
 * momImplVertAdv = F, no 3-D Coriolis, no NH metric terms.  deepFac/rhoFac = 1.
 */
#include "oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define L(a, i, j) (a)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx]
#define W3(a, i, j, k) (a)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx + (long)((k) - 1) * n2]

void oracle_mom_vecinv(OModel *m, int t, int k, const double *hFacZ, const double *r_hFacZ,
                       const double *h0FacZ, const double *kappaRU, const double *kappaRV,
                       const double *fVerUkm, const double *fVerVkm, double *fVerUkp, double *fVerVkp,
                       double *guDiss, double *gvDiss) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long n2 = m->n2;
  const int iMin = 0, iMax = sNx + 1, jMin = 0, jMax = sNy + 1;
  if (m->viscA4D != 0.0 || m->viscA4Z != 0.0 || m->useNHMTerms ||
      m->select3dCoriScheme > 0 || m->useCDscheme) {
    fprintf(stderr, "oracle_mom_vecinv: option outside the restated subset\n");
    abort();
  }
  double *gU = m->gU + t * m->n3, *gV = m->gV + t * m->n3;
  const double *uVel = m->uVel + t * m->n3, *vVel = m->vVel + t * m->n3, *wVel = m->wVel + t * m->n3;
  const double *hFacW = m->hFacW + t * m->n3, *hFacS = m->hFacS + t * m->n3;
  const double *h0FacW = m->h0FacW + t * m->n3, *h0FacS = m->h0FacS + t * m->n3;
  const double *rhFacW = m->recip_hFacW + t * m->n3, *rhFacS = m->recip_hFacS + t * m->n3;
  const double *rhFacC = m->recip_hFacC + t * m->n3;
  const double *maskW = m->maskW + t * m->n3, *maskS = m->maskS + t * m->n3, *maskC = m->maskC + t * m->n3;
  const double *dxC = m->dxC + t * n2, *dyC = m->dyC + t * n2, *dxG = m->dxG + t * n2, *dyG = m->dyG + t * n2;
  const double *dxV = m->dxV + t * n2, *dyU = m->dyU + t * n2;
  const double *rA = m->rA + t * n2, *rAw = m->rAw + t * n2, *rAs = m->rAs + t * n2;
  const double *recip_rA = m->recip_rA + t * n2, *recip_rAw = m->recip_rAw + t * n2;
  const double *recip_rAs = m->recip_rAs + t * n2, *recip_rAz = m->recip_rAz + t * n2;
  const double *recip_dxC = m->recip_dxC + t * n2, *recip_dyC = m->recip_dyC + t * n2;
  const double *recip_dxG = m->recip_dxG + t * n2, *recip_dyG = m->recip_dyG + t * n2;
  const double *recip_dyU = m->recip_dyU + t * n2, *recip_dxV = m->recip_dxV + t * n2;
  const double *fCoriG = m->fCoriG + t * n2;
  (void)dxV; (void)dyU; (void)recip_dxV;

  double *uFld = calloc(n2, 8), *vFld = calloc(n2, 8), *KE = calloc(n2, 8), *vort3 = calloc(n2, 8);
  double *hDiv = calloc(n2, 8), *uCf = calloc(n2, 8), *vCf = calloc(n2, 8), *vF = calloc(n2, 8);
  double *vrF = calloc(n2, 8), *cDrag = calloc(n2, 8);
  for (long p = 0; p < n2; p++) { guDiss[p] = 0.0; gvDiss[p] = 0.0; }

  const double ArDudrFac = m->vfFacMom * 1.0, ArDvdrFac = m->vfFacMom * 1.0;
  const int bottomDragTerms = m->no_slip_bottom;   /* selectImplicitDrag = 0, no linear/quadratic drag */
  const int useHarmonicVisc = m->viscAhD != 0.0 || m->viscAhZ != 0.0;

  for (int j = 1 - OLy; j <= sNy + OLy; j++)
    for (int i = 1 - OLx; i <= sNx + OLx; i++) {
      L(uFld, i, j) = W3(uVel, i, j, k);
      L(vFld, i, j) = W3(vVel, i, j, k);
    }

  /* MOM_CALC_KE (pkg/mom_common/mom_calc_ke.F:66-150) */
  for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
    for (int i = 1 - OLx; i <= sNx + OLx - 1; i++) {
      const double u0 = L(uFld, i, j), u1 = L(uFld, i + 1, j), v0 = L(vFld, i, j), v1 = L(vFld, i, j + 1);
      switch (m->selectKEscheme) {
        case 0:
          L(KE, i, j) = 0.25 * ((u0 * u0 + u1 * u1) + (v0 * v0 + v1 * v1));
          break;
        case 1:
          L(KE, i, j) = 0.25 * ((u0 * u0 * L(rAw, i, j) + u1 * u1 * L(rAw, i + 1, j)) +
                                (v0 * v0 * L(rAs, i, j) + v1 * v1 * L(rAs, i, j + 1))) * L(recip_rA, i, j);
          break;
        case 2:
          L(KE, i, j) = 0.25 * ((u0 * u0 * W3(hFacW, i, j, k) + u1 * u1 * W3(hFacW, i + 1, j, k)) +
                                (v0 * v0 * W3(hFacS, i, j, k) + v1 * v1 * W3(hFacS, i, j + 1, k))) *
                        W3(rhFacC, i, j, k);
          break;
        case 3:
          L(KE, i, j) = 0.25 * ((u0 * u0 * W3(hFacW, i, j, k) * L(rAw, i, j) +
                                 u1 * u1 * W3(hFacW, i + 1, j, k) * L(rAw, i + 1, j)) +
                                (v0 * v0 * W3(hFacS, i, j, k) * L(rAs, i, j) +
                                 v1 * v1 * W3(hFacS, i, j + 1, k) * L(rAs, i, j + 1))) *
                        W3(rhFacC, i, j, k) * L(recip_rA, i, j);
          break;
        default:
          fprintf(stderr, "oracle_mom_vecinv: selectKEscheme %d\n", m->selectKEscheme); abort();
      }
    }

  /* MOM_CALC_RELVORT3 (pkg/mom_common/mom_calc_relvort3.F:72-233) */
  for (int j = 2 - OLy; j <= sNy + OLy; j++)
    for (int i = 2 - OLx; i <= sNx + OLx; i++)
      L(vort3, i, j) = L(recip_rAz, i, j) *
                       ((L(vFld, i, j) * L(dyC, i, j) - L(vFld, i - 1, j) * L(dyC, i - 1, j)) -
                        (L(uFld, i, j) * L(dxC, i, j) - L(uFld, i, j - 1) * L(dxC, i, j - 1)));
  if (m->useCubedSphereExchange) {
    const int face = m->tileFace[t], e = m->tileEdge[t];
    const int isN = e & 1, isS = e & 2, isE = e & 4, isW = e & 8;
#define U_(i, j) L(uFld, i, j) * L(dxC, i, j)
#define V_(i, j) L(vFld, i, j) * L(dyC, i, j)
    if (isW && isS) {
      const int i = 1, j = 1;
      L(vort3, i, j) = L(recip_rAz, i, j) * ((V_(i, j) - U_(i, j)) + U_(i, j - 1));
    }
    if (isE && isS) {
      const int i = sNx + 1, j = 1;
      if (face == 2)
        L(vort3, i, j) = L(recip_rAz, i, j) * ((-U_(i, j) - V_(i - 1, j)) + U_(i, j - 1));
      else if (face == 4)
        L(vort3, i, j) = L(recip_rAz, i, j) * ((-V_(i - 1, j) + U_(i, j - 1)) - U_(i, j));
      else
        L(vort3, i, j) = L(recip_rAz, i, j) * ((U_(i, j - 1) - U_(i, j)) - V_(i - 1, j));
    }
    if (isW && isN) {
      const int i = 1, j = sNy + 1;
      if (face == 1)
        L(vort3, i, j) = L(recip_rAz, i, j) * ((U_(i, j - 1) + V_(i, j)) - U_(i, j));
      else if (face == 3)
        L(vort3, i, j) = L(recip_rAz, i, j) * ((-U_(i, j) + U_(i, j - 1)) + V_(i, j));
      else
        L(vort3, i, j) = L(recip_rAz, i, j) * ((V_(i, j) - U_(i, j)) + U_(i, j - 1));
    }
    if (isE && isN) {
      const int i = sNx + 1, j = sNy + 1;
      if (face % 2 == 1)
        L(vort3, i, j) = L(recip_rAz, i, j) * ((-U_(i, j) - V_(i - 1, j)) + U_(i, j - 1));
      else
        L(vort3, i, j) = L(recip_rAz, i, j) * ((U_(i, j - 1) - U_(i, j)) - V_(i - 1, j));
    }
#undef U_
#undef V_
  }
  /* mom_vecinv.F:395-403: vort3 = 0 where hFacZ = 0 */
  for (int j = 1 - OLy; j <= sNy + OLy; j++)
    for (int i = 1 - OLx; i <= sNx + OLx; i++)
      if (L(hFacZ, i, j) == 0.0) L(vort3, i, j) = 0.0;

  if (m->momViscosity) {
    /* MOM_CALC_HDIV(hDivScheme = 2) (pkg/mom_common/mom_calc_hdiv.F:76-89) */
    for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
      for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
        L(hDiv, i, j) = ((L(uFld, i + 1, j) * L(dyG, i + 1, j) * W3(hFacW, i + 1, j, k) -
                          L(uFld, i, j) * L(dyG, i, j) * W3(hFacW, i, j, k)) +
                         (L(vFld, i, j + 1) * L(dxG, i, j + 1) * W3(hFacS, i, j + 1, k) -
                          L(vFld, i, j) * L(dxG, i, j) * W3(hFacS, i, j, k))) *
                        L(recip_rA, i, j) * W3(rhFacC, i, j, k);
    /* MOM_VI_HDISSIP (pkg/mom_vecinv/mom_vi_hdissip.F:105-131), constant viscosity, cosFac = 1 */
    for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
      for (int i = 2 - OLx; i <= sNx + OLx - 1; i++) {
        if (useHarmonicVisc) {
          const double Dim = L(hDiv, i, j - 1), Dij = L(hDiv, i, j), Dmj = L(hDiv, i - 1, j);
          const double Zip = L(hFacZ, i, j + 1) * L(vort3, i, j + 1), Zij = L(hFacZ, i, j) * L(vort3, i, j);
          const double Zpj = L(hFacZ, i + 1, j) * L(vort3, i + 1, j);
          const double uD2 = m->viscAhD * 1.0 * (Dij - Dmj) * L(recip_dxC, i, j) -
                             m->viscAhZ * W3(rhFacW, i, j, k) * (Zip - Zij) * L(recip_dyG, i, j);
          const double vD2 = m->viscAhZ * W3(rhFacS, i, j, k) * 1.0 * (Zpj - Zij) * L(recip_dxG, i, j) +
                             m->viscAhD * (Dij - Dim) * L(recip_dyC, i, j);
          L(guDiss, i, j) = uD2 * W3(maskW, i, j, k);
          L(gvDiss, i, j) = vD2 * W3(maskS, i, j, k);
        } else {
          L(guDiss, i, j) = 0.0;
          L(gvDiss, i, j) = 0.0;
        }
      }
    /* MOM_U_RVISCFLUX(k+1) (pkg/mom_common/mom_u_rviscflux.F) -> fVerUkp; mom_vecinv.F:444-463,
     * skipped with implicitViscosity (MOM_U_IMPLICIT_R solves it after the k loop) */
    if (!m->implicitViscosity) {
      const int kk = k + 1;
      for (long p = 0; p < n2; p++) vrF[p] = 0.0;
      if (kk > 1 && kk <= Nr)
        for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
          for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
            L(vrF, i, j) = -kappaRU[(long)(kk - 1) * n2 + (i + OLx - 1) + (long)(j + OLy - 1) * nx] * L(rAw, i, j) *
                           (W3(uVel, i, j, kk) - W3(uVel, i, j, kk - 1)) * m->rkSign * m->recip_drC[kk - 1] *
                           W3(maskW, i, j, kk) * W3(maskW, i, j, kk - 1);
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) L(fVerUkp, i, j) = ArDudrFac * L(vrF, i, j);
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++)
          L(guDiss, i, j) = L(guDiss, i, j) - W3(rhFacW, i, j, k) * m->recip_drF[k - 1] * L(recip_rAw, i, j) *
                                                  (L(fVerUkp, i, j) - L(fVerUkm, i, j)) * m->rkSign;
    }
    if (m->no_slip_sides) {
      /* MOM_U_SIDEDRAG (pkg/mom_common/mom_u_sidedrag.F:100-145), sideDragFactor > 0 form */
      for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
        for (int i = 2 - OLx; i <= sNx + OLx - 1; i++) {
          const double hS = W3(h0FacW, i, j, k) - L(h0FacZ, i, j);
          const double hN = W3(h0FacW, i, j, k) - L(h0FacZ, i, j + 1);
          L(vF, i, j) = -W3(rhFacW, i, j, k) * m->recip_drF[k - 1] * L(recip_rAw, i, j) *
                        (hS * L(dxV, i, j) * L(recip_dyU, i, j) * (m->viscAhZ * L(uFld, i, j) - m->viscA4Z * 0.0) +
                         hN * L(dxV, i, j + 1) * L(recip_dyU, i, j + 1) * (m->viscAhZ * L(uFld, i, j) - m->viscA4Z * 0.0)) *
                        m->drF[k - 1] * m->sideDragFactor;
        }
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) L(guDiss, i, j) = L(guDiss, i, j) + L(vF, i, j);
    }
    if (bottomDragTerms) {
      /* MOM_U_BOTDRAG_COEFF (pkg/mom_common/mom_u_botdrag_coeff.F), no quadratic drag */
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
          L(guDiss, i, j) = L(guDiss, i, j) + -L(cDrag, i, j) * L(uFld, i, j) * W3(rhFacW, i, j, k) * m->recip_drF[k - 1];
    }
    /* V: MOM_V_RVISCFLUX(k+1), MOM_V_SIDEDRAG, MOM_V_BOTDRAG_COEFF (mom_vecinv.F:556-575, 630-720);
     * the vertical viscous flux is skipped with implicitViscosity */
    if (!m->implicitViscosity) {
      const int kk = k + 1;
      for (long p = 0; p < n2; p++) vrF[p] = 0.0;
      if (kk > 1 && kk <= Nr)
        for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
          for (int i = 1 - OLx; i <= sNx + OLx - 1; i++)
            L(vrF, i, j) = -kappaRV[(long)(kk - 1) * n2 + (i + OLx - 1) + (long)(j + OLy - 1) * nx] * L(rAs, i, j) *
                           (W3(vVel, i, j, kk) - W3(vVel, i, j, kk - 1)) * m->rkSign * m->recip_drC[kk - 1] *
                           W3(maskS, i, j, kk) * W3(maskS, i, j, kk - 1);
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) L(fVerVkp, i, j) = ArDvdrFac * L(vrF, i, j);
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++)
          L(gvDiss, i, j) = L(gvDiss, i, j) - W3(rhFacS, i, j, k) * m->recip_drF[k - 1] * L(recip_rAs, i, j) *
                                                  (L(fVerVkp, i, j) - L(fVerVkm, i, j)) * m->rkSign;
    }
    if (m->no_slip_sides) {
      /* MOM_V_SIDEDRAG (pkg/mom_common/mom_v_sidedrag.F) */
      for (int j = 2 - OLy; j <= sNy + OLy - 1; j++)
        for (int i = 2 - OLx; i <= sNx + OLx - 1; i++) {
          const double hW = W3(h0FacS, i, j, k) - L(h0FacZ, i, j);
          const double hE = W3(h0FacS, i, j, k) - L(h0FacZ, i + 1, j);
          L(vF, i, j) = -W3(rhFacS, i, j, k) * m->recip_drF[k - 1] * L(recip_rAs, i, j) *
                        (hW * L(dyU, i, j) * L(recip_dxV, i, j) * (m->viscAhZ * L(vFld, i, j) - m->viscA4Z * 0.0) +
                         hE * L(dyU, i + 1, j) * L(recip_dxV, i + 1, j) * (m->viscAhZ * L(vFld, i, j) - m->viscA4Z * 0.0)) *
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
          L(gvDiss, i, j) = L(gvDiss, i, j) + -L(cDrag, i, j) * L(vFld, i, j) * W3(rhFacS, i, j, k) * m->recip_drF[k - 1];
    }
  }

  /* Coriolis: MOM_VI_CORIOLIS (pkg/mom_vecinv/mom_vi_coriolis.F:60-190) */
  if (m->useCoriolis) {
    for (long p = 0; p < n2; p++) { uCf[p] = 0.0; vCf[p] = 0.0; }
    const int cs = m->selectCoriScheme;
    const double epsil = 1.0e-9;
    for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
      for (int i = 2 - OLx; i <= sNx + OLx; i++) {
        double vBarXY, c;
#define VX(i_, j_) L(vFld, i_, j_) * L(dxG, i_, j_)
#define VXH(i_, j_) L(vFld, i_, j_) * L(dxG, i_, j_) * W3(hFacS, i_, j_, k)
        if (cs == 0) {
          vBarXY = 0.25 * ((VX(i, j) + VX(i - 1, j)) + (VX(i, j + 1) + VX(i - 1, j + 1)));
          c = 0.5 * (L(fCoriG, i, j) + L(fCoriG, i, j + 1)) * vBarXY * L(recip_dxC, i, j) * W3(maskW, i, j, k);
        } else if (cs == 1) {
          vBarXY = ((VXH(i, j) + VXH(i - 1, j)) + (VXH(i, j + 1) + VXH(i - 1, j + 1))) /
                   fmax(epsil, (W3(hFacS, i, j, k) + W3(hFacS, i - 1, j, k)) +
                                   (W3(hFacS, i, j + 1, k) + W3(hFacS, i - 1, j + 1, k)));
          c = 0.5 * (L(fCoriG, i, j) + L(fCoriG, i, j + 1)) * vBarXY * L(recip_dxC, i, j) * W3(maskW, i, j, k);
        } else if (cs == 2) {
          vBarXY = 0.25 * ((VXH(i, j) + VXH(i - 1, j)) + (VXH(i, j + 1) + VXH(i - 1, j + 1)));
          c = 0.5 * (L(fCoriG, i, j) + L(fCoriG, i, j + 1)) * vBarXY * L(recip_dxC, i, j) * W3(rhFacW, i, j, k);
        } else {
          const double vm = 0.5 * (VXH(i, j) + VXH(i - 1, j)), vp = 0.5 * (VXH(i, j + 1) + VXH(i - 1, j + 1));
          c = 0.5 * (vm * L(fCoriG, i, j) + vp * L(fCoriG, i, j + 1)) * L(recip_dxC, i, j) * W3(rhFacW, i, j, k);
        }
        L(uCf, i, j) = c;
      }
    for (int j = 2 - OLy; j <= sNy + OLy; j++)
      for (int i = 1 - OLx; i <= sNx + OLx - 1; i++) {
        double uBarXY, c;
#define UY(i_, j_) L(uFld, i_, j_) * L(dyG, i_, j_)
#define UYH(i_, j_) L(uFld, i_, j_) * L(dyG, i_, j_) * W3(hFacW, i_, j_, k)
        if (cs == 0) {
          uBarXY = 0.25 * ((UY(i, j) + UY(i, j - 1)) + (UY(i + 1, j) + UY(i + 1, j - 1)));
          c = -0.5 * (L(fCoriG, i, j) + L(fCoriG, i + 1, j)) * uBarXY * L(recip_dyC, i, j) * W3(maskS, i, j, k);
        } else if (cs == 1) {
          uBarXY = ((UYH(i, j) + UYH(i, j - 1)) + (UYH(i + 1, j) + UYH(i + 1, j - 1))) /
                   fmax(epsil, (W3(hFacW, i, j, k) + W3(hFacW, i, j - 1, k)) +
                                   (W3(hFacW, i + 1, j, k) + W3(hFacW, i + 1, j - 1, k)));
          c = -0.5 * (L(fCoriG, i, j) + L(fCoriG, i + 1, j)) * uBarXY * L(recip_dyC, i, j) * W3(maskS, i, j, k);
        } else if (cs == 2) {
          uBarXY = 0.25 * ((UYH(i, j) + UYH(i, j - 1)) + (UYH(i + 1, j) + UYH(i + 1, j - 1)));
          c = -0.5 * (L(fCoriG, i, j) + L(fCoriG, i + 1, j)) * uBarXY * L(recip_dyC, i, j) * W3(rhFacS, i, j, k);
        } else {
          const double um = 0.5 * (UYH(i, j) + UYH(i, j - 1)), up = 0.5 * (UYH(i + 1, j) + UYH(i + 1, j - 1));
          c = -0.5 * (um * L(fCoriG, i, j) + up * L(fCoriG, i + 1, j)) * L(recip_dyC, i, j) * W3(rhFacS, i, j, k);
        }
        L(vCf, i, j) = c;
      }
    for (int j = jMin; j <= jMax; j++)
      for (int i = iMin; i <= iMax; i++) {
        W3(gU, i, j, k) = L(uCf, i, j);
        W3(gV, i, j, k) = L(vCf, i, j);
      }
  } else {
    for (int j = jMin; j <= jMax; j++)
      for (int i = iMin; i <= iMax; i++) { W3(gU, i, j, k) = 0.0; W3(gV, i, j, k) = 0.0; }
  }

  if (m->momAdvection) {
    /* MOM_VI_U_CORIOLIS / MOM_VI_V_CORIOLIS with omega3 = vort3
     * (pkg/mom_vecinv/mom_vi_u_coriolis.F:70-190, mom_vi_v_coriolis.F) */
    const int vs = m->selectVortScheme;
    const double epsil = 1.0e-9, oneThird = 1.0 / 3.0;
    for (long p = 0; p < n2; p++) { uCf[p] = 0.0; vCf[p] = 0.0; }
#define OM(i_, j_) L(vort3, i_, j_)
#define RZ(i_, j_) L(r_hFacZ, i_, j_)
    for (int j = 1 - OLy; j <= sNy + OLy - 1; j++)
      for (int i = 2 - OLx; i <= sNx + OLx - (vs == 3 ? 1 : 0); i++) {
        double c;
        if (vs == 0) {
          const double vBarXY = 0.25 * ((VXH(i, j) + VXH(i - 1, j)) + (VXH(i, j + 1) + VXH(i - 1, j + 1)));
          const double v3 = 0.5 * (OM(i, j) * RZ(i, j) + OM(i, j + 1) * RZ(i, j + 1));
          c = v3 * vBarXY * L(recip_dxC, i, j) * W3(maskW, i, j, k);
        } else if (vs == 1) {
          const double vBarXY = 0.5 * ((VX(i, j) * L(hFacZ, i, j) + VX(i - 1, j) * L(hFacZ, i, j)) +
                                       (VX(i, j + 1) * L(hFacZ, i, j + 1) + VX(i - 1, j + 1) * L(hFacZ, i, j + 1))) /
                                fmax(epsil, L(hFacZ, i, j) + L(hFacZ, i, j + 1));
          const double v3 = 0.5 * (OM(i, j) + OM(i, j + 1));
          c = v3 * vBarXY * L(recip_dxC, i, j) * W3(maskW, i, j, k);
        } else if (vs == 2) {
          const double vm = 0.5 * (VXH(i, j) + VXH(i - 1, j)), vp = 0.5 * (VXH(i, j + 1) + VXH(i - 1, j + 1));
          const double v3 = (vm * RZ(i, j) * OM(i, j) + vp * RZ(i, j + 1) * OM(i, j + 1)) * 0.5;
          c = v3 * L(recip_dxC, i, j) * W3(maskW, i, j, k);
        } else {
          const double mj = (RZ(i, j) * OM(i, j) + (RZ(i, j + 1) * OM(i, j + 1) + RZ(i - 1, j) * OM(i - 1, j))) *
                            oneThird * VXH(i - 1, j);
          const double ij = (RZ(i, j) * OM(i, j) + (RZ(i, j + 1) * OM(i, j + 1) + RZ(i + 1, j) * OM(i + 1, j))) *
                            oneThird * VXH(i, j);
          const double mp = (RZ(i, j + 1) * OM(i, j + 1) + (RZ(i, j) * OM(i, j) + RZ(i - 1, j + 1) * OM(i - 1, j + 1))) *
                            oneThird * VXH(i - 1, j + 1);
          const double ip = (RZ(i, j + 1) * OM(i, j + 1) + (RZ(i, j) * OM(i, j) + RZ(i + 1, j + 1) * OM(i + 1, j + 1))) *
                            oneThird * VXH(i, j + 1);
          c = ((mj + ij) + (mp + ip)) * 0.25 * L(recip_dxC, i, j) * W3(maskW, i, j, k);
        }
        L(uCf, i, j) = c;
      }
    for (int j = jMin; j <= jMax; j++)
      for (int i = iMin; i <= iMax; i++) W3(gU, i, j, k) = W3(gU, i, j, k) + L(uCf, i, j);
    for (int j = 2 - OLy; j <= sNy + OLy - (vs == 3 ? 1 : 0); j++)
      for (int i = 1 - OLx; i <= sNx + OLx - 1; i++) {
        double c;
        if (vs == 0) {
          const double uBarXY = 0.25 * ((UYH(i, j) + UYH(i, j - 1)) + (UYH(i + 1, j) + UYH(i + 1, j - 1)));
          const double v3 = 0.5 * (OM(i, j) * RZ(i, j) + OM(i + 1, j) * RZ(i + 1, j));
          c = -v3 * uBarXY * L(recip_dyC, i, j) * W3(maskS, i, j, k);
        } else if (vs == 1) {
          const double uBarXY = 0.5 * ((UY(i, j) * L(hFacZ, i, j) + UY(i, j - 1) * L(hFacZ, i, j)) +
                                       (UY(i + 1, j) * L(hFacZ, i + 1, j) + UY(i + 1, j - 1) * L(hFacZ, i + 1, j))) /
                                fmax(epsil, L(hFacZ, i, j) + L(hFacZ, i + 1, j));
          const double v3 = 0.5 * (OM(i, j) + OM(i + 1, j));
          c = -v3 * uBarXY * L(recip_dyC, i, j) * W3(maskS, i, j, k);
        } else if (vs == 2) {
          const double um = 0.5 * (UYH(i, j) + UYH(i, j - 1)), up = 0.5 * (UYH(i + 1, j) + UYH(i + 1, j - 1));
          const double v3 = (um * RZ(i, j) * OM(i, j) + up * RZ(i + 1, j) * OM(i + 1, j)) * 0.5;
          c = -v3 * L(recip_dyC, i, j) * W3(maskS, i, j, k);
        } else {
          const double im = (RZ(i, j) * OM(i, j) + (RZ(i + 1, j) * OM(i + 1, j) + RZ(i, j - 1) * OM(i, j - 1))) *
                            oneThird * UYH(i, j - 1);
          const double ij = (RZ(i, j) * OM(i, j) + (RZ(i + 1, j) * OM(i + 1, j) + RZ(i, j + 1) * OM(i, j + 1))) *
                            oneThird * UYH(i, j);
          const double pm = (RZ(i + 1, j) * OM(i + 1, j) + (RZ(i, j) * OM(i, j) + RZ(i + 1, j - 1) * OM(i + 1, j - 1))) *
                            oneThird * UYH(i + 1, j - 1);
          const double pj = (RZ(i + 1, j) * OM(i + 1, j) + (RZ(i, j) * OM(i, j) + RZ(i + 1, j + 1) * OM(i + 1, j + 1))) *
                            oneThird * UYH(i + 1, j);
          c = -((im + ij) + (pm + pj)) * 0.25 * L(recip_dyC, i, j) * W3(maskS, i, j, k);
        }
        L(vCf, i, j) = c;
      }
    for (int j = jMin; j <= jMax; j++)
      for (int i = iMin; i <= iMax; i++) W3(gV, i, j, k) = W3(gV, i, j, k) + L(vCf, i, j);
#undef OM
#undef RZ

    /* MOM_VI_U_VERTSHEAR / MOM_VI_V_VERTSHEAR (mom_vi_u_vertshear.F:60-110), upwindShear */
    {
      const int Kp1 = k + 1 < Nr ? k + 1 : Nr, Km1 = k - 1 > 1 ? k - 1 : 1;
      const double mKp1 = (k == Nr) ? 0.0 : 1.0, mKm1 = (k == 1) ? 0.0 : 1.0;
      const int areaW = !(m->selectKEscheme == 1 || m->selectKEscheme == 3);
      for (int j = 1 - OLy; j <= sNy + OLy; j++)
        for (int i = 2 - OLx; i <= sNx + OLx; i++) {
          double wm, wp;
          if (areaW) {
            wm = 0.5 * (W3(wVel, i, j, k) * L(rA, i, j) * W3(maskC, i, j, Km1) +
                        W3(wVel, i - 1, j, k) * L(rA, i - 1, j) * W3(maskC, i - 1, j, Km1)) * mKm1 * L(recip_rAw, i, j);
            wp = 0.5 * (W3(wVel, i, j, Kp1) * L(rA, i, j) + W3(wVel, i - 1, j, Kp1) * L(rA, i - 1, j)) * mKp1 *
                 L(recip_rAw, i, j);
          } else {
            wm = 0.5 * (W3(wVel, i, j, k) * W3(maskC, i, j, Km1) + W3(wVel, i - 1, j, k) * W3(maskC, i - 1, j, Km1)) * mKm1;
            wp = 0.5 * (W3(wVel, i, j, Kp1) + W3(wVel, i - 1, j, Kp1)) * mKp1;
          }
          const double uZm = (W3(uVel, i, j, k) - mKm1 * W3(uVel, i, j, Km1)) * m->rkSign;
          const double uZp = (mKp1 * W3(uVel, i, j, Kp1) - W3(uVel, i, j, k)) * m->rkSign;
          if (m->upwindShear)
            L(uCf, i, j) = -0.5 * ((wp * uZp + wm * uZm) + (fabs(wp) * uZp - fabs(wm) * uZm)) *
                           W3(rhFacW, i, j, k) * m->recip_drF[k - 1];
          else
            L(uCf, i, j) = -0.5 * (wp * uZp + wm * uZm) * W3(rhFacW, i, j, k) * m->recip_drF[k - 1];
        }
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) W3(gU, i, j, k) = W3(gU, i, j, k) + L(uCf, i, j);
      for (int j = 2 - OLy; j <= sNy + OLy; j++)
        for (int i = 1 - OLx; i <= sNx + OLx; i++) {
          double wm, wp;
          if (areaW) {
            wm = 0.5 * (W3(wVel, i, j, k) * L(rA, i, j) * W3(maskC, i, j, Km1) +
                        W3(wVel, i, j - 1, k) * L(rA, i, j - 1) * W3(maskC, i, j - 1, Km1)) * mKm1 * L(recip_rAs, i, j);
            wp = 0.5 * (W3(wVel, i, j, Kp1) * L(rA, i, j) + W3(wVel, i, j - 1, Kp1) * L(rA, i, j - 1)) * mKp1 *
                 L(recip_rAs, i, j);
          } else {
            wm = 0.5 * (W3(wVel, i, j, k) * W3(maskC, i, j, Km1) + W3(wVel, i, j - 1, k) * W3(maskC, i, j - 1, Km1)) * mKm1;
            wp = 0.5 * (W3(wVel, i, j, Kp1) + W3(wVel, i, j - 1, Kp1)) * mKp1;
          }
          const double vZm = (W3(vVel, i, j, k) - mKm1 * W3(vVel, i, j, Km1)) * m->rkSign;
          const double vZp = (mKp1 * W3(vVel, i, j, Kp1) - W3(vVel, i, j, k)) * m->rkSign;
          if (m->upwindShear)
            L(vCf, i, j) = -0.5 * ((wp * vZp + wm * vZm) + (fabs(wp) * vZp - fabs(wm) * vZm)) *
                           W3(rhFacS, i, j, k) * m->recip_drF[k - 1];
          else
            L(vCf, i, j) = -0.5 * (wp * vZp + wm * vZm) * W3(rhFacS, i, j, k) * m->recip_drF[k - 1];
        }
      for (int j = jMin; j <= jMax; j++)
        for (int i = iMin; i <= iMax; i++) W3(gV, i, j, k) = W3(gV, i, j, k) + L(vCf, i, j);
    }

    /* MOM_VI_U_GRAD_KE / MOM_VI_V_GRAD_KE (mom_vi_u_grad_ke.F:49-55) */
    for (int j = 1 - OLy; j <= sNy + OLy; j++)
      for (int i = 2 - OLx; i <= sNx + OLx; i++)
        L(uCf, i, j) = -L(recip_dxC, i, j) * (L(KE, i, j) - L(KE, i - 1, j)) * W3(maskW, i, j, k);
    for (int j = jMin; j <= jMax; j++)
      for (int i = iMin; i <= iMax; i++) W3(gU, i, j, k) = W3(gU, i, j, k) + L(uCf, i, j);
    for (int j = 2 - OLy; j <= sNy + OLy; j++)
      for (int i = 1 - OLx; i <= sNx + OLx; i++)
        L(vCf, i, j) = -L(recip_dyC, i, j) * (L(KE, i, j) - L(KE, i, j - 1)) * W3(maskS, i, j, k);
    for (int j = jMin; j <= jMax; j++)
      for (int i = iMin; i <= iMax; i++) W3(gV, i, j, k) = W3(gV, i, j, k) + L(vCf, i, j);
  }
#undef VX
#undef VXH
#undef UY
#undef UYH

  /* mom_vecinv.F:1044-1051 */
  for (int j = jMin; j <= jMax; j++)
    for (int i = iMin; i <= iMax; i++) {
      W3(gU, i, j, k) = W3(gU, i, j, k) * W3(maskW, i, j, k);
      W3(gV, i, j, k) = W3(gV, i, j, k) * W3(maskS, i, j, k);
    }
  free(uFld); free(vFld); free(KE); free(vort3); free(hDiv); free(uCf); free(vCf); free(vF);
  free(vrF); free(cDrag);
}
