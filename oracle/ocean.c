/*
 * ocean.c -- ocean physics of the lat-lon global set-ups (tutorial_global_oce_latlon,
 * global_ocean.90x40x15): periodic external forcing, surface forcing, freezing,
 * the Jackett & McDougall (1995) equation of state and the GM/Redi tensor.
 * TEST INFRASTRUCTURE (see oracle.h): never linked into the product.
 *
 * Restated from (reference file:line):
 *   EXTERNAL_FIELDS_LOAD   model/src/external_fields_load.F:56-330
 *   GET_PERIODIC_INTERVAL  eesupp/src/get_periodic_interval.F:60-120
 *   FREEZE_SURFACE         model/src/freeze_surface.F:40-69
 *   EXTERNAL_FORCING_SURF  model/src/external_forcing_surf.F:90-330 + forcing_surf_relax.F:75-100
 *   FIND_RHO_2D (JMD95Z)   model/src/find_rho.F:146-180, FIND_RHOP0 :274-409, FIND_BULKMOD :411-590,
 *                          coefficients model/src/ini_eos.F:113-160, PRESSURE_FOR_EOS
 *                          model/src/pressure_for_eos.F:88-96 (selectP_inEOS_Zc = 0: pRef4EOS(k),
 *                          set_ref_state.F:92-97)
 *   GMREDI_CALC_TENSOR     pkg/gmredi/gmredi_calc_tensor.F:231-700 (GM_NON_UNITY_DIAGONAL,
 *                          GM_EXTRA_DIAGONAL compiled; GM_ExtraDiag = F, skew-flux form, all
 *                          GM_isoFac/bolFac = 1), GMREDI_SLOPE_LIMIT gkw91 branch
 *                          pkg/gmredi/gmredi_slope_limit.F:280-370
 * deepFac/rhoFac/wUnit2rVel/z2rUnit factors are 1.0 for these z-coordinate Boussinesq
 * set-ups and are dropped (bit-exact).
 */
#include "oracle.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#define L(a, i, j) (a)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx]
#define W3(a, i, j, k) (a)[(long)((i) + OLx - 1) + (long)((j) + OLy - 1) * nx + (long)((k) - 1) * n2]

/* ------------------------------------------------------- external forcing */
static void get_periodic_interval(double cycleLength, double recSpacing, double deltaT, double currentTime,
                                  int *tRec0, int *tRec1, int *tRec2, double *wght1, double *wght2) {
  const int nbRec = (int)lround(cycleLength / recSpacing);
  /* cycleLength > 0 branch (get_periodic_interval.F:106-117); NINT rounds half away from 0 */
  double locTime = currentTime - recSpacing * 0.5 + cycleLength * (2 - lround(currentTime / cycleLength));
  double tmpTime = fmod(locTime, cycleLength);
  *tRec1 = 1 + (int)(tmpTime / recSpacing);
  *tRec2 = 1 + (*tRec1 % nbRec);
  *wght2 = (tmpTime - recSpacing * (*tRec1 - 1)) / recSpacing;
  *wght1 = 1.0 - *wght2;
  tmpTime = fmod(locTime - deltaT, cycleLength);
  *tRec0 = 1 + (int)(tmpTime / recSpacing);
}

void oracle_fields_load(OModel *m) {
  if (!m->periodicExternalForcing) return;
  int iP, i0, i1;
  double bW, aW;
  get_periodic_interval(m->externForcingCycle, m->externForcingPeriod, m->deltaTClock, m->myTime, &iP, &i0, &i1,
                        &bW, &aW);
  const long N2 = m->n2 * m->nTiles;
  const double *r0[6] = {m->forcSST, m->forcSSS, m->forcTaux, m->forcTauy, m->forcQnet, m->forcEmPmR};
  double *dst[6] = {m->SST, m->SSS, m->fu, m->fv, m->Qnet, m->EmPmR};
  for (int f = 0; f < 6; f++) {
    const double *a = r0[f] + (long)(i0 - 1) * N2, *b = r0[f] + (long)(i1 - 1) * N2;
    for (long p = 0; p < N2; p++) dst[f][p] = bW * a[p] + aW * b[p];
  }
}

void oracle_freeze_surface(OModel *m) {
  const double Tfreezing = -1.9;
  for (int t = 0; t < m->nTiles; t++)
    for (long p = 0; p < m->n2; p++) {
      double *th = m->theta + t * m->n3 + p;   /* k = 1 */
      if (*th < Tfreezing) *th = Tfreezing;
    }
}

/* Full halo range iMin..iMax = 1-OLx..sNx+OLx (do_oceanic_phys.F:555-558), ks = 1 */
void oracle_external_forcing_surf(OModel *m) {
  const long N2 = m->n2 * m->nTiles;
  const double recip_Cp = 1.0 / m->HeatCapacity_Cp, mass2rUnit = 1.0 / m->rhoConst;
  const double UNSET_RL = 123456.7;
  for (int t = 0; t < m->nTiles; t++)
    for (long p = 0; p < m->n2; p++) {
      const long q = t * m->n2 + p, q3 = t * m->n3 + p;
      /* FORCING_SURF_RELAX */
      double sfT = -(m->lambdaThetaClimRelax[q] * (m->theta[q3] - m->SST[q]) * m->drF[0] * m->hFacC[q3]);
      double sfS = -(m->lambdaSaltClimRelax[q] * (m->salt[q3] - m->SSS[q]) * m->drF[0] * m->hFacC[q3]);
      m->surfaceForcingU[q] = m->fu[q] * mass2rUnit;
      m->surfaceForcingV[q] = m->fv[q] * mass2rUnit;
      sfT = sfT - m->Qnet[q] * recip_Cp * mass2rUnit;
      sfS = sfS - m->saltFlux[q] * mass2rUnit;
      if (m->nonlinFreeSurf > 0 && m->useRealFreshWaterFlux) {
        /* external_forcing_surf.F:253-277: PmEpR changes the column height */
        if (m->temp_EvPrRn != UNSET_RL) sfT = sfT + m->PmEpR[q] * (m->temp_EvPrRn - m->theta[q3]) * mass2rUnit;
        if (m->salt_EvPrRn != UNSET_RL) sfS = sfS + m->PmEpR[q] * (m->salt_EvPrRn - m->salt[q3]) * mass2rUnit;
      } else {
        /* the convertFW2Salt branch (:278-310) */
        if (m->convertFW2Salt == -1.0) {
          if (m->temp_EvPrRn != UNSET_RL)
            sfT = sfT + m->EmPmR[q] * (m->theta[q3] - m->temp_EvPrRn) * mass2rUnit;
          if (m->salt_EvPrRn != UNSET_RL)
            sfS = sfS + m->EmPmR[q] * (m->salt[q3] - m->salt_EvPrRn) * mass2rUnit;
        } else {
          if (m->temp_EvPrRn != UNSET_RL)
            sfT = sfT + m->EmPmR[q] * (m->tRef[0] - m->temp_EvPrRn) * mass2rUnit;
          if (m->salt_EvPrRn != UNSET_RL)
            sfS = sfS + m->EmPmR[q] * (m->convertFW2Salt - m->salt_EvPrRn) * mass2rUnit;
        }
      }
      m->surfaceForcingT[q] = sfT;
      m->surfaceForcingS[q] = sfS;
    }
  (void)N2;
}

/* ------------------------------------------------------------ JMD95 EOS */
static const double eosJMDCFw[6] = {999.842594, 6.793952e-02, -9.095290e-03, 1.001685e-04, -1.120083e-06,
                                    6.536332e-09};
static const double eosJMDCSw[9] = {8.24493e-01, -4.0899e-03, 7.6438e-05, -8.2467e-07, 5.3875e-09,
                                    -5.72466e-03, 1.0227e-04, -1.6546e-06, 4.8314e-04};
static const double eosJMDCKFw[5] = {1.965933e+04, 1.444304e+02, -1.706103e+00, 9.648704e-03, -4.190253e-05};
static const double eosJMDCKSw[7] = {5.284855e+01, -3.101089e-01, 6.283263e-03, -5.084188e-05, 3.886640e-01,
                                     9.085835e-03, -4.619924e-04};
static const double eosJMDCKP[14] = {3.186519e+00, 2.212276e-02, -2.984642e-04, 1.956415e-06, 6.704388e-03,
                                     -1.847318e-04, 2.059331e-07, 1.480266e-04, 2.102898e-04, -1.202016e-05,
                                     1.394680e-07, -2.040237e-06, 6.128773e-08, 6.207323e-10};
static const double SItoBar = 1.0e-05;

static double find_rhop0(double t, double s) {
  const double t2 = t * t, t3 = t2 * t, t4 = t3 * t;
  double s3o2;
  if (s > 0.0) s3o2 = s * sqrt(s);
  else { s = 0.0; s3o2 = 0.0; }
  const double rfresh = eosJMDCFw[0] + eosJMDCFw[1] * t + eosJMDCFw[2] * t2 + eosJMDCFw[3] * t3 +
                        eosJMDCFw[4] * t4 + eosJMDCFw[5] * t4 * t;
  const double rsalt = s * (eosJMDCSw[0] + eosJMDCSw[1] * t + eosJMDCSw[2] * t2 + eosJMDCSw[3] * t3 +
                            eosJMDCSw[4] * t4) +
                       s3o2 * (eosJMDCSw[5] + eosJMDCSw[6] * t + eosJMDCSw[7] * t2) + eosJMDCSw[8] * s * s;
  return rfresh + rsalt;
}

static double find_bulkmod(double locPres, double t, double s) {
  const double t2 = t * t, t3 = t2 * t, t4 = t3 * t;
  double s3o2;
  if (s > 0.0) s3o2 = s * sqrt(s);
  else { s = 0.0; s3o2 = 0.0; }
  const double p = locPres * SItoBar, p2 = p * p;
  const double bMfresh = eosJMDCKFw[0] + eosJMDCKFw[1] * t + eosJMDCKFw[2] * t2 + eosJMDCKFw[3] * t3 +
                         eosJMDCKFw[4] * t4;
  const double bMsalt = s * (eosJMDCKSw[0] + eosJMDCKSw[1] * t + eosJMDCKSw[2] * t2 + eosJMDCKSw[3] * t3) +
                        s3o2 * (eosJMDCKSw[4] + eosJMDCKSw[5] * t + eosJMDCKSw[6] * t2);
  const double bMpres = p * (eosJMDCKP[0] + eosJMDCKP[1] * t + eosJMDCKP[2] * t2 + eosJMDCKP[3] * t3) +
                        p * s * (eosJMDCKP[4] + eosJMDCKP[5] * t + eosJMDCKP[6] * t2) + p * s3o2 * eosJMDCKP[7] +
                        p2 * (eosJMDCKP[8] + eosJMDCKP[9] * t + eosJMDCKP[10] * t2) +
                        p2 * s * (eosJMDCKP[11] + eosJMDCKP[12] * t + eosJMDCKP[13] * t2);
  return bMfresh + bMsalt + bMpres;
}

/* PRESSURE_FOR_EOS (pressure_for_eos.F:51-105), z-coordinates, dpRef = 0:
 * selectP_inEOS_Zc = 2 (JMD95P default): rhoConst*(totPhiHyd + phiRef(2k));
 * 0/1: pRef4EOS(k).  p3 = flat 3-D offset of the point (level kRef). */
double oracle_pressure_for_eos(const OModel *m, int kRef, long p3) {
  if (m->selectP_inEOS_Zc == 2) return m->rhoConst * (m->totPhiHyd[p3] + m->phiRef[2 * kRef - 1]) + 0.0;
  return m->pRef4EOS[kRef - 1] + 0.0;
}

double oracle_find_rho(const OModel *m, int kRef, double t, double s) {
  return oracle_find_rho_p(m, kRef, t, s, m->pRef4EOS[kRef - 1] + 0.0);
}

double oracle_find_rho_p(const OModel *m, int kRef, double t, double s, double locPres) {
  if (m->eosType == 0) {
    /* LINEAR (find_rho.F:84-99) */
    const double dRho = m->rhoNil - m->rhoConst;
    return m->rhoNil * (m->sBeta * (s - m->sRef[kRef - 1]) - m->tAlpha * (t - m->tRef[kRef - 1])) + dRho;
  }
  /* JMD95Z / JMD95P (find_rho.F:136-160): same formula, locPres from PRESSURE_FOR_EOS */
  const double rhoP0 = find_rhop0(t, s);
  const double bulkMod = find_bulkmod(locPres, t, s);
  return rhoP0 / (1.0 - locPres * SItoBar / bulkMod) - m->rhoConst;
}

/* ------------------------------------------------------------- GM / Redi */
static void slope_limit_gkw91(const OModel *m, const double *dSigmaDx, const double *dSigmaDy, double *dSigmaDr,
                              double *SlopeX, double *SlopeY, double *SlopeSqr, double *taperFct) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, nx = m->nx;
  const double GM_bigSlope = 1.0e+02;          /* x wUnit2rVel = x z2rUnit = 1 */
  const double maxSlopeSqr = m->GM_maxSlope * m->GM_maxSlope;
  for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
    for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++)
      if (L(dSigmaDr, i, j) != 0.0 && L(dSigmaDr, i, j) <= m->GM_Small_Number) L(dSigmaDr, i, j) = m->GM_Small_Number;
  for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
    for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
      if (L(dSigmaDr, i, j) == 0.0) {
        L(SlopeX, i, j) = L(dSigmaDx, i, j) != 0.0 ? copysign(GM_bigSlope, L(dSigmaDx, i, j)) : 0.0;
        L(SlopeY, i, j) = L(dSigmaDy, i, j) != 0.0 ? copysign(GM_bigSlope, L(dSigmaDy, i, j)) : 0.0;
      } else {
        const double dRdSigmaLtd = 1.0 / L(dSigmaDr, i, j);
        L(SlopeX, i, j) = L(dSigmaDx, i, j) * dRdSigmaLtd;
        L(SlopeY, i, j) = L(dSigmaDy, i, j) * dRdSigmaLtd;
      }
    }
  for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
    for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
      L(SlopeSqr, i, j) = L(SlopeX, i, j) * L(SlopeX, i, j) + L(SlopeY, i, j) * L(SlopeY, i, j);
      L(taperFct, i, j) = 1.0;
      if (L(SlopeSqr, i, j) >= m->GM_slopeSqCutoff) {
        L(SlopeSqr, i, j) = m->GM_slopeSqCutoff;
        L(taperFct, i, j) = 0.0;
      }
    }
  for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
    for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
      if (L(SlopeSqr, i, j) == 0.0) L(taperFct, i, j) = 1.0;
      else if (L(SlopeSqr, i, j) > maxSlopeSqr && L(SlopeSqr, i, j) < m->GM_slopeSqCutoff)
        L(taperFct, i, j) = maxSlopeSqr / L(SlopeSqr, i, j);
    }
}

/* GMREDI_CALC_PSI_B (gmredi_calc_psi_b.F:86-212) with GMREDI_SLOPE_PSI's gkw91 branch
 * (gmredi_slope_psi.F:196-290): the bolus stream-function GM_PsiX/Y at the top face of
 * level k = 2..Nr (level 1 stays 0), U / V points.  z-coordinates: wUnit2rVel = 1. */
static void gmredi_calc_psi_b(OModel *m, int t) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long n2 = m->n2, n3 = m->n3;
  const double op25 = 0.25, halfRL = 0.5, halfSign = halfRL * m->gravitySign;
  const double *sigmaX = m->sigmaX + t * n3, *sigmaY = m->sigmaY + t * n3, *sigmaR = m->sigmaR + t * n3;
  const double *maskW = m->maskW + t * n3, *maskS = m->maskS + t * n3;
  double *PsiX = m->GM_PsiX + t * n3, *PsiY = m->GM_PsiY + t * n3;
  const double slopeCutoff = sqrt(m->GM_slopeSqCutoff);
  const double loc_maxSlope = m->GM_maxSlope * 1.0, maxSlopeSqr = loc_maxSlope * loc_maxSlope;
  for (int k = 2; k <= Nr; k++) {
    const int km1 = k - 1;
    const double half_K = m->GM_background_K * (1.0 + 1.0) * op25;
    for (int j = 1 - OLy; j <= sNy + OLy; j++)
      for (int i = 1 - OLx + 1; i <= sNx + OLx; i++) {
        const double mk = W3(maskW, i, j, km1) * W3(maskW, i, j, k);
        double SlopeX = (W3(sigmaX, i, j, km1) + W3(sigmaX, i, j, k)) * halfRL * mk;
        double dSdr = (W3(sigmaR, i - 1, j, k) + W3(sigmaR, i, j, k)) * halfSign * mk;
        if (dSdr <= m->GM_Small_Number) dSdr = m->GM_Small_Number;
        SlopeX = SlopeX / dSdr;
        double taper = 1.0;
        if (fabs(SlopeX) >= slopeCutoff) { SlopeX = copysign(slopeCutoff, SlopeX); taper = 0.0; }
        const double Smod = fabs(SlopeX);
        if (Smod > loc_maxSlope && Smod < slopeCutoff) taper = maxSlopeSqr / (SlopeX * SlopeX + m->GM_Small_Number);
        W3(PsiX, i, j, k) = SlopeX * taper * (half_K * (1.0 + 1.0));
      }
    for (int j = 1 - OLy + 1; j <= sNy + OLy; j++)
      for (int i = 1 - OLx; i <= sNx + OLx; i++) {
        const double mk = W3(maskS, i, j, km1) * W3(maskS, i, j, k);
        double SlopeY = (W3(sigmaY, i, j, km1) + W3(sigmaY, i, j, k)) * halfRL * mk;
        double dSdr = (W3(sigmaR, i, j - 1, k) + W3(sigmaR, i, j, k)) * halfSign * mk;
        if (dSdr <= m->GM_Small_Number) dSdr = m->GM_Small_Number;
        SlopeY = SlopeY / dSdr;
        double taper = 1.0;
        if (fabs(SlopeY) >= slopeCutoff) { SlopeY = copysign(slopeCutoff, SlopeY); taper = 0.0; }
        const double Smod = fabs(SlopeY);
        if (Smod > loc_maxSlope && Smod < slopeCutoff) taper = maxSlopeSqr / (SlopeY * SlopeY + m->GM_Small_Number);
        W3(PsiY, i, j, k) = SlopeY * taper * (half_K * (1.0 + 1.0));
      }
  }
}

void oracle_gmredi_calc_tensor(OModel *m, int t) {
  const int sNx = m->sNx, sNy = m->sNy, OLx = m->OLx, OLy = m->OLy, Nr = m->Nr, nx = m->nx;
  const long n2 = m->n2, n3 = m->n3;
  const double op25 = 0.25, op5 = 0.5, gravitySign = m->gravitySign;
  const double *sigmaX = m->sigmaX + t * n3, *sigmaY = m->sigmaY + t * n3, *sigmaR = m->sigmaR + t * n3;
  const double *maskC = m->maskC + t * n3, *maskW = m->maskW + t * n3, *maskS = m->maskS + t * n3;
  double *Kwx = m->Kwx + t * n3, *Kwy = m->Kwy + t * n3, *Kwz = m->Kwz + t * n3;
  double *Kux = m->Kux + t * n3, *Kvy = m->Kvy + t * n3, *Kuz = m->Kuz + t * n3, *Kvz = m->Kvz + t * n3;
  double *dSx = calloc(n2, 8), *dSy = calloc(n2, 8), *dSr = calloc(n2, 8), *maskFk = calloc(n2, 8);
  double *SlopeX = calloc(n2, 8), *SlopeY = calloc(n2, 8), *SlopeSqr = calloc(n2, 8), *taper = calloc(n2, 8);
  /* Kwx, Kwy, Kwz at W points, k = Nr..2 (gmredi_calc_tensor.F:259-405) */
  for (int k = Nr; k >= 2; k--) {
    for (int j = 1 - OLy; j <= sNy + OLy; j++)
      for (int i = 1 - OLx; i <= sNx + OLx; i++) L(maskFk, i, j) = W3(maskC, i, j, k - 1) * W3(maskC, i, j, k);
    for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
      for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
        L(dSx, i, j) = op25 * (W3(sigmaX, i + 1, j, k - 1) + W3(sigmaX, i, j, k - 1) + W3(sigmaX, i + 1, j, k) +
                               W3(sigmaX, i, j, k)) * L(maskFk, i, j);
        L(dSy, i, j) = op25 * (W3(sigmaY, i, j + 1, k - 1) + W3(sigmaY, i, j, k - 1) + W3(sigmaY, i, j + 1, k) +
                               W3(sigmaY, i, j, k)) * L(maskFk, i, j);
      }
    for (int j = 1 - OLy; j <= sNy + OLy; j++)
      for (int i = 1 - OLx; i <= sNx + OLx; i++) L(dSr, i, j) = gravitySign * W3(sigmaR, i, j, k);
    slope_limit_gkw91(m, dSx, dSy, dSr, SlopeX, SlopeY, SlopeSqr, taper);
    for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
      for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
        W3(Kwx, i, j, k) = -gravitySign * L(SlopeX, i, j) * L(taper, i, j);
        W3(Kwy, i, j, k) = -gravitySign * L(SlopeY, i, j) * L(taper, i, j);
        W3(Kwz, i, j, k) = L(SlopeSqr, i, j) * L(taper, i, j);
      }
  }
  for (int k = 1; k <= Nr; k++) {
    const double isopycK = m->GM_isopycK * (1.0 + 1.0) * op5;      /* GM_isoFac1d = 1 */
    const double bolus_K = m->GM_background_K * (1.0 + 1.0) * op5; /* GM_bolFac1d = 1 */
    for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
      for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
        const double Kgm_tmp = isopycK * 1.0 + m->GM_skewflx * bolus_K * 1.0;
        W3(Kwx, i, j, k) = Kgm_tmp * W3(Kwx, i, j, k);
        W3(Kwy, i, j, k) = Kgm_tmp * W3(Kwy, i, j, k);
        W3(Kwz, i, j, k) = (isopycK * 1.0) * W3(Kwz, i, j, k);
      }
  }
  /* Kux at U points (gmredi_calc_tensor.F:560-640), k = Nr..1 */
  for (int k = Nr; k >= 1; k--) {
    const int kp1 = k + 1 < Nr ? k + 1 : Nr;
    const double maskp1 = k >= Nr ? 0.0 : 1.0;
    for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
      for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
        L(dSx, i, j) = W3(sigmaX, i, j, k) * W3(maskW, i, j, k);
        L(dSy, i, j) = op25 * (W3(sigmaY, i - 1, j + 1, k) + W3(sigmaY, i, j + 1, k) + W3(sigmaY, i - 1, j, k) +
                               W3(sigmaY, i, j, k)) * W3(maskW, i, j, k);
        L(dSr, i, j) = op25 * (W3(sigmaR, i - 1, j, k) + W3(sigmaR, i, j, k) +
                               (W3(sigmaR, i - 1, j, kp1) + W3(sigmaR, i, j, kp1)) * maskp1) *
                       W3(maskW, i, j, k) * gravitySign;
      }
    slope_limit_gkw91(m, dSx, dSy, dSr, SlopeX, SlopeY, SlopeSqr, taper);
    for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
      for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
        W3(Kux, i, j, k) = (m->GM_isopycK * 1.0 * op5 * (1.0 + 1.0)) * L(taper, i, j);
        W3(Kux, i, j, k) = fmax(W3(Kux, i, j, k), m->GM_Kmin_horiz);
      }
    if (m->GM_ExtraDiag) /* GM_EXTRA_DIAGONAL (gmredi_calc_tensor.F:808-850) */
      for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
        for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++)
          W3(Kuz, i, j, k) = -gravitySign *
                             (m->GM_isopycK * 1.0 * op5 * (1.0 + 1.0) -
                              m->GM_skewflx * m->GM_background_K * 1.0 * op5 * (1.0 + 1.0)) *
                             L(SlopeX, i, j) * L(taper, i, j);
  }
  /* Kvy at V points (gmredi_calc_tensor.F:700-790) */
  for (int k = Nr; k >= 1; k--) {
    const int kp1 = k + 1 < Nr ? k + 1 : Nr;
    const double maskp1 = k >= Nr ? 0.0 : 1.0;
    for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
      for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
        L(dSx, i, j) = op25 * (W3(sigmaX, i, j, k) + W3(sigmaX, i + 1, j, k) + W3(sigmaX, i, j - 1, k) +
                               W3(sigmaX, i + 1, j - 1, k)) * W3(maskS, i, j, k);
        L(dSy, i, j) = W3(sigmaY, i, j, k) * W3(maskS, i, j, k);
        L(dSr, i, j) = op25 * (W3(sigmaR, i, j - 1, k) + W3(sigmaR, i, j, k) +
                               (W3(sigmaR, i, j - 1, kp1) + W3(sigmaR, i, j, kp1)) * maskp1) *
                       W3(maskS, i, j, k) * gravitySign;
      }
    slope_limit_gkw91(m, dSx, dSy, dSr, SlopeX, SlopeY, SlopeSqr, taper);
    for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
      for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++) {
        W3(Kvy, i, j, k) = (m->GM_isopycK * 1.0 * op5 * (1.0 + 1.0)) * L(taper, i, j);
        W3(Kvy, i, j, k) = fmax(W3(Kvy, i, j, k), m->GM_Kmin_horiz);
      }
    if (m->GM_ExtraDiag) /* gmredi_calc_tensor.F:1053-1090 */
      for (int j = 1 - OLy + 1; j <= sNy + OLy - 1; j++)
        for (int i = 1 - OLx + 1; i <= sNx + OLx - 1; i++)
          W3(Kvz, i, j, k) = -gravitySign *
                             (m->GM_isopycK * 1.0 * op5 * (1.0 + 1.0) -
                              m->GM_skewflx * m->GM_background_K * 1.0 * op5 * (1.0 + 1.0)) *
                             L(SlopeY, i, j) * L(taper, i, j);
  }
  if (m->GM_AdvForm) gmredi_calc_psi_b(m, t);
  free(dSx); free(dSy); free(dSr); free(maskFk); free(SlopeX); free(SlopeY); free(SlopeSqr); free(taper);
}
