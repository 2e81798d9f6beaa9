// phys.h -- DO_OCEANIC_PHYS's per-point work (EOS, surface forcing, IVDC), shared by
// k_oceanic_phys (kernels_thermo.hip) and the fused DO_OCEANIC_PHYS + CALC_PHI_HYD column
// pass k_phys_phi (kernels_dyn.hip).
#pragma once
#include "common.h"

namespace mgcm {

// FIND_RHO_2D at one point (find_rho.F:84-99 LINEAR, :146-180 JMD95Z with
// FIND_RHOP0 :274-409 and FIND_BULKMOD :411-590, coefficients ini_eos.F:113-160;
// selectP_inEOS_Zc = 0: locPres = pRef4EOS(kRef), pressure_for_eos.F:88-96).
__device__ __forceinline__ double jmd95_rho(const Params &p, double locPres, double t, double s) {
  const double t2 = t * t, t3 = t2 * t, t4 = t3 * t;
  double s3o2;
  if (s > 0.0) s3o2 = s * sqrt(s);
  else { s = 0.0; s3o2 = 0.0; }
  const double rfresh = 999.842594 + 6.793952e-02 * t + -9.095290e-03 * t2 + 1.001685e-04 * t3 +
                        -1.120083e-06 * t4 + 6.536332e-09 * t4 * t;
  const double rsalt = s * (8.24493e-01 + -4.0899e-03 * t + 7.6438e-05 * t2 + -8.2467e-07 * t3 + 5.3875e-09 * t4) +
                       s3o2 * (-5.72466e-03 + 1.0227e-04 * t + -1.6546e-06 * t2) + 4.8314e-04 * s * s;
  const double rhoP0 = rfresh + rsalt;
  const double pb = locPres * 1.0e-05, p2 = pb * pb;
  const double bMfresh = 1.965933e+04 + 1.444304e+02 * t + -1.706103e+00 * t2 + 9.648704e-03 * t3 +
                         -4.190253e-05 * t4;
  const double bMsalt = s * (5.284855e+01 + -3.101089e-01 * t + 6.283263e-03 * t2 + -5.084188e-05 * t3) +
                        s3o2 * (3.886640e-01 + 9.085835e-03 * t + -4.619924e-04 * t2);
  const double bMpres = pb * (3.186519e+00 + 2.212276e-02 * t + -2.984642e-04 * t2 + 1.956415e-06 * t3) +
                        pb * s * (6.704388e-03 + -1.847318e-04 * t + 2.059331e-07 * t2) + pb * s3o2 * 1.480266e-04 +
                        p2 * (2.102898e-04 + -1.202016e-05 * t + 1.394680e-07 * t2) +
                        p2 * s * (-2.040237e-06 + 6.128773e-08 * t + 6.207323e-10 * t2);
  const double bulkMod = bMfresh + bMsalt + bMpres;
  return rhoP0 / (1.0 - locPres * 1.0e-05 / bulkMod) - p.rhoConst;
}
// PRESSURE_FOR_EOS (pressure_for_eos.F:51-105), z-coordinates, dpRef = 0: JMD95P
// (selectP_inEOS_Zc = 2) uses the hydrostatic pressure rhoConst*(totPhiHyd + phiRef(2k))
// of the point q3 (level kRef); JMD95Z the reference profile pRef4EOS(kRef).
__device__ __forceinline__ double pressure_for_eos(const Params &p, const Fields &f, int kRef, long q3) {
  if (p.selectP_inEOS_Zc == 2) return p.rhoConst * (f.totPhiHyd[q3] + f.phiRefC[kRef - 1]) + 0.0;
  return f.pRef4EOS[kRef - 1] + 0.0;
}
// q3: flat offset of the point at level kRef (for the JMD95P pressure)
__device__ __forceinline__ double find_rho(const Params &p, const Fields &f, int kRef, long q3, double t, double s) {
  if (p.eosType == 1) return jmd95_rho(p, pressure_for_eos(p, f, kRef, q3), t, s);
  const double refTemp = f.tRef[kRef - 1], refSalt = f.sRef[kRef - 1];
  const double dRho = p.rhoNil - p.rhoConst;
  return p.rhoNil * (p.sBeta * (s - refSalt) - p.tAlpha * (t - refTemp)) + dRho;
}

// DO_OCEANIC_PHYS (do_oceanic_phys.F:548-882) per column over the full halo range:
// FREEZE_SURFACE (freeze_surface.F:55-66), EXTERNAL_FORCING_SURF with
// FORCING_SURF_RELAX (external_forcing_surf.F:90-290, forcing_surf_relax.F:75-100;
// linear free surface), FIND_RHO_2D at every level (kRef = k), GRAD_SIGMA's sigmaR with
// rho(theta(k-1), kRef = k) (grad_sigma.F:103-117) and CALC_IVDC (calc_ivdc.F:60-71).
// LOAD_FIELDS_DRIVER's EXTERNAL_FIELDS_LOAD (external_fields_load.F:56-330, with
// GET_PERIODIC_INTERVAL get_periodic_interval.F:106-117, at myTime = myIter*deltaTClock read
// from the device step counter) is folded in: the k = 1 thread of each column interpolates
// the six monthly records at its point -- the only point DO_OCEANIC_PHYS reads them at --
// and stores them for the later readers (momentum, continuity): one launch fewer per step.
// One point (i,j,k) of the full halo range: FREEZE_SURFACE only changes theta(k=1), so
// every reader of theta(k=1) applies the clamp itself and the k = 1 thread stores it.
// Returns rhoInSitu(i,j,k) (also stored).
__device__ __forceinline__ double oceanic_phys_point(const Dims &d, const Params &p, const Fields &f, const int *iterPtr,
                                                     int i, int j, int k, int t) {
  const long q = MG_I2(d, i, j, t), q31 = MG_I3(d, i, j, 1, t);
  auto theta_at = [&](int kk) {
    const double v = f.theta[MG_I3(d, i, j, kk, t)];
    return (kk == 1 && p.allowFreezing && v < -1.9) ? -1.9 : v;
  };
  if (k == 1 && p.periodicExternalForcing) {
    const long N2 = d.n2 * d.nTiles;
    const double cycleLength = p.externForcingCycle, recSpacing = p.externForcingPeriod;
    const double currentTime = (double)(*iterPtr) * p.deltaTClock;
    const int nbRec = (int)llround(cycleLength / recSpacing);
    const double locTime = currentTime - recSpacing * 0.5 + cycleLength * (double)(2 - llround(currentTime / cycleLength));
    const double tmpTime = fmod(locTime, cycleLength);
    const int tRec1 = 1 + (int)(tmpTime / recSpacing);
    const int tRec2 = 1 + tRec1 % nbRec;
    const double aW = (tmpTime - recSpacing * (double)(tRec1 - 1)) / recSpacing;
    const double bW = 1.0 - aW;
    double *dst[6] = {f.SST, f.SSS, f.fu, f.fv, f.Qnet, f.EmPmR};
#pragma unroll
    for (int v = 0; v < 6; v++) {
      const double *r = f.forcRec + (long)v * p.nForcRec * N2;
      dst[v][q] = bW * r[(long)(tRec1 - 1) * N2 + q] + aW * r[(long)(tRec2 - 1) * N2 + q];
    }
  }
  if (k == 1) {
    const double th1 = theta_at(1), s1 = f.salt[q31];
    if (p.allowFreezing) f.theta[q31] = th1;
    const double mass2rUnit = 1.0 / p.rhoConst, recip_Cp = 1.0 / p.HeatCapacity_Cp;
    double sfT = -(f.lambdaThetaClimRelax[q] * (th1 - f.SST[q]) * f.drF[0] * f.hFacC[q31]);
    double sfS = -(f.lambdaSaltClimRelax[q] * (s1 - f.SSS[q]) * f.drF[0] * f.hFacC[q31]);
    sfT = sfT - f.Qnet[q] * recip_Cp * mass2rUnit;
    sfS = sfS - 0.0 * mass2rUnit;   // saltFlux = 0
    const double UNSET_RL = 123456.7;
    if (p.nonlinFreeSurf > 0 && p.useRealFreshWaterFlux) {
      // external_forcing_surf.F:253-277: PmEpR changes the column height
      if (p.temp_EvPrRn != UNSET_RL) sfT = sfT + f.PmEpR[q] * (p.temp_EvPrRn - th1) * mass2rUnit;
      if (p.salt_EvPrRn != UNSET_RL) sfS = sfS + f.PmEpR[q] * (p.salt_EvPrRn - s1) * mass2rUnit;
    } else if (p.convertFW2Salt == -1.0) {
      if (p.temp_EvPrRn != UNSET_RL) sfT = sfT + f.EmPmR[q] * (th1 - p.temp_EvPrRn) * mass2rUnit;
      if (p.salt_EvPrRn != UNSET_RL) sfS = sfS + f.EmPmR[q] * (s1 - p.salt_EvPrRn) * mass2rUnit;
    } else {
      if (p.temp_EvPrRn != UNSET_RL) sfT = sfT + f.EmPmR[q] * (f.tRef[0] - p.temp_EvPrRn) * mass2rUnit;
      if (p.salt_EvPrRn != UNSET_RL) sfS = sfS + f.EmPmR[q] * (p.convertFW2Salt - p.salt_EvPrRn) * mass2rUnit;
    }
    f.surfaceForcingT[q] = sfT;
    f.surfaceForcingS[q] = sfS;
  }
  const long q3 = MG_I3(d, i, j, k, t);
  const double rho = find_rho(p, f, k, q3, theta_at(k), f.salt[q3]);
  f.rhoInSitu[q3] = rho;
  const bool calcConvect = p.ivdc_kappa != 0.0;
  double conv = 0.0, sigmaR = 0.0;
  if (k >= 2 && (calcConvect || p.useGMRedi)) {
    const long q3u = MG_I3(d, i, j, k - 1, t);
    const double rhoKm1 = find_rho(p, f, k, q3, theta_at(k - 1), f.salt[q3u]);
    sigmaR = f.maskC[q3] * f.maskC[q3u] * f.recip_drC[k - 1] * p.rkSign * (rho - rhoKm1);
    if (calcConvect) conv = (-sigmaR * p.gravitySign > 0.0) ? 1.0 : 0.0;
  }
  f.IVDConvCount[q3] = conv;
  if (p.useGMRedi) f.sigmaR[q3] = sigmaR;
  return rho;
}


}  // namespace mgcm
