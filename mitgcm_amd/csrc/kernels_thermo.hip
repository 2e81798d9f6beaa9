// kernels_thermo.hip -- the tracer half of the step on the MI355X.
//
//   k_oceanic_phys  DO_OCEANIC_PHYS subset (model/src/do_oceanic_phys.F:555-882):
//                   surfaceForcingT from FORCING_SURF_RELAX (forcing_surf_relax.F:52-80),
//                   rhoInSitu = FIND_RHO_2D LINEAR (find_rho.F:125-136) at every level,
//                   IVDConvCount from GRAD_SIGMA/CALC_IVDC (grad_sigma.F:103-117, calc_ivdc.F:60-71).
//   tracer step     TEMP_INTEGRATE / SALT_INTEGRATE (model/src/temp_integrate.F) for one
//                   tracer: GAD C2 advection (gad_c2_adv_x/y/r.F) with AB2 on the tendency
//                   (adams_bashforth2.F:81-88), or the multi-dimensional DST3 flux-limited
//                   advection (gad_advection.F + gad_dst3fl_adv_x/y/r.F, k_adv_x/y/r) stepped
//                   forward; Laplacian diffusion (gad_diff_x/y.F), surface forcing
//                   (apply_forcing.F:687-695), TIMESTEP_TRACER, vertical diffusion explicit
//                   (gad_diff_r.F) or implicit (GAD_IMPLICIT_R, gad_implicit_r.F:96-140, Thomas
//                   sweep of SOLVE_TRIDIAGONAL), CYCLE_TRACER.
//
// k_tracer_rhs runs one thread per interior (i,j,k) point: both vertical faces of
// the level (the fVerT(kUp/kDown) ping-pong of temp_integrate.F) and the four
// horizontal faces are recomputed from the neighbours' state with the
// reference's operand order (bit-exact under -ffp-contract=off).  k_tracer_impl
// then runs the implicit vertical solve one thread per column.  The new theta
// goes to the other buffer of a ping-pong pair (neighbours still read the old
// one); the Thomas coefficients live in per-column scratch (L2-resident).  Only
// the interior is produced: the halo of theta is refilled by the end-of-step
// EXCH (do_fields_blocking_exchanges.F).
#include "common.h"

namespace mgcm {

__device__ __forceinline__ double rho_linear(const Params &p, const Fields &f, int kRef, double t, double s) {
  const double refTemp = f.tRef[kRef - 1], refSalt = f.sRef[kRef - 1];
  const double dRho = p.rhoNil - p.rhoConst;
  return p.rhoNil * (p.sBeta * (s - refSalt) - p.tAlpha * (t - refTemp)) + dRho;
}

__global__ void __launch_bounds__(256) k_oceanic_phys(Dims d, Params p, Fields f) {
  MG_PLANE(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, tz)
  const int t = d.t0 + tz;
  if (i > d.sNx + d.OLx || j > d.sNy + d.OLy) return;
  const long q = MG_I2(d, i, j, t);
  f.surfaceForcingT[q] =
      -(f.lambdaThetaClimRelax[q] * (f.theta[MG_I3(d, i, j, 1, t)] - f.SST[q]) * f.drF[0] * f.hFacC[MG_I3(d, i, j, 1, t)]);
  double rhoUp = 0.0, thUp = 0.0, sUp = 0.0, mUp = 0.0;
  for (int k = 1; k <= d.Nr; k++) {
    const long q3 = MG_I3(d, i, j, k, t);
    const double th = f.theta[q3], sa = f.salt[q3], mC = f.maskC[q3];
    const double rho = rho_linear(p, f, k, th, sa);
    f.rhoInSitu[q3] = rho;
    double conv = 0.0;
    if (k >= 2 && p.ivdc_kappa != 0.0) {
      const double rhoKm1 = rho_linear(p, f, k, thUp, sUp);
      const double sigmaR = mC * mUp * f.recip_drC[k - 1] * p.rkSign * (rho - rhoKm1);
      conv = (-sigmaR * p.gravitySign > 0.0) ? 1.0 : 0.0;
    }
    f.IVDConvCount[q3] = conv;
    rhoUp = rho; thUp = th; sUp = sa; mUp = mC;
  }
  (void)rhoUp;
}

// ---------------------------------------------------------------------------
// GAD_DST3FL_ADV_X/Y/R (gad_dst3fl_adv_x.F:47-99, _y.F, _r.F:70-119)
__device__ __forceinline__ double dst3fl_limit(double d0, double d1, double theta, double cfl) {
  const double psi = d0 + d1 * theta;
  return fmax(0.0, fmin(fmin(1.0, psi), theta * (1.0 - cfl) / (cfl + 1.0e-20)));
}
__device__ __forceinline__ double dst3fl_theta(double Rj, double Rother) {
  const double thetaMax = 1.0e+20;
  if (fabs(Rj) * thetaMax <= fabs(Rother)) return copysign(thetaMax, Rother * Rj);
  return Rother / Rj;
}
// face flux between cells m1 (upstream for positive transport) and p0
__device__ __forceinline__ double dst3fl_h(double uTr, double cfl, double tm2, double tm1, double t0, double tp1,
                                           double mWm1, double mW0, double mWp1) {
  const double oneSixth = 1.0 / 6.0;
  const double Rjp = (tp1 - t0) * mWp1, Rj = (t0 - tm1) * mW0, Rjm = (tm1 - tm2) * mWm1;
  const double d0 = (2.0 - cfl) * (1.0 - cfl) * oneSixth, d1 = (1.0 - cfl * cfl) * oneSixth;
  const double psiP = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjm), cfl);
  const double psiM = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjp), cfl);
  return 0.5 * (uTr + fabs(uTr)) * (tm1 + psiP * Rj) + 0.5 * (uTr - fabs(uTr)) * (t0 - psiM * Rj);
}

// GAD_ADVECTION (gad_advection.F), lat-lon operator splitting (npass = 2), X pass:
// loc1 = T - dT/(h drF rA) * (afx(i+1) - afx(i) - T*(uTrans(i+1) - uTrans(i))) * maskInC
// on i = 2-OLx..sNx+OLx-1, every j; elsewhere loc1 = T.
__global__ void __launch_bounds__(256) k_adv_x(Dims d, Fields f, TracerArgs a) {
  MG_PLANE(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  if (i > d.sNx + d.OLx || j > d.sNy + d.OLy) return;
  const double *__restrict__ T = a.tr;
  const long q3 = MG_I3(d, i, j, k, t);
  double v = T[q3];
  if (i >= 2 - d.OLx && i <= d.sNx + d.OLx - 1) {
    const double drF = f.drF[k - 1], dT = a.dT;
    auto uTr = [&](int ii) { return f.uVel[MG_I3(d, ii, j, k, t)] * (f.dyG[MG_I2(d, ii, j, t)] * drF * f.hFacW[MG_I3(d, ii, j, k, t)]); };
    auto afx = [&](int ii) {   // zero at i = 1-OLx, 2-OLx, sNx+OLx
      if (ii < 3 - d.OLx || ii > d.sNx + d.OLx - 1) return 0.0;
      const double cfl = fabs(f.uVel[MG_I3(d, ii, j, k, t)] * dT * f.recip_dxC[MG_I2(d, ii, j, t)]);
      return dst3fl_h(uTr(ii), cfl, T[MG_I3(d, ii - 2, j, k, t)], T[MG_I3(d, ii - 1, j, k, t)], T[MG_I3(d, ii, j, k, t)],
                      T[MG_I3(d, ii + 1, j, k, t)], f.maskW[MG_I3(d, ii - 1, j, k, t)], f.maskW[MG_I3(d, ii, j, k, t)],
                      f.maskW[MG_I3(d, ii + 1, j, k, t)]);
    };
    const long q = MG_I2(d, i, j, t);
    v = v - dT * f.recip_hFacC[q3] * f.recip_drF[k - 1] * f.recip_rA[q] *
                (afx(i + 1) - afx(i) - T[q3] * (uTr(i + 1) - uTr(i))) * f.maskInC[q];
  }
  f.advScr1[q3] = v;
}

// Y pass on the interior (the only rows the vertical pass and the tendency use):
// loc2 = loc1 - dT/(h drF rA) * (afy(j+1) - afy(j) - T*(vTrans(j+1) - vTrans(j))) * maskInC
__global__ void __launch_bounds__(256) k_adv_y(Dims d, Fields f, TracerArgs a) {
  MG_PLANE(1, d.sNx, 1, d.sNy, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  if (i > d.sNx || j > d.sNy) return;
  const double *__restrict__ L1 = f.advScr1;
  const long q3 = MG_I3(d, i, j, k, t);
  const double drF = f.drF[k - 1], dT = a.dT;
  auto vTr = [&](int jj) { return f.vVel[MG_I3(d, i, jj, k, t)] * (f.dxG[MG_I2(d, i, jj, t)] * drF * f.hFacS[MG_I3(d, i, jj, k, t)]); };
  auto afy = [&](int jj) {   // zero at j = 1-OLy, 2-OLy, sNy+OLy
    if (jj < 3 - d.OLy || jj > d.sNy + d.OLy - 1) return 0.0;
    const double cfl = fabs(f.vVel[MG_I3(d, i, jj, k, t)] * dT * f.recip_dyC[MG_I2(d, i, jj, t)]);
    return dst3fl_h(vTr(jj), cfl, L1[MG_I3(d, i, jj - 2, k, t)], L1[MG_I3(d, i, jj - 1, k, t)], L1[MG_I3(d, i, jj, k, t)],
                    L1[MG_I3(d, i, jj + 1, k, t)], f.maskS[MG_I3(d, i, jj - 1, k, t)], f.maskS[MG_I3(d, i, jj, k, t)],
                    f.maskS[MG_I3(d, i, jj + 1, k, t)]);
  };
  const long q = MG_I2(d, i, j, t);
  f.advScr2[q3] = L1[q3] - dT * f.recip_hFacC[q3] * f.recip_drF[k - 1] * f.recip_rA[q] *
                               (afy(j + 1) - afy(j) - a.tr[q3] * (vTr(j + 1) - vTr(j))) * f.maskInC[q];
}

// vertical pass + advective tendency gAdv = (loc - T)/dT (gad_advection.F k = Nr..1 loop)
__global__ void __launch_bounds__(256) k_adv_r(Dims d, Params p, Fields f, TracerArgs a) {
  MG_PLANE(1, d.sNx, 1, d.sNy, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  if (i > d.sNx || j > d.sNy) return;
  const int Nr = d.Nr;
  const double *__restrict__ L2 = f.advScr2;
  const long q = MG_I2(d, i, j, t), q3 = MG_I3(d, i, j, k, t);
  const double rA = f.rA[q], dT = a.dT;
#define MC(kk) f.maskC[MG_I3(d, i, j, kk, t)]
#define LT(kk) L2[MG_I3(d, i, j, kk, t)]
  auto rtr = [&](int kk) { return (kk <= 1 || kk > Nr) ? 0.0 : f.wVel[MG_I3(d, i, j, kk, t)] * rA * MC(kk - 1); };
  auto fver = [&](int kk) {   // fVerT through the top of level kk, 0 at kk = 1 and below Nr
    if (kk <= 1 || kk > Nr) return 0.0;
    const int km2 = kk - 2 > 1 ? kk - 2 : 1, km1 = kk - 1 > 1 ? kk - 1 : 1, kp1 = kk + 1 < Nr ? kk + 1 : Nr;
    const double Rjp = (LT(kk) - LT(kp1)) * MC(kp1);
    const double Rj = (LT(km1) - LT(kk)) * MC(kk) * MC(km1);
    const double Rjm = (LT(km2) - LT(km1)) * MC(km1);
    const double cfl = fabs(f.wVel[MG_I3(d, i, j, kk, t)] * dT * f.recip_drC[kk - 1]);
    const double oneSixth = 1.0 / 6.0;
    const double d0 = (2.0 - cfl) * (1.0 - cfl) * oneSixth, d1 = (1.0 - cfl * cfl) * oneSixth;
    const double psiP = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjm), cfl);
    const double psiM = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjp), cfl);
    const double rT = rtr(kk);
    return 0.5 * (rT + fabs(rT)) * (LT(kk) + psiM * Rj) + 0.5 * (rT - fabs(rT)) * (LT(km1) - psiP * Rj);
  };
  const double kp1Msk = (k == Nr) ? 0.0 : 1.0;
  const double rTrans = rtr(k), rTransKp = kp1Msk * rtr(k + 1);
  const double fUp = fver(k), fDn = fver(k + 1);
  const double lt = LT(k) - dT * f.recip_hFacC[q3] * f.recip_drF[k - 1] * f.recip_rA[q] *
                                (fDn - fUp - a.tr[q3] * (rTransKp - rTrans)) * p.rkSign * f.maskInC[q];
  f.gAdv[q3] = (lt - a.tr[q3]) / dT;
#undef MC
#undef LT
}

// GAD_CALC_RHS + forcing + AB2 + TIMESTEP_TRACER for one interior (i,j,k) point:
// writes gNm1 (AB tracers) and gTscr = tracer + dTtracer*gT (the right-hand side of
// the implicit vertical solve, or the new tracer with explicit vertical diffusion).
__global__ void __launch_bounds__(256) k_tracer_rhs(Dims d, Params p, Fields f, TracerArgs a, const int *iterPtr) {
  MG_PLANE(1, d.sNx, 1, d.sNy, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  if (i > d.sNx || j > d.sNy) return;
  const int Nr = d.Nr;
  const int myIter = *iterPtr;
  const double abFac = (myIter == p.nIter0 && p.nIter0 == 0) ? 0.0 : 0.5 + p.abEps;
  const bool calcAdv = a.advection && !a.multiDim;
  const double advFac = calcAdv ? 1.0 : 0.0, rAdvFac = p.rkSign * advFac;
  const double *__restrict__ T = a.tr;
  const long q = MG_I2(d, i, j, t);
  const double maskInC = f.maskInC[q], recip_rA = f.recip_rA[q], rA = f.rA[q];
#define T3(ii, jj, kk) T[MG_I3(d, ii, jj, kk, t)]
#define G2(a_, ii, jj) f.a_[MG_I2(d, ii, jj, t)]
#define G3(a_, ii, jj, kk) f.a_[MG_I3(d, ii, jj, kk, t)]
  const double drF = f.drF[k - 1];
  // west / south face fluxes of the column (fZon, fMer): GAD_C2_ADV_X/Y + GAD_DIFF_X/Y
  auto fzon = [&](int ii) {
    const double xA = G2(dyG, ii, j) * drF * G3(hFacW, ii, j, k);
    double fz = 0.0;
    if (calcAdv) fz = fz + (G3(uVel, ii, j, k) * xA) * (T3(ii, j, k) + T3(ii - 1, j, k)) * 0.5;
    double df = 0.0;
    if (a.diffKh != 0.0) df = -a.diffKh * xA * G2(recip_dxC, ii, j) * (T3(ii, j, k) - T3(ii - 1, j, k));
    return fz + df;
  };
  auto fmer = [&](int jj) {
    const double yA = G2(dxG, i, jj) * drF * G3(hFacS, i, jj, k);
    double fm = 0.0;
    if (calcAdv) fm = fm + (G3(vVel, i, jj, k) * yA) * (T3(i, jj, k) + T3(i, jj - 1, k)) * 0.5;
    double df = 0.0;
    if (a.diffKh != 0.0) df = -a.diffKh * yA * G2(recip_dyC, i, jj) * (T3(i, jj, k) - T3(i, jj - 1, k));
    return fm + df;
  };
  // CALC_ADV_FLOW rTrans of level kk (0 at the surface and below the bottom level)
  auto rtrans = [&](int kk) {
    if (kk <= 1 || kk > Nr) return 0.0;
    const double maskUp = G3(maskC, i, j, kk - 1) * G3(maskC, i, j, kk);
    return G3(wVel, i, j, kk) * rA * maskUp;
  };
  // fVerT through the top face of level kk: GAD_C2_ADV_R + vertical diffusive flux
  // (GAD_DIFF_R when diffusion is explicit, 0 with implicitDiffusion)
  auto fvert = [&](int kk, double rTr) {
    double fv = 0.0;
    if (kk >= 2 && kk <= Nr && calcAdv) {
      const double wT = G3(maskC, i, j, kk - 1) * rTr * (T3(i, j, kk) + T3(i, j, kk - 1)) * 0.5;
      fv = fv + wT * maskInC;
    }
    double dfr = 0.0;
    if (!p.implicitDiffusion && kk >= 2 && kk <= Nr) {
      const double kap = (G3(IVDConvCount, i, j, kk) * p.ivdc_kappa + 0.0) + a.diffKr;
      const double maskUp = G3(maskC, i, j, kk - 1) * G3(maskC, i, j, kk);
      dfr = -kap * maskUp * rA * f.recip_drC[kk - 1] * (T3(i, j, kk) - T3(i, j, kk - 1)) * p.rkSign;
    }
    return fv + dfr;
  };
  const long q3 = MG_I3(d, i, j, k, t);
  const double Tk = T[q3];
  const double uT0 = G3(uVel, i, j, k) * (G2(dyG, i, j) * drF * G3(hFacW, i, j, k));
  const double uT1 = G3(uVel, i + 1, j, k) * (G2(dyG, i + 1, j) * drF * G3(hFacW, i + 1, j, k));
  const double vT0 = G3(vVel, i, j, k) * (G2(dxG, i, j) * drF * G3(hFacS, i, j, k));
  const double vT1 = G3(vVel, i, j + 1, k) * (G2(dxG, i, j + 1) * drF * G3(hFacS, i, j + 1, k));
  const double rTrans = rtrans(k), rTransKp = rtrans(k + 1);
  const double fVerUp = fvert(k, rTrans), fVerDn = fvert(k + 1, rTransKp);
  const double fZi = fzon(i), fZe = fzon(i + 1);
  const double fMi = fmer(j), fMn = fmer(j + 1);
  const double g0 = a.multiDim ? f.gAdv[q3] : 0.0;
  double gT = g0 - f.recip_hFacC[q3] * f.recip_drF[k - 1] * recip_rA *
                       ((fZe - fZi) * maskInC + (fMn - fMi) * maskInC + (fVerDn - fVerUp) * p.rkSign -
                        Tk * ((uT1 - uT0) * advFac + (vT1 - vT0) * advFac + (rTransKp - rTrans) * rAdvFac) * maskInC);
  double gtForc = 0.0;
  if (a.forcing && a.sfc && k == 1) gtForc = gtForc + a.sfc[q] * f.recip_drF[0] * f.recip_hFacC[q3];
  gT = gT + gtForc;
  if (a.useAB) {   // ADAMS_BASHFORTH2(k)
    const double ab = abFac * (gT - a.gNm1[q3]);
    a.gNm1[q3] = gT;
    gT = gT + ab;
  }
  // TIMESTEP_TRACER
  const double v = Tk + p.deltaTtracer * gT;
  if (p.implicitDiffusion) f.gTscr[q3] = v;
  else a.trNext[q3] = v;   // CYCLE_TRACER directly
#undef T3
#undef G2
#undef G3
}

// GAD_IMPLICIT_R (implicitDiffusion) + SOLVE_TRIDIAGONAL (Thomas) + CYCLE_TRACER,
// one thread per interior column; writes the new tracer into its other buffer.
__global__ void __launch_bounds__(256) k_tracer_impl(Dims d, Params p, Fields f, TracerArgs a) {
  MG_PLANE(1, d.sNx, 1, d.sNy, tz)
  const int t = d.t0 + tz;
  if (i > d.sNx || j > d.sNy) return;
  const int Nr = d.Nr;
#define G3(a_, ii, jj, kk) f.a_[MG_I3(d, ii, jj, kk, t)]
  double cpPrev = 0.0, ypPrev = 0.0;
  for (int k = 1; k <= Nr; k++) {
    const long q3 = MG_I3(d, i, j, k, t);
    const double rh = f.recip_hFacC[q3], rdrF = f.recip_drF[k - 1];
    double sub = 0.0, sup = 0.0;
    if (k >= 2)
      sub = -(p.deltaTtracer * G3(maskC, i, j, k - 1) * rh * rdrF *
              ((G3(IVDConvCount, i, j, k) * p.ivdc_kappa + 0.0) + a.diffKr) * f.recip_drC[k - 1]);
    if (k <= Nr - 1)
      sup = -(p.deltaTtracer * G3(maskC, i, j, k + 1) * rh * rdrF *
              ((G3(IVDConvCount, i, j, k + 1) * p.ivdc_kappa + 0.0) + a.diffKr) * f.recip_drC[k]);
    const double diag = 1.0 - (sub + sup);
    const double y = f.gTscr[q3];
    double cp, yp;
    if (k == 1) {
      if (diag != 0.0) { const double rec = 1.0 / diag; cp = sup * rec; yp = y * rec; }
      else { cp = 0.0; yp = 0.0; }
    } else {
      const double tmp = diag - sub * cpPrev;
      if (tmp != 0.0) { const double rec = 1.0 / tmp; cp = sup * rec; yp = (y - sub * ypPrev) * rec; }
      else { cp = 0.0; yp = 0.0; }
    }
    f.gTscr[q3] = yp;
    f.cpScr[q3] = cp;
    cpPrev = cp; ypPrev = yp;
  }
  double below = 0.0;
  for (int k = Nr; k >= 1; k--) {
    const long q3 = MG_I3(d, i, j, k, t);
    const double v = (k == Nr) ? f.gTscr[q3] : f.gTscr[q3] - f.cpScr[q3] * below;
    a.trNext[q3] = v;
    below = v;
  }
#undef G3
}

hipError_t launch_oceanic_phys(const Dims &d, const Params &p, const Fields &f, hipStream_t s) {
  hipLaunchKernelGGL(k_oceanic_phys, dim3(mg_plane_blocks(d.nx, d.ny, d.nT)), dim3(MG_PLANE_THREADS), 0, s, d, p, f);
  return hipGetLastError();
}

hipError_t launch_tracer_step(const Dims &d, const Params &p, const Fields &f, const TracerArgs &a, const int *iterPtr,
                              hipStream_t s) {
  const dim3 blk(MG_PLANE_THREADS), grd(mg_plane_blocks(d.sNx, d.sNy, d.nT * d.Nr));
  if (a.multiDim) {
    const dim3 fgrd(mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr));
    hipLaunchKernelGGL(k_adv_x, fgrd, blk, 0, s, d, f, a);
    hipLaunchKernelGGL(k_adv_y, grd, blk, 0, s, d, f, a);
    hipLaunchKernelGGL(k_adv_r, grd, blk, 0, s, d, p, f, a);
  }
  hipLaunchKernelGGL(k_tracer_rhs, grd, blk, 0, s, d, p, f, a, iterPtr);
  if (p.implicitDiffusion) {
    const dim3 cgrd(mg_plane_blocks(d.sNx, d.sNy, d.nT));
    hipLaunchKernelGGL(k_tracer_impl, cgrd, blk, 0, s, d, p, f, a);
  }
  return hipGetLastError();
}

}  // namespace mgcm
