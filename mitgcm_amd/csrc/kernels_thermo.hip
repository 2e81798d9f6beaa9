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
#include "phys.h"

namespace mgcm {

// DO_OCEANIC_PHYS (phys.h: oceanic_phys_point), one thread per (i,j,k) of the full halo range
__global__ void __launch_bounds__(256) k_oceanic_phys(Dims d, Params p, Fields f, const int *iterPtr) {
  MG_PLANE(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  oceanic_phys_point(d, p, f, iterPtr, i, j, k, t);
}

// k_oceanic_phys with 16-byte accesses: a thread takes two consecutive points of a level's
// full-halo plane (contiguous in memory: i fastest over the whole nx, then j), so every load
// and store of levels k >= 2 is one double2 per lane instead of one double -- the stream
// kernels' 8-B-lane rate (3.3-4.9 TB/s) against the 16-B copy rate (MI355X_MICROARCH.md).
// Same per-point arithmetic (find_rho, the sigmaR / IVDC expressions of oceanic_phys_point);
// the surface level keeps oceanic_phys_point itself (forcing, FREEZE_SURFACE).  Launched where
// n2 is even and the fields are 16-B aligned (launch_oceanic_phys).
__global__ void __launch_bounds__(256) k_oceanic_phys2(Dims d, Params p, Fields f, const int *iterPtr) {
  const int h2 = (int)(d.n2 >> 1), nb = (h2 + 255) / 256, lb = mg_xcd_block();
  const int z = lb / nb, pr = (lb % nb) * 256 + (int)threadIdx.x;
  if (pr >= h2) return;
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  const long q2 = 2L * pr;   // 2-D offset inside the tile
  if (k == 1) {
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const int ii = (int)((q2 + e) % d.nx) + 1 - d.OLx, jj = (int)((q2 + e) / d.nx) + 1 - d.OLy;
      oceanic_phys_point(d, p, f, iterPtr, ii, jj, 1, t);
    }
    return;
  }
  const long q3 = (long)t * d.n3 + (long)(k - 1) * d.n2 + q2, q3u = q3 - d.n2;
  typedef __attribute__((ext_vector_type(2))) double d2;
  auto ld2 = [](const double *a, long q) { return *reinterpret_cast<const d2 *>(a + q); };
  auto st2 = [](double *a, long q, double x, double y) { d2 v; v.x = x; v.y = y; *reinterpret_cast<d2 *>(a + q) = v; };
  const d2 th = ld2(f.theta, q3), sa = ld2(f.salt, q3);
  const bool calcConvect = p.ivdc_kappa != 0.0, sig = calcConvect || p.useGMRedi;
  d2 thU = th, saU = sa, mC = th, mCu = th;
  if (sig) { thU = ld2(f.theta, q3u); saU = ld2(f.salt, q3u); mC = ld2(f.maskC, q3); mCu = ld2(f.maskC, q3u); }
  auto clampU = [&](double v) { return (k - 1 == 1 && p.allowFreezing && v < -1.9) ? -1.9 : v; };
  double rho[2], conv[2] = {0.0, 0.0}, sigmaR[2] = {0.0, 0.0};
#pragma unroll
  for (int e = 0; e < 2; e++) {
    const double tk = e ? th.y : th.x, sk = e ? sa.y : sa.x;
    rho[e] = find_rho(p, f, k, q3 + e, tk, sk);
    if (sig) {
      const double rhoKm1 = find_rho(p, f, k, q3 + e, clampU(e ? thU.y : thU.x), e ? saU.y : saU.x);
      sigmaR[e] = (e ? mC.y : mC.x) * (e ? mCu.y : mCu.x) * f.recip_drC[k - 1] * p.rkSign * (rho[e] - rhoKm1);
      if (calcConvect) conv[e] = (-sigmaR[e] * p.gravitySign > 0.0) ? 1.0 : 0.0;
    }
  }
  st2(f.rhoInSitu, q3, rho[0], rho[1]);
  st2(f.IVDConvCount, q3, conv[0], conv[1]);
  if (p.useGMRedi) st2(f.sigmaR, q3, sigmaR[0], sigmaR[1]);
}

// GMREDI_CALC_TENSOR (pkg/gmredi/gmredi_calc_tensor.F:231-790; skew flux, GM_ExtraDiag
// = F, all isoFac/bolFac = 1) with GMREDI_SLOPE_LIMIT's gkw91 taper
// (gmredi_slope_limit.F:280-370), one thread per (i,j,k) on i,j = 2-OL..sN+OL-1.
// sigmaX/Y (GRAD_SIGMA, grad_sigma.F:80-101) are recomputed from rhoInSitu.
__device__ __forceinline__ void gm_slope_gkw91(const Params &p, double dSx, double dSy, double dSr, double &SlopeX,
                                               double &SlopeY, double &SlopeSqr, double &taper) {
  const double GM_bigSlope = 1.0e+02, maxSlopeSqr = p.GM_maxSlope * p.GM_maxSlope;
  if (dSr != 0.0 && dSr <= p.GM_Small_Number) dSr = p.GM_Small_Number;
  if (dSr == 0.0) {
    SlopeX = dSx != 0.0 ? copysign(GM_bigSlope, dSx) : 0.0;
    SlopeY = dSy != 0.0 ? copysign(GM_bigSlope, dSy) : 0.0;
  } else {
    const double dRdSigmaLtd = 1.0 / dSr;
    SlopeX = dSx * dRdSigmaLtd;
    SlopeY = dSy * dRdSigmaLtd;
  }
  SlopeSqr = SlopeX * SlopeX + SlopeY * SlopeY;
  taper = 1.0;
  if (SlopeSqr >= p.GM_slopeSqCutoff) { SlopeSqr = p.GM_slopeSqCutoff; taper = 0.0; }
  if (SlopeSqr == 0.0) taper = 1.0;
  else if (SlopeSqr > maxSlopeSqr && SlopeSqr < p.GM_slopeSqCutoff) taper = maxSlopeSqr / SlopeSqr;
}

__device__ __forceinline__ void gm_tensor_body(const Dims &d, const Params &p, const Fields &f, int lb) {
  MG_PLANE_LB(2 - d.OLx, d.nx - 2, 2 - d.OLy, d.ny - 2, z, lb)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  const int Nr = d.Nr;
  auto rho = [&](int ii, int jj, int kk) { return f.rhoInSitu[MG_I3(d, ii, jj, kk, t)]; };
  auto sX = [&](int ii, int jj, int kk) {
    return f.maskW[MG_I3(d, ii, jj, kk, t)] * f.recip_dxC[MG_I2(d, ii, jj, t)] * (rho(ii, jj, kk) - rho(ii - 1, jj, kk));
  };
  auto sY = [&](int ii, int jj, int kk) {
    return f.maskS[MG_I3(d, ii, jj, kk, t)] * f.recip_dyC[MG_I2(d, ii, jj, t)] * (rho(ii, jj, kk) - rho(ii, jj - 1, kk));
  };
  auto sR = [&](int ii, int jj, int kk) { return f.sigmaR[MG_I3(d, ii, jj, kk, t)]; };
  const double op25 = 0.25, op5 = 0.5, gs = p.gravitySign;
  const long q3 = MG_I3(d, i, j, k, t);
  const double isopycK = p.GM_isopycK * (1.0 + 1.0) * op5, bolus_K = p.GM_background_K * (1.0 + 1.0) * op5;
  double SlopeX, SlopeY, SlopeSqr, taper;
  // Kwx, Kwy, Kwz (W points, k >= 2; k = 1 stays 0)
  double kwx = 0.0, kwy = 0.0, kwz = 0.0;
  if (k >= 2) {
    const double maskFk = f.maskC[MG_I3(d, i, j, k - 1, t)] * f.maskC[q3];
    const double dSx = op25 * (sX(i + 1, j, k - 1) + sX(i, j, k - 1) + sX(i + 1, j, k) + sX(i, j, k)) * maskFk;
    const double dSy = op25 * (sY(i, j + 1, k - 1) + sY(i, j, k - 1) + sY(i, j + 1, k) + sY(i, j, k)) * maskFk;
    gm_slope_gkw91(p, dSx, dSy, gs * sR(i, j, k), SlopeX, SlopeY, SlopeSqr, taper);
    kwx = -gs * SlopeX * taper;
    kwy = -gs * SlopeY * taper;
    kwz = SlopeSqr * taper;
  }
  const double Kgm_tmp = isopycK * 1.0 + p.GM_skewflx * bolus_K * 1.0;
  f.Kwx[q3] = Kgm_tmp * kwx;
  f.Kwy[q3] = Kgm_tmp * kwy;
  f.Kwz[q3] = (isopycK * 1.0) * kwz;
  const int kp1 = k + 1 < Nr ? k + 1 : Nr;
  const double maskp1 = k >= Nr ? 0.0 : 1.0;
  {  // Kux (U points)
    const double mW = f.maskW[q3];
    const double dSx = sX(i, j, k) * mW;
    const double dSy = op25 * (sY(i - 1, j + 1, k) + sY(i, j + 1, k) + sY(i - 1, j, k) + sY(i, j, k)) * mW;
    const double dSr = op25 * (sR(i - 1, j, k) + sR(i, j, k) + (sR(i - 1, j, kp1) + sR(i, j, kp1)) * maskp1) * mW * gs;
    gm_slope_gkw91(p, dSx, dSy, dSr, SlopeX, SlopeY, SlopeSqr, taper);
    f.Kux[q3] = fmax((p.GM_isopycK * 1.0 * op5 * (1.0 + 1.0)) * taper, p.GM_Kmin_horiz);
    if (p.GM_ExtraDiag)   // GM_EXTRA_DIAGONAL Kuz (gmredi_calc_tensor.F:808-850)
      f.Kuz[q3] = -gs * (p.GM_isopycK * 1.0 * op5 * (1.0 + 1.0) - p.GM_skewflx * p.GM_background_K * 1.0 * op5 * (1.0 + 1.0)) *
                  SlopeX * taper;
  }
  {  // Kvy (V points)
    const double mS = f.maskS[q3];
    const double dSx = op25 * (sX(i, j, k) + sX(i + 1, j, k) + sX(i, j - 1, k) + sX(i + 1, j - 1, k)) * mS;
    const double dSy = sY(i, j, k) * mS;
    const double dSr = op25 * (sR(i, j - 1, k) + sR(i, j, k) + (sR(i, j - 1, kp1) + sR(i, j, kp1)) * maskp1) * mS * gs;
    gm_slope_gkw91(p, dSx, dSy, dSr, SlopeX, SlopeY, SlopeSqr, taper);
    f.Kvy[q3] = fmax((p.GM_isopycK * 1.0 * op5 * (1.0 + 1.0)) * taper, p.GM_Kmin_horiz);
    if (p.GM_ExtraDiag)   // Kvz (gmredi_calc_tensor.F:1053-1090)
      f.Kvz[q3] = -gs * (p.GM_isopycK * 1.0 * op5 * (1.0 + 1.0) - p.GM_skewflx * p.GM_background_K * 1.0 * op5 * (1.0 + 1.0)) *
                  SlopeY * taper;
  }
  if (p.GM_AdvForm) {
    // GMREDI_CALC_PSI_B (gmredi_calc_psi_b.F:86-212) + GMREDI_SLOPE_PSI gkw91
    // (gmredi_slope_psi.F:196-290): bolus stream-function at the top face of level k >= 2
    double psx = 0.0, psy = 0.0;
    if (k >= 2) {
      const double halfRL = 0.5, halfSign = halfRL * gs, half_K = p.GM_background_K * (1.0 + 1.0) * op25;
      const double slopeCutoff = sqrt(p.GM_slopeSqCutoff), loc_maxSlope = p.GM_maxSlope * 1.0;
      const double maxSlopeSqr = loc_maxSlope * loc_maxSlope;
      auto psi = [&](double Slope, double dSdr) {
        if (dSdr <= p.GM_Small_Number) dSdr = p.GM_Small_Number;
        Slope = Slope / dSdr;
        double tp = 1.0;
        if (fabs(Slope) >= slopeCutoff) { Slope = copysign(slopeCutoff, Slope); tp = 0.0; }
        const double Smod = fabs(Slope);
        if (Smod > loc_maxSlope && Smod < slopeCutoff) tp = maxSlopeSqr / (Slope * Slope + p.GM_Small_Number);
        return Slope * tp * (half_K * (1.0 + 1.0));
      };
      const double mkW = f.maskW[MG_I3(d, i, j, k - 1, t)] * f.maskW[q3];
      psx = psi((sX(i, j, k - 1) + sX(i, j, k)) * halfRL * mkW, (sR(i - 1, j, k) + sR(i, j, k)) * halfSign * mkW);
      const double mkS = f.maskS[MG_I3(d, i, j, k - 1, t)] * f.maskS[q3];
      psy = psi((sY(i, j, k - 1) + sY(i, j, k)) * halfRL * mkS, (sR(i, j - 1, k) + sR(i, j, k)) * halfSign * mkS);
    }
    f.GM_PsiX[q3] = psx;
    f.GM_PsiY[q3] = psy;
  }
}
__global__ void __launch_bounds__(256) k_gm_tensor(Dims d, Params p, Fields f) { gm_tensor_body(d, p, f, mg_xcd_block()); }

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
// face flux between cells m1 (upstream for positive transport) and p0; lim = 0 is
// GAD_DST3_ADV_X/Y (gad_dst3_adv_x.F:71-118, not OLD_DST3_FORMULATION): no limiter
__device__ __forceinline__ double dst3fl_h(double uTr, double cfl, double tm2, double tm1, double t0, double tp1,
                                           double mWm1, double mW0, double mWp1, int lim = 1) {
  const double oneSixth = 1.0 / 6.0;
  const double Rjp = (tp1 - t0) * mWp1, Rj = (t0 - tm1) * mW0, Rjm = (tm1 - tm2) * mWm1;
  const double d0 = (2.0 - cfl) * (1.0 - cfl) * oneSixth, d1 = (1.0 - cfl * cfl) * oneSixth;
  if (!lim)
    return 0.5 * (uTr + fabs(uTr)) * (tm1 + (d0 * Rj + d1 * Rjm)) + 0.5 * (uTr - fabs(uTr)) * (t0 - (d0 * Rj + d1 * Rjp));
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
                      f.maskW[MG_I3(d, ii + 1, j, k, t)], a.limiter);
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
                    f.maskS[MG_I3(d, i, jj + 1, k, t)], a.limiter);
  };
  const long q = MG_I2(d, i, j, t);
  f.advScr2[q3] = L1[q3] - dT * f.recip_hFacC[q3] * f.recip_drF[k - 1] * f.recip_rA[q] *
                               (afy(j + 1) - afy(j) - a.tr[q3] * (vTr(j + 1) - vTr(j))) * f.maskInC[q];
}

// vertical pass + advective tendency (gad_advection.F k = Nr..1 loop) on the horizontally
// advected tracer L (and, GAD_MULTIDIM_COMPRESSIBLE, the local volume V, :1036-1057):
// gAdv = (loc - T)/dT, or (tmpTrac - T*vol)/(rA drF hFac dT) in the compressible form
template <bool COMP>
__global__ void __launch_bounds__(256) k_adv_r(Dims d, Params p, Fields f, TracerArgs a, const double *__restrict__ L2,
                                               const double *__restrict__ V) {
  MG_PLANE(1, d.sNx, 1, d.sNy, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  if (i > d.sNx || j > d.sNy) return;
  const int Nr = d.Nr;
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
    const double rT = rtr(kk);
    if (!a.limiter)   // GAD_DST3_ADV_R (gad_dst3_adv_r.F:70-119)
      return 0.5 * (rT + fabs(rT)) * (LT(kk) + (d0 * Rj + d1 * Rjp)) + 0.5 * (rT - fabs(rT)) * (LT(km1) - (d0 * Rj + d1 * Rjm));
    const double psiP = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjm), cfl);
    const double psiM = dst3fl_limit(d0, d1, dst3fl_theta(Rj, Rjp), cfl);
    return 0.5 * (rT + fabs(rT)) * (LT(kk) + psiM * Rj) + 0.5 * (rT - fabs(rT)) * (LT(km1) - psiP * Rj);
  };
  const double kp1Msk = (k == Nr) ? 0.0 : 1.0;
  const double rTrans = rtr(k), rTransKp = kp1Msk * rtr(k + 1);
  const double fUp = fver(k), fDn = fver(k + 1);
  if (COMP) {
    const double tmpTrac = LT(k) * V[q3] - dT * (fDn - fUp) * p.rkSign * f.maskInC[q];
    const double lv = V[q3] - dT * (rTransKp - rTrans) * p.rkSign * f.maskInC[q];
    f.gAdv[q3] = (tmpTrac - a.tr[q3] * lv) * f.recip_rA[q] * f.recip_drF[k - 1] * f.recip_hFacC[q3] / dT;
  } else {
    const double lt = LT(k) - dT * f.recip_hFacC[q3] * f.recip_drF[k - 1] * f.recip_rA[q] *
                                  (fDn - fUp - a.tr[q3] * (rTransKp - rTrans)) * p.rkSign * f.maskInC[q];
    f.gAdv[q3] = (lt - a.tr[q3]) / dT;
  }
#undef MC
#undef LT
}

// ---------------------------------------------------------------------------
// GAD_ADVECTION in its general form (gad_advection.F:292-811): cube tiles (3 passes whose
// direction and overlap-only / interior-only updates depend on the tile's face, :339-367,
// with FILL_CS_CORNER_TR_RL around the overlap-only fluxes and FILL_CS_CORNER_UV_RS on the
// masks) and/or GAD_MULTIDIM_COMPRESSIBLE (the local volume carried through the passes).
// The passes run as explicit steps over the whole slab: loc (advScr1) and vol (advScr2)
// are updated in place, the face fluxes of a pass go to gTscr (free until k_tracer_rhs).
struct AdvCfg { bool ov, in, cx, cy; };
__device__ __forceinline__ AdvCfg adv_cfg(bool cube, int face, int ipass) {
  AdvCfg c{false, false, false, false};
  if (cube) {
    if (ipass == 1) {
      c.ov = face % 3 == 0; c.in = face % 3 != 0;
      c.cx = face == 6 || face == 1 || face == 2; c.cy = face == 3 || face == 4 || face == 5;
    } else if (ipass == 2) {
      c.ov = face % 3 == 2; c.in = face % 3 == 1;
      c.cx = face == 2 || face == 3 || face == 4; c.cy = face == 5 || face == 6 || face == 1;
    } else {
      c.in = true;
      c.cx = face == 5 || face == 6; c.cy = face == 2 || face == 3;
    }
  } else {
    c.cx = ipass % 2 == 1; c.cy = !c.cx;
  }
  return c;
}
// maskLocW / maskLocS after FILL_CS_CORNER_UV_RS(withSigns = .FALSE.): corner halo points
// take the other component's mask at the rotated position (the sources are never corners)
__device__ __forceinline__ double mask_loc(const Dims &d, const Fields &f, bool cube, int edges, bool isW, int i, int j,
                                           int k, int t) {
  const int sNx = d.sNx, sNy = d.sNy;
  const bool N = edges & 1, S = edges & 2, E = edges & 4, W = edges & 8;
  if (cube) {
    const double *other = isW ? f.maskS : f.maskW;
    int si = 0, sj = 0;
    bool hit = false;
    if (i <= 0 && j <= 0 && W && S) { hit = true; if (isW) { si = j; sj = 2 - i; } else { si = 2 - j; sj = i; } }
    else if (i > sNx && j <= 0 && E && S) {
      if (isW) { if (i >= sNx + 2) { hit = true; si = sNx + 1 - j; sj = i - sNx; } }
      else { hit = true; si = sNx + j; sj = 1 + sNx - i; }
    } else if (i <= 0 && j > sNy && W && N) {
      if (isW) { hit = true; si = 1 + sNy - j; sj = sNy + i; }
      else if (j >= sNy + 2) { hit = true; si = j - sNy; sj = sNy + 1 - i; }
    } else if (i > sNx && j > sNy && E && N) {
      if (isW) { if (i >= sNx + 2) { hit = true; si = sNx + j - sNy; sj = sNy + sNx + 2 - i; } }
      else if (j >= sNy + 2) { hit = true; si = sNx + sNy + 2 - j; sj = sNy + i - sNx; }
    }
    if (hit) return other[MG_I3(d, si, sj, k, t)];
  }
  return (isW ? f.maskW : f.maskS)[MG_I3(d, i, j, k, t)];
}

__global__ void __launch_bounds__(256) k_advg_init(Dims d, Fields f, TracerArgs a, int comp) {
  MG_PLANE(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  if (i > d.sNx + d.OLx || j > d.sNy + d.OLy) return;
  const long q3 = MG_I3(d, i, j, k, t);
  f.advScr1[q3] = a.tr[q3];
  if (comp)
    f.advScr2[q3] = f.rA[MG_I2(d, i, j, t)] * f.drF[k - 1] * f.hFacC[q3] + (1.0 - f.maskC[q3]);
}

// FILL_CS_CORNER_TR_RL(dir) on loc for the tiles whose pass calls it at this stage:
// stage 0 X-before (X flux, overlap-only, N/S edge), 1 X-after (+ ipass = 1), 2 Y-before
// (Y flux, overlap-only, E/W edge), 3 Y-after (+ ipass = 1); one thread per corner point
__global__ void __launch_bounds__(256) k_advg_fill(Dims d, Fields f, int ipass, int stage) {
  const int OLx = d.OLx, OLy = d.OLy, per = 4 * OLx * OLy;
  const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long)per * d.nT * d.Nr) return;
  const int c = (int)(g % per), z = (int)(g / per);
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  const int face = f.tileFace[t], edges = f.tileEdge[t];
  const bool N = edges & 1, S = edges & 2, E = edges & 4, W = edges & 8;
  const AdvCfg cf = adv_cfg(true, face, ipass);
  bool run;
  if (stage < 2) run = cf.cx && cf.ov && (N || S) && (stage == 0 || ipass == 1);
  else run = cf.cy && cf.ov && (E || W) && (stage == 2 || ipass == 1);
  if (!run) return;
  const int dir = (stage == 0 || stage == 3) ? 1 : 2;
  const int corner = c / (OLx * OLy), ii = c % OLx + 1, jj = (c / OLx) % OLy + 1;
  const int sNx = d.sNx, sNy = d.sNy;
  int di, dj, si, sj;
  if (corner == 0) { if (!(W && S)) return; di = 1 - ii; dj = 1 - jj; if (dir == 1) { si = 1 - jj; sj = ii; } else { si = jj; sj = 1 - ii; } }
  else if (corner == 1) { if (!(E && S)) return; di = sNx + ii; dj = 1 - jj; if (dir == 1) { si = sNx + jj; sj = ii; } else { si = sNx + 1 - jj; sj = 1 - ii; } }
  else if (corner == 2) { if (!(W && N)) return; di = 1 - ii; dj = sNy + jj; if (dir == 1) { si = 1 - jj; sj = sNy + 1 - ii; } else { si = jj; sj = sNy + ii; } }
  else { if (!(E && N)) return; di = sNx + ii; dj = sNy + jj; if (dir == 1) { si = sNx + jj; sj = sNy + 1 - ii; } else { si = sNx + 1 - jj; sj = sNy + ii; } }
  f.advScr1[MG_I3(d, di, dj, k, t)] = f.advScr1[MG_I3(d, si, sj, k, t)];
}

// the X (ydir = 0) or Y (1) DST3FL face fluxes of a pass into gTscr, on the tiles that
// compute them (GAD_DST3FL_ADV_X over i = 3-OLx..sNx+OLx-1, _Y over j = 3-OLy..sNy+OLy-1)
__global__ void __launch_bounds__(256) k_advg_flux(Dims d, Fields f, TracerArgs a, int ipass, int ydir, int cube) {
  MG_PLANE(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  if (i > d.sNx + d.OLx || j > d.sNy + d.OLy) return;
  const int face = cube ? f.tileFace[t] : 0, edges = cube ? f.tileEdge[t] : 0;
  const bool N = edges & 1, S = edges & 2, E = edges & 4, W = edges & 8;
  const AdvCfg cf = adv_cfg(cube, face, ipass);
  if (ydir ? !(cf.cy && (!cf.ov || E || W)) : !(cf.cx && (!cf.ov || N || S))) return;
  const double *__restrict__ Lc = f.advScr1;
  const long q3 = MG_I3(d, i, j, k, t);
  const double dT = a.dT, drF = f.drF[k - 1];
  double af = 0.0;
  if (!ydir && i >= 3 - d.OLx && i <= d.sNx + d.OLx - 1) {
    const double uTr = f.uVel[q3] * (f.dyG[MG_I2(d, i, j, t)] * drF * f.hFacW[q3]);
    const double cfl = fabs(f.uVel[q3] * dT * f.recip_dxC[MG_I2(d, i, j, t)]);
    af = dst3fl_h(uTr, cfl, Lc[MG_I3(d, i - 2, j, k, t)], Lc[MG_I3(d, i - 1, j, k, t)], Lc[q3], Lc[MG_I3(d, i + 1, j, k, t)],
                  mask_loc(d, f, cube, edges, true, i - 1, j, k, t), mask_loc(d, f, cube, edges, true, i, j, k, t),
                  mask_loc(d, f, cube, edges, true, i + 1, j, k, t), a.limiter);
  } else if (ydir && j >= 3 - d.OLy && j <= d.sNy + d.OLy - 1) {
    const double vTr = f.vVel[q3] * (f.dxG[MG_I2(d, i, j, t)] * drF * f.hFacS[q3]);
    const double cfl = fabs(f.vVel[q3] * dT * f.recip_dyC[MG_I2(d, i, j, t)]);
    af = dst3fl_h(vTr, cfl, Lc[MG_I3(d, i, j - 2, k, t)], Lc[MG_I3(d, i, j - 1, k, t)], Lc[q3], Lc[MG_I3(d, i, j + 1, k, t)],
                  mask_loc(d, f, cube, edges, false, i, j - 1, k, t), mask_loc(d, f, cube, edges, false, i, j, k, t),
                  mask_loc(d, f, cube, edges, false, i, j + 1, k, t), a.limiter);
  }
  f.gTscr[q3] = af;
}

// the update of loc (and vol) by the X / Y flux divergence on the pass's update region
__global__ void __launch_bounds__(256) k_advg_upd(Dims d, Fields f, TracerArgs a, int ipass, int ydir, int cube, int comp) {
  MG_PLANE(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  if (i > d.sNx + d.OLx || j > d.sNy + d.OLy) return;
  const int face = cube ? f.tileFace[t] : 0, edges = cube ? f.tileEdge[t] : 0;
  const bool N = edges & 1, S = edges & 2, E = edges & 4, W = edges & 8;
  const AdvCfg cf = adv_cfg(cube, face, ipass);
  const int sNx = d.sNx, sNy = d.sNy, OLx = d.OLx, OLy = d.OLy;
  bool upd = false;
  if (!ydir) {
    if (!cf.cx) return;
    if (cf.ov) {
      const int iMin = W ? 1 : 2 - OLx, iMax = E ? sNx : sNx + OLx - 1;
      upd = i >= iMin && i <= iMax && ((S && j <= 0) || (N && j >= sNy + 1));
    } else {
      const int jMin = (cf.in && S) ? 1 : 1 - OLy, jMax = (cf.in && N) ? sNy : sNy + OLy;
      upd = j >= jMin && j <= jMax && i >= 2 - OLx && i <= sNx + OLx - 1;
    }
  } else {
    if (!cf.cy) return;
    if (cf.ov) {
      const int jMin = S ? 1 : 2 - OLy, jMax = N ? sNy : sNy + OLy - 1;
      upd = j >= jMin && j <= jMax && ((W && i <= 0) || (E && i >= sNx + 1));
    } else {
      const int iMin = (cf.in && W) ? 1 : 1 - OLx, iMax = (cf.in && E) ? sNx : sNx + OLx;
      upd = i >= iMin && i <= iMax && j >= 2 - OLy && j <= sNy + OLy - 1;
    }
  }
  if (!upd) return;
  const long q3 = MG_I3(d, i, j, k, t), q = MG_I2(d, i, j, t);
  const double dT = a.dT, drF = f.drF[k - 1];
  const long q3n = ydir ? MG_I3(d, i, j + 1, k, t) : MG_I3(d, i + 1, j, k, t);
  const double dF = f.gTscr[q3n] - f.gTscr[q3];
  double dU;
  if (ydir) dU = f.vVel[q3n] * (f.dxG[MG_I2(d, i, j + 1, t)] * drF * f.hFacS[q3n]) - f.vVel[q3] * (f.dxG[q] * drF * f.hFacS[q3]);
  else dU = f.uVel[q3n] * (f.dyG[MG_I2(d, i + 1, j, t)] * drF * f.hFacW[q3n]) - f.uVel[q3] * (f.dyG[q] * drF * f.hFacW[q3]);
  if (comp) {
    const double tmpTrac = f.advScr1[q3] * f.advScr2[q3] - dT * dF * f.maskInC[q];
    const double vol = f.advScr2[q3] - dT * dU * f.maskInC[q];
    f.advScr2[q3] = vol;
    f.advScr1[q3] = tmpTrac / vol;
  } else {
    f.advScr1[q3] = f.advScr1[q3] - dT * f.recip_hFacC[q3] * f.recip_drF[k - 1] * f.recip_rA[q] *
                                        (dF - a.tr[q3] * dU) * f.maskInC[q];
  }
}

// tracer_rhs_body with its operands loaded behind the reference's conditions: the form the
// fused 2-D kernels (k_dt_front, k_dt_l2) keep. There the unconditional loads below raise
// the fused kernel from 125 to 196 VGPRs (4 -> 2 waves per SIMD) and C2 measured 1.5 %
// slower (0.2901 against 0.2852 ms/step); capping the kernel at 128 spills
// (profiles/r05/gm_loads/). Same arithmetic, bit-identical results.
template <bool GM>
__device__ __forceinline__ void tracer_rhs_body_br(const Dims &d, const Params &p, const Fields &f, const TracerArgs &a,
                                                const int *iterPtr, int lb) {
  MG_PLANE_LB(1, d.sNx, 1, d.sNy, z, lb)
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
  // uFld, vFld, wFld of thermodynamics.F:252-268: the Eulerian velocity plus, with
  // GM_AdvForm, GMREDI_RESIDUAL_FLOW's bolus velocity (gmredi_residual_flow.F:58-97)
  const bool bolus = GM && p.GM_AdvForm;
  const double flip = -p.gravitySign;
  const int kp1b = k + 1 < Nr ? k + 1 : Nr;
  const double maskp1b = k >= Nr ? 0.0 : 1.0;
  auto uFld = [&](int ii, int jj) {
    double u = G3(uVel, ii, jj, k);
    if (bolus) {
      const double delPsi = G3(GM_PsiX, ii, jj, kp1b) * 1.0 * maskp1b - G3(GM_PsiX, ii, jj, k) * 1.0;
      u = u + delPsi * f.recip_drF[k - 1] * G3(recip_hFacW, ii, jj, k) * 1.0 * flip;
    }
    return u;
  };
  auto vFld = [&](int ii, int jj) {
    double v = G3(vVel, ii, jj, k);
    if (bolus) {
      const double delPsi = G3(GM_PsiY, ii, jj, kp1b) * 1.0 * maskp1b - G3(GM_PsiY, ii, jj, k) * 1.0;
      v = v + delPsi * f.recip_drF[k - 1] * G3(recip_hFacS, ii, jj, k) * 1.0 * flip;
    }
    return v;
  };
  auto wFld = [&](int kk) {
    double w = G3(wVel, i, j, kk);
    if (bolus) {
      const double delPsi = (G2(dyG, i + 1, j) * G3(GM_PsiX, i + 1, j, kk) - G2(dyG, i, j) * G3(GM_PsiX, i, j, kk) +
                             G2(dxG, i, j + 1) * G3(GM_PsiY, i, j + 1, kk) - G2(dxG, i, j) * G3(GM_PsiY, i, j, kk));
      w = w + delPsi * recip_rA * 1.0 * flip;
    }
    return w;
  };
  // GM_EXTRA_DIAGONAL vertical gradient at the west (dir 0) / south (dir 1) face of (ii, jj)
  // (gmredi_xtransport.F:117-146, gmredi_ytransport.F; maskFk = CALC_ADV_FLOW's maskUp)
  auto gm_dTdz = [&](int ii, int jj, int dir) {
    const int km1 = k > 1 ? k - 1 : 1, kp1 = k + 1 < Nr ? k + 1 : Nr;
    const double maskp1 = k >= Nr ? 0.0 : 1.0;
    const int i0 = dir == 0 ? ii - 1 : ii, j0 = dir == 0 ? jj : jj - 1;
    auto mUp = [&](int a, int b) { return k == 1 ? 0.0 : G3(maskC, a, b, k - 1) * G3(maskC, a, b, k); };
    return 0.5 * (+0.5 * f.recip_drC[k - 1] *
                      (mUp(i0, j0) * (T3(i0, j0, km1) - T3(i0, j0, k)) + mUp(ii, jj) * (T3(ii, jj, km1) - T3(ii, jj, k))) +
                  0.5 * f.recip_drC[kp1 - 1] *
                      (G3(maskC, i0, j0, k) * G3(maskC, i0, j0, kp1) * maskp1 * (T3(i0, j0, k) - T3(i0, j0, kp1)) +
                       G3(maskC, ii, jj, k) * G3(maskC, ii, jj, kp1) * maskp1 * (T3(ii, jj, k) - T3(ii, jj, kp1))));
  };
  // west / south face fluxes of the column (fZon, fMer): GAD_C2_ADV_X/Y + GAD_DIFF_X/Y
  auto fzon = [&](int ii) {
    const double xA = G2(dyG, ii, j) * drF * G3(hFacW, ii, j, k);
    double fz = 0.0;
    if (calcAdv) fz = fz + (uFld(ii, j) * xA) * (T3(ii, j, k) + T3(ii - 1, j, k)) * 0.5;
    double df = 0.0;
    if (a.diffKh != 0.0) df = -a.diffKh * xA * G2(recip_dxC, ii, j) * (T3(ii, j, k) - T3(ii - 1, j, k));
    if (GM)   // GMREDI_XTRANSPORT (gmredi_xtransport.F:94-101)
      df = df - xA * G3(Kux, ii, j, k) * G2(recip_dxC, ii, j) * (T3(ii, j, k) - T3(ii - 1, j, k));
    if (GM && p.GM_ExtraDiag) df = df - xA * G3(Kuz, ii, j, k) * gm_dTdz(ii, j, 0);
    return fz + df;
  };
  auto fmer = [&](int jj) {
    const double yA = G2(dxG, i, jj) * drF * G3(hFacS, i, jj, k);
    double fm = 0.0;
    if (calcAdv) fm = fm + (vFld(i, jj) * yA) * (T3(i, jj, k) + T3(i, jj - 1, k)) * 0.5;
    double df = 0.0;
    if (a.diffKh != 0.0) df = -a.diffKh * yA * G2(recip_dyC, i, jj) * (T3(i, jj, k) - T3(i, jj - 1, k));
    if (GM)   // GMREDI_YTRANSPORT
      df = df - yA * G3(Kvy, i, jj, k) * G2(recip_dyC, i, jj) * (T3(i, jj, k) - T3(i, jj - 1, k));
    if (GM && p.GM_ExtraDiag) df = df - yA * G3(Kvz, i, jj, k) * gm_dTdz(i, jj, 1);
    return fm + df;
  };
  // CALC_ADV_FLOW rTrans of level kk (0 at the surface and below the bottom level)
  auto rtrans = [&](int kk) {
    if (kk <= 1 || kk > Nr) return 0.0;
    const double maskUp = G3(maskC, i, j, kk - 1) * G3(maskC, i, j, kk);
    return wFld(kk) * rA * maskUp;
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
      double kap = (G3(IVDConvCount, i, j, kk) * p.ivdc_kappa + 0.0) + a.diffKr;
      if (GM) kap = kap + G3(Kwz, i, j, kk) * maskInC;
      const double maskUp = G3(maskC, i, j, kk - 1) * G3(maskC, i, j, kk);
      dfr = -kap * maskUp * rA * f.recip_drC[kk - 1] * (T3(i, j, kk) - T3(i, j, kk - 1)) * p.rkSign;
    }
    if (GM && kk >= 2 && kk <= Nr) {   // GMREDI_RTRANSPORT (gmredi_rtransport.F:75-130)
      const double dTdx =
          0.5 * (0.5 * (G3(maskW, i + 1, j, kk) * G2(recip_dxC, i + 1, j) * (T3(i + 1, j, kk) - T3(i, j, kk)) +
                        G3(maskW, i, j, kk) * G2(recip_dxC, i, j) * (T3(i, j, kk) - T3(i - 1, j, kk))) +
                 0.5 * (G3(maskW, i + 1, j, kk - 1) * G2(recip_dxC, i + 1, j) * (T3(i + 1, j, kk - 1) - T3(i, j, kk - 1)) +
                        G3(maskW, i, j, kk - 1) * G2(recip_dxC, i, j) * (T3(i, j, kk - 1) - T3(i - 1, j, kk - 1))));
      const double dTdy =
          0.5 * (0.5 * (G3(maskS, i, j + 1, kk) * G2(recip_dyC, i, j + 1) * (T3(i, j + 1, kk) - T3(i, j, kk)) +
                        G3(maskS, i, j, kk) * G2(recip_dyC, i, j) * (T3(i, j, kk) - T3(i, j - 1, kk))) +
                 0.5 * (G3(maskS, i, j + 1, kk - 1) * G2(recip_dyC, i, j + 1) * (T3(i, j + 1, kk - 1) - T3(i, j, kk - 1)) +
                        G3(maskS, i, j, kk - 1) * G2(recip_dyC, i, j) * (T3(i, j, kk - 1) - T3(i, j - 1, kk - 1))));
      const double maskUp = G3(maskC, i, j, kk - 1) * G3(maskC, i, j, kk);
      dfr = dfr - rA * maskInC * (G3(Kwx, i, j, kk) * dTdx + G3(Kwy, i, j, kk) * dTdy) * maskUp;
    }
    return fv + dfr;
  };
  const long q3 = MG_I3(d, i, j, k, t);
  const double Tk = T[q3];
  const double uT0 = uFld(i, j) * (G2(dyG, i, j) * drF * G3(hFacW, i, j, k));
  const double uT1 = uFld(i + 1, j) * (G2(dyG, i + 1, j) * drF * G3(hFacW, i + 1, j, k));
  const double vT0 = vFld(i, j) * (G2(dxG, i, j) * drF * G3(hFacS, i, j, k));
  const double vT1 = vFld(i, j + 1) * (G2(dxG, i, j + 1) * drF * G3(hFacS, i, j + 1, k));
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
  if (!p.tracForcingOutAB) gT = gT + gtForc;   // inside (0) / after (1) AB2: temp_integrate.F:373-410
  if (a.useAB) {   // ADAMS_BASHFORTH2(k)
    const double ab = abFac * (gT - a.gNm1[q3]);
    double gN = gT;
    gT = gT + ab;
    // FREESURF_RESCALE_G of gT and gtNm1 under r* (temp_integrate.F:412-446)
    if (p.nonlinFreeSurf > 0 && p.select_rStar > 0) gN = gN / f.rStarExpC[q];
    a.gNm1[q3] = gN;
  }
  if (p.tracForcingOutAB) gT = gT + gtForc;
  if (p.nonlinFreeSurf > 0 && p.select_rStar > 0) gT = gT / f.rStarExpC[q];
  // TIMESTEP_TRACER
  const double v = Tk + p.deltaTtracer * gT;
  if (p.implicitDiffusion) a.scr[q3] = v;
  else a.trNext[q3] = v;   // CYCLE_TRACER directly
#undef T3
#undef G2
#undef G3
}

// GAD_CALC_RHS + forcing + AB2 + TIMESTEP_TRACER for one interior (i,j,k) point:
// writes gNm1 (AB tracers) and a.scr = tracer + dTtracer*gT (the right-hand side of
// the implicit vertical solve, or the new tracer with explicit vertical diffusion).
// GAD_U3_ADV_X/Y (gad_u3_adv_x.F:70-92, scheme 3) and GAD_C4_ADV_X/Y (gad_c4_adv_x.F:70-93,
// scheme 4) at one face: transport uTr, the tracer at the two cells either side (tm2, tm1 | t0,
// tp1) and maskLocW (= maskW(k) without OBCS, gad_calc_rhs.F:262-268) at the faces i-1, i, i+1
__device__ __forceinline__ double gad_u3c4_face(bool c4, double uTr, double tm2, double tm1, double t0, double tp1,
                                                double mm1, double m0, double mp1) {
  const double oneSixth = 1.0 / 6.0;
  const double Rjp = (tp1 - t0) * mp1, Rj = (t0 - tm1) * m0, Rjm = (tm1 - tm2) * mm1;
  const double Rjjp = Rjp - Rj, Rjjm = Rj - Rjm;
  double v = uTr * (t0 + tm1 - oneSixth * (Rjjp + Rjjm)) * 0.5;
  if (c4) v = v + fabs(uTr) * 0.5 * oneSixth * (Rjjp - Rjjm) * (1.0 - mm1 * mp1);
  else v = v + fabs(uTr) * 0.5 * oneSixth * (Rjjp - Rjjm);
  return v;
}
// GAD_U3_ADV_R (gad_u3_adv_r.F:58-88) / GAD_C4_ADV_R (gad_c4_adv_r.F:58-92) through the top face of
// level k (2 <= k <= Nr): km1 = k-1, km2 = max(1, k-2), kp1 = min(Nr, k+1); U3 masks Rjm at km2,
// C4 at km1 and adds its boundary factor
__device__ __forceinline__ double gad_u3c4_r(bool c4, int k, int Nr, double rTr, double tkm2, double tkm1, double tk,
                                             double tkp1, double mkm2, double mkm1, double mkp1) {
  const double oneSixth = 1.0 / 6.0;
  const double Rjp = (tkp1 - tk) * mkp1, Rj = (tk - tkm1), Rjm = (tkm1 - tkm2) * (c4 ? mkm1 : mkm2);
  const double Rjjp = Rjp - Rj, Rjjm = Rj - Rjm;
  if (c4) {
    const double maskPM = (k <= 2 || k >= Nr) ? 0.0 : 1.0;
    const double maskBound = maskPM * mkm2 * mkp1;
    return mkm1 * (rTr * ((tk + tkm1) * 0.5 - oneSixth * (Rjjm + Rjjp) * 0.5) +
                   fabs(rTr) * oneSixth * (Rjjm - Rjjp) * 0.5 * (1.0 - maskBound));
  }
  return mkm1 * (rTr * ((tk + tkm1) * 0.5 - oneSixth * (Rjjm + Rjjp) * 0.5) + fabs(rTr) * oneSixth * (Rjjm - Rjjp) * 0.5);
}
template <bool GM>
__device__ __forceinline__ void tracer_rhs_body(const Dims &d, const Params &p, const Fields &f, const TracerArgs &a,
                                                const int *iterPtr, int lb) {
  MG_PLANE_LB(1, d.sNx, 1, d.sNy, z, lb)
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
  // uFld, vFld, wFld of thermodynamics.F:252-268: the Eulerian velocity plus, with
  // GM_AdvForm, GMREDI_RESIDUAL_FLOW's bolus velocity (gmredi_residual_flow.F:58-97)
  const bool bolus = GM && p.GM_AdvForm;
  const double flip = -p.gravitySign;
  const int kp1b = k + 1 < Nr ? k + 1 : Nr;
  const double maskp1b = k >= Nr ? 0.0 : 1.0;
  // (every operand below is loaded unconditionally, at clamped levels where the reference's
  // condition would not reach it, and the conditions then select among the values: the same
  // arithmetic, but no load waits behind a branch -- vmcnt counts stores too)
  auto uFld = [&](int ii, int jj) {
    double u = G3(uVel, ii, jj, k);
    const double ps1 = G3(GM_PsiX, ii, jj, kp1b), ps0 = G3(GM_PsiX, ii, jj, k), rdr = f.recip_drF[k - 1];
    const double rh = G3(recip_hFacW, ii, jj, k);
    if (bolus) {
      const double delPsi = ps1 * 1.0 * maskp1b - ps0 * 1.0;
      u = u + delPsi * rdr * rh * 1.0 * flip;
    }
    return u;
  };
  auto vFld = [&](int ii, int jj) {
    double v = G3(vVel, ii, jj, k);
    const double ps1 = G3(GM_PsiY, ii, jj, kp1b), ps0 = G3(GM_PsiY, ii, jj, k), rdr = f.recip_drF[k - 1];
    const double rh = G3(recip_hFacS, ii, jj, k);
    if (bolus) {
      const double delPsi = ps1 * 1.0 * maskp1b - ps0 * 1.0;
      v = v + delPsi * rdr * rh * 1.0 * flip;
    }
    return v;
  };
  auto wFld = [&](int kk) {   // (kk in 1..Nr)
    double w = G3(wVel, i, j, kk);
    const double dyE = G2(dyG, i + 1, j), pxE = G3(GM_PsiX, i + 1, j, kk), dyW = G2(dyG, i, j), pxW = G3(GM_PsiX, i, j, kk);
    const double dxN = G2(dxG, i, j + 1), pyN = G3(GM_PsiY, i, j + 1, kk), dxS = G2(dxG, i, j), pyS = G3(GM_PsiY, i, j, kk);
    if (bolus) {
      const double delPsi = (dyE * pxE - dyW * pxW + dxN * pyN - dxS * pyS);
      w = w + delPsi * recip_rA * 1.0 * flip;
    }
    return w;
  };
  // GM_EXTRA_DIAGONAL vertical gradient at the west (dir 0) / south (dir 1) face of (ii, jj)
  // (gmredi_xtransport.F:117-146, gmredi_ytransport.F; maskFk = CALC_ADV_FLOW's maskUp)
  auto gm_dTdz = [&](int ii, int jj, int dir) {
    const int km1 = k > 1 ? k - 1 : 1, kp1 = k + 1 < Nr ? k + 1 : Nr;
    const double maskp1 = k >= Nr ? 0.0 : 1.0;
    const int i0 = dir == 0 ? ii - 1 : ii, j0 = dir == 0 ? jj : jj - 1;
    auto mUp = [&](int a_, int b_) {
      const double mm = G3(maskC, a_, b_, km1), m0 = G3(maskC, a_, b_, k);
      return k == 1 ? 0.0 : mm * m0;
    };
    const double rdc0 = f.recip_drC[k - 1], rdc1 = f.recip_drC[kp1 - 1];
    return 0.5 * (+0.5 * rdc0 *
                      (mUp(i0, j0) * (T3(i0, j0, km1) - T3(i0, j0, k)) + mUp(ii, jj) * (T3(ii, jj, km1) - T3(ii, jj, k))) +
                  0.5 * rdc1 *
                      (G3(maskC, i0, j0, k) * G3(maskC, i0, j0, kp1) * maskp1 * (T3(i0, j0, k) - T3(i0, j0, kp1)) +
                       G3(maskC, ii, jj, k) * G3(maskC, ii, jj, kp1) * maskp1 * (T3(ii, jj, k) - T3(ii, jj, kp1))));
  };
  // west / south face fluxes of the column (fZon, fMer): GAD_C2_ADV_X/Y + GAD_DIFF_X/Y
  auto fzon = [&](int ii) {
    const double xA = G2(dyG, ii, j) * drF * G3(hFacW, ii, j, k);
    const double uf = uFld(ii, j), t0 = T3(ii, j, k), tw = T3(ii - 1, j, k), rdx = G2(recip_dxC, ii, j);
    const double ku = G3(Kux, ii, j, k), kz = G3(Kuz, ii, j, k);
    const double dz = GM ? gm_dTdz(ii, j, 0) : 0.0;
    double fz = 0.0;
    if (calcAdv && a.scheme == 2) fz = fz + (uf * xA) * (t0 + tw) * 0.5;
    else if (calcAdv)
      fz = fz + gad_u3c4_face(a.scheme == 4, uf * xA, T3(ii - 2, j, k), tw, t0, T3(ii + 1, j, k), G3(maskW, ii - 1, j, k),
                              G3(maskW, ii, j, k), G3(maskW, ii + 1, j, k));
    double df = 0.0;
    if (a.diffKh != 0.0) df = -a.diffKh * xA * rdx * (t0 - tw);
    if (GM)   // GMREDI_XTRANSPORT (gmredi_xtransport.F:94-101)
      df = df - xA * ku * rdx * (t0 - tw);
    if (GM && p.GM_ExtraDiag) df = df - xA * kz * dz;
    return fz + df;
  };
  auto fmer = [&](int jj) {
    const double yA = G2(dxG, i, jj) * drF * G3(hFacS, i, jj, k);
    const double vf = vFld(i, jj), t0 = T3(i, jj, k), ts = T3(i, jj - 1, k), rdy = G2(recip_dyC, i, jj);
    const double kv = G3(Kvy, i, jj, k), kz = G3(Kvz, i, jj, k);
    const double dz = GM ? gm_dTdz(i, jj, 1) : 0.0;
    double fm = 0.0;
    if (calcAdv && a.scheme == 2) fm = fm + (vf * yA) * (t0 + ts) * 0.5;
    else if (calcAdv)
      fm = fm + gad_u3c4_face(a.scheme == 4, vf * yA, T3(i, jj - 2, k), ts, t0, T3(i, jj + 1, k), G3(maskS, i, jj - 1, k),
                              G3(maskS, i, jj, k), G3(maskS, i, jj + 1, k));
    double df = 0.0;
    if (a.diffKh != 0.0) df = -a.diffKh * yA * rdy * (t0 - ts);
    if (GM)   // GMREDI_YTRANSPORT
      df = df - yA * kv * rdy * (t0 - ts);
    if (GM && p.GM_ExtraDiag) df = df - yA * kz * dz;
    return fm + df;
  };
  // CALC_ADV_FLOW rTrans of level kk (0 at the surface and below the bottom level)
  auto rtrans = [&](int kk) {
    const int kc = kk < 2 ? 2 : (kk > Nr ? Nr : kk), kcm = kc > 1 ? kc - 1 : 1;   // (clamped; Nr = 1: 1, 1)
    const double mm = G3(maskC, i, j, kcm), m0 = G3(maskC, i, j, kc);
    const double w = wFld(kc);
    if (kk <= 1 || kk > Nr) return 0.0;
    const double maskUp = mm * m0;
    return w * rA * maskUp;
  };
  // fVerT through the top face of level kk: GAD_C2_ADV_R + vertical diffusive flux
  // (GAD_DIFF_R when diffusion is explicit, 0 with implicitDiffusion)
  auto fvert = [&](int kk, double rTr) {
    const int kc = kk < 2 ? 2 : (kk > Nr ? Nr : kk), kcm = kc > 1 ? kc - 1 : 1;
    const bool in = kk >= 2 && kk <= Nr;
    const double mm = G3(maskC, i, j, kcm), m0 = G3(maskC, i, j, kc);
    const double tk = T3(i, j, kc), tm = T3(i, j, kcm);
    const double ivd = G3(IVDConvCount, i, j, kc), kwz = G3(Kwz, i, j, kc), rdc = f.recip_drC[kcm];
    double fv = 0.0;
    if (in && calcAdv) {
      double wT;
      if (a.scheme == 2) wT = mm * rTr * (tk + tm) * 0.5;
      else {
        const int kp = kc + 1 <= Nr ? kc + 1 : Nr, km2 = kc - 2 >= 1 ? kc - 2 : 1;
        wT = gad_u3c4_r(a.scheme == 4, kc, Nr, rTr, T3(i, j, km2), tm, tk, T3(i, j, kp), G3(maskC, i, j, km2), mm,
                        G3(maskC, i, j, kp));
      }
      fv = fv + wT * maskInC;
    }
    double dfr = 0.0;
    if (!p.implicitDiffusion && in) {
      double kap = (ivd * p.ivdc_kappa + 0.0) + a.diffKr;
      if (GM) kap = kap + kwz * maskInC;
      const double maskUp = mm * m0;
      dfr = -kap * maskUp * rA * rdc * (tk - tm) * p.rkSign;
    }
    if (GM && in) {   // GMREDI_RTRANSPORT (gmredi_rtransport.F:75-130)
      const double dTdx =
          0.5 * (0.5 * (G3(maskW, i + 1, j, kc) * G2(recip_dxC, i + 1, j) * (T3(i + 1, j, kc) - T3(i, j, kc)) +
                        G3(maskW, i, j, kc) * G2(recip_dxC, i, j) * (T3(i, j, kc) - T3(i - 1, j, kc))) +
                 0.5 * (G3(maskW, i + 1, j, kcm) * G2(recip_dxC, i + 1, j) * (T3(i + 1, j, kcm) - T3(i, j, kcm)) +
                        G3(maskW, i, j, kcm) * G2(recip_dxC, i, j) * (T3(i, j, kcm) - T3(i - 1, j, kcm))));
      const double dTdy =
          0.5 * (0.5 * (G3(maskS, i, j + 1, kc) * G2(recip_dyC, i, j + 1) * (T3(i, j + 1, kc) - T3(i, j, kc)) +
                        G3(maskS, i, j, kc) * G2(recip_dyC, i, j) * (T3(i, j, kc) - T3(i, j - 1, kc))) +
                 0.5 * (G3(maskS, i, j + 1, kcm) * G2(recip_dyC, i, j + 1) * (T3(i, j + 1, kcm) - T3(i, j, kcm)) +
                        G3(maskS, i, j, kcm) * G2(recip_dyC, i, j) * (T3(i, j, kcm) - T3(i, j - 1, kcm))));
      const double maskUp = mm * m0;
      dfr = dfr - rA * maskInC * (G3(Kwx, i, j, kc) * dTdx + G3(Kwy, i, j, kc) * dTdy) * maskUp;
    }
    return fv + dfr;
  };
  const long q3 = MG_I3(d, i, j, k, t);
  const double Tk = T[q3];
  const double uT0 = uFld(i, j) * (G2(dyG, i, j) * drF * G3(hFacW, i, j, k));
  const double uT1 = uFld(i + 1, j) * (G2(dyG, i + 1, j) * drF * G3(hFacW, i + 1, j, k));
  const double vT0 = vFld(i, j) * (G2(dxG, i, j) * drF * G3(hFacS, i, j, k));
  const double vT1 = vFld(i, j + 1) * (G2(dxG, i, j + 1) * drF * G3(hFacS, i, j + 1, k));
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
  if (!p.tracForcingOutAB) gT = gT + gtForc;   // inside (0) / after (1) AB2: temp_integrate.F:373-410
  if (a.useAB && p.useAB3) {   // ADAMS_BASHFORTH3(k) (adams_bashforth3.F:60-103; startAB = nIter0)
    const int n0 = p.nIter0, startAB = p.nIter0;
    double ab0, ab1, ab2;
    if (myIter == n0 && startAB == 0) { ab0 = 0.0; ab1 = 0.0; ab2 = 0.0; }
    else if ((myIter == n0 && startAB == 1) || (myIter == 1 + n0 && startAB == 0)) { ab0 = p.alph_AB; ab1 = -p.alph_AB; ab2 = 0.0; }
    else { ab0 = p.alph_AB + p.beta_AB; ab1 = -p.alph_AB - 2. * p.beta_AB; ab2 = p.beta_AB; }
    const bool m1first = (myIter + 1) % 2 == 0;   // m1 = 1 + MOD(myIter+1, 2): slot 1 is gNm1, slot 2 gNm2
    double *gA = m1first ? a.gNm1 : a.gNm2, *gB = m1first ? a.gNm2 : a.gNm1;
    const double g = gT;
    const double abG = ab0 * g + ab1 * gA[q3] + ab2 * gB[q3];
    gB[q3] = g;
    gT = g + abG;
  } else if (a.useAB) {   // ADAMS_BASHFORTH2(k)
    const double ab = abFac * (gT - a.gNm1[q3]);
    double gN = gT;
    gT = gT + ab;
    // FREESURF_RESCALE_G of gT and gtNm1 under r* (temp_integrate.F:412-446)
    if (p.nonlinFreeSurf > 0 && p.select_rStar > 0) gN = gN / f.rStarExpC[q];
    a.gNm1[q3] = gN;
  }
  if (p.tracForcingOutAB) gT = gT + gtForc;
  if (p.nonlinFreeSurf > 0 && p.select_rStar > 0) gT = gT / f.rStarExpC[q];
  // TIMESTEP_TRACER
  const double v = Tk + p.deltaTtracer * gT;
  if (p.implicitDiffusion) a.scr[q3] = v;
  else a.trNext[q3] = v;   // CYCLE_TRACER directly
#undef T3
#undef G2
#undef G3
}
template <bool GM>
__global__ void __launch_bounds__(256) k_tracer_rhs(Dims d, Params p, Fields f, TracerArgs a, const int *iterPtr) {
  tracer_rhs_body<GM>(d, p, f, a, iterPtr, mg_xcd_block());
}

// k_tracer_rhs without GM/Redi, every load issued up front: the same expression trees as
// k_tracer_rhs<false> (bit-identical), but the 35 operands of a point are fetched before any
// arithmetic, unconditionally (vertical neighbours at clamped levels, whose terms the
// reference's kk >= 2 / kk <= Nr conditions then drop; 2-D/3-D fields the options do not
// use read and discarded), so a wave waits on memory once instead of once per branch.
// The operands of one point: 2-D (k-invariant) and 3-D at levels k-1, k, k+1.
struct TrCol {   // the k-invariant operands of a column
  double dyG0, dyG1, dxG0, dxG1, rdxC0, rdxC1, rdyC0, rdyC1, maskInC, recip_rA, rA, sfc, rsx;
};
struct TrLev {   // level k's operands (Tu/mCu/... at k-1 and Td/w1/mCd/ivd1 at k+1, clamped)
  double T0, Tw, Te, Ts, Tn, Tu, Td, u0, u1, v0, v1, w0, w1, hW0, hW1, hS0, hS1, mCu, mC0, mCd, ivd0, ivd1, rhC, gAdv,
      gOld;
};
__device__ __forceinline__ void tracer_load_col(const Dims &d, const Fields &f, const TracerArgs &a, long q, TrCol &c) {
  const long nx = d.nx;
  c.dyG0 = f.dyG[q]; c.dyG1 = f.dyG[q + 1]; c.dxG0 = f.dxG[q]; c.dxG1 = f.dxG[q + nx];
  c.rdxC0 = f.recip_dxC[q]; c.rdxC1 = f.recip_dxC[q + 1]; c.rdyC0 = f.recip_dyC[q]; c.rdyC1 = f.recip_dyC[q + nx];
  c.maskInC = f.maskInC[q]; c.recip_rA = f.recip_rA[q]; c.rA = f.rA[q];
  c.sfc = a.sfc ? a.sfc[q] : 0.0; c.rsx = f.rStarExpC[q];
}
// T*, and (useAB) the new AB history value into *gN, from the operands: k_tracer_rhs<false>'s
// arithmetic, term for term
__device__ __forceinline__ double tracer_flat_arith(const Params &p, const Fields &f, const TracerArgs &a, int Nr, int k,
                                                    int myIter, const TrCol &c, const TrLev &o, double *gN) {
  const double abFac = (myIter == p.nIter0 && p.nIter0 == 0) ? 0.0 : 0.5 + p.abEps;
  const bool calcAdv = a.advection && !a.multiDim;
  const double advFac = calcAdv ? 1.0 : 0.0, rAdvFac = p.rkSign * advFac;
  const double drF = f.drF[k - 1];
  auto face = [&](double vel, double g, double h, double rd, double tp, double tm) {   // fzon / fmer
    const double A = g * drF * h;
    double fz = 0.0;
    if (calcAdv) fz = fz + (vel * A) * (tp + tm) * 0.5;
    double df = 0.0;
    if (a.diffKh != 0.0) df = -a.diffKh * A * rd * (tp - tm);
    return fz + df;
  };
  const double rTrans = k <= 1 ? 0.0 : o.w0 * c.rA * (o.mCu * o.mC0);
  const double rTransKp = k + 1 > Nr ? 0.0 : o.w1 * c.rA * (o.mC0 * o.mCd);
  // the level's 1-D factors read at its start (behind the branches each load waited alone)
  const double rdcUp = f.recip_drC[k - 1], rdcDn = f.recip_drC[k < Nr ? k : Nr - 1];
  const double rdrFk = f.recip_drF[k - 1], rdrF0 = f.recip_drF[0];
  auto fvert = [&](int kk, double rTr, double mUpper, double mLower, double tLower, double tUpper, double ivd, double rdc) {
    double fv = 0.0;
    if (kk >= 2 && kk <= Nr && calcAdv) {
      const double wT = mUpper * rTr * (tLower + tUpper) * 0.5;
      fv = fv + wT * c.maskInC;
    }
    double dfr = 0.0;
    if (!p.implicitDiffusion && kk >= 2 && kk <= Nr) {
      const double kap = (ivd * p.ivdc_kappa + 0.0) + a.diffKr;
      const double maskUp = mUpper * mLower;
      dfr = -kap * maskUp * c.rA * rdc * (tLower - tUpper) * p.rkSign;
    }
    return fv + dfr;
  };
  const double uT0 = o.u0 * (c.dyG0 * drF * o.hW0), uT1 = o.u1 * (c.dyG1 * drF * o.hW1);
  const double vT0 = o.v0 * (c.dxG0 * drF * o.hS0), vT1 = o.v1 * (c.dxG1 * drF * o.hS1);
  const double fVerUp = fvert(k, rTrans, o.mCu, o.mC0, o.T0, o.Tu, o.ivd0, rdcUp);
  const double fVerDn = fvert(k + 1, rTransKp, o.mC0, o.mCd, o.Td, o.T0, o.ivd1, rdcDn);
  const double fZi = face(o.u0, c.dyG0, o.hW0, c.rdxC0, o.T0, o.Tw), fZe = face(o.u1, c.dyG1, o.hW1, c.rdxC1, o.Te, o.T0);
  const double fMi = face(o.v0, c.dxG0, o.hS0, c.rdyC0, o.T0, o.Ts), fMn = face(o.v1, c.dxG1, o.hS1, c.rdyC1, o.Tn, o.T0);
  const double g0 = a.multiDim ? o.gAdv : 0.0;
  double gT = g0 - o.rhC * rdrFk * c.recip_rA *
                       ((fZe - fZi) * c.maskInC + (fMn - fMi) * c.maskInC + (fVerDn - fVerUp) * p.rkSign -
                        o.T0 * ((uT1 - uT0) * advFac + (vT1 - vT0) * advFac + (rTransKp - rTrans) * rAdvFac) * c.maskInC);
  double gtForc = 0.0;
  if (a.forcing && a.sfc && k == 1) gtForc = gtForc + c.sfc * rdrF0 * o.rhC;
  if (!p.tracForcingOutAB) gT = gT + gtForc;
  const bool rs = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
  if (a.useAB) {
    const double ab = abFac * (gT - o.gOld);
    double gNv = gT;
    gT = gT + ab;
    if (rs) gNv = gNv / c.rsx;
    *gN = gNv;
  }
  if (p.tracForcingOutAB) gT = gT + gtForc;
  if (rs) gT = gT / c.rsx;
  return o.T0 + p.deltaTtracer * gT;
}
__device__ __forceinline__ double tracer_flat_point(const Dims &d, const Params &p, const Fields &f, const TracerArgs &a,
                                                   int i, int j, int k, int t, int myIter) {
  const int Nr = d.Nr;
  const long nx = d.nx, q = MG_I2(d, i, j, t), q3 = MG_I3(d, i, j, k, t);
  const long dku = (k > 1 ? -1L : 0L) * d.n2, dkd = (k < Nr ? 1L : 0L) * d.n2;
  const double *__restrict__ T = a.tr;
  TrLev o;
  o.T0 = T[q3]; o.Tw = T[q3 - 1]; o.Te = T[q3 + 1]; o.Ts = T[q3 - nx]; o.Tn = T[q3 + nx];
  o.Tu = T[q3 + dku]; o.Td = T[q3 + dkd];
  o.u0 = f.uVel[q3]; o.u1 = f.uVel[q3 + 1]; o.v0 = f.vVel[q3]; o.v1 = f.vVel[q3 + nx];
  o.w0 = f.wVel[q3]; o.w1 = f.wVel[q3 + dkd];
  o.hW0 = f.hFacW[q3]; o.hW1 = f.hFacW[q3 + 1]; o.hS0 = f.hFacS[q3]; o.hS1 = f.hFacS[q3 + nx];
  o.mCu = f.maskC[q3 + dku]; o.mC0 = f.maskC[q3]; o.mCd = f.maskC[q3 + dkd];
  o.ivd0 = f.IVDConvCount[q3]; o.ivd1 = f.IVDConvCount[q3 + dkd];
  TrCol c;
  tracer_load_col(d, f, a, q, c);
  o.rhC = f.recip_hFacC[q3]; o.gAdv = f.gAdv[q3]; o.gOld = a.gNm1[q3];
  double gN = 0.0;
  const double v = tracer_flat_arith(p, f, a, Nr, k, myIter, c, o, &gN);
  if (a.useAB) a.gNm1[q3] = gN;
  return v;
}

// The flat right-hand side as a k-march (LLC-sized grids): a workgroup owns a 32 x 8 (i, j)
// tile of one tile's interior and walks levels k0..k0+KC-1, each thread one column.  The
// column's k-invariant operands are loaded once, its own T, w, maskC and IVDConvCount at k-1,
// k, k+1 are carried in registers from level to level (one new level per step instead of
// three), so the vertical neighbours are never re-fetched by another workgroup -- the flat
// kernel's over-fetch (616 MB HBM for 173 MB of operands on LLC-90).  Same operands, same
// arithmetic (tracer_flat_arith): bit-identical.
constexpr int TRM_TX = 32, TRM_TY = 8;
// At most 2 waves per SIMD (MGCM_TRM_WPE; tools/wpe_variant.sh builds other caps): alone the
// k-march takes the same time at 2, 3 or 4 (HBM-bound), but beside the multi-workgroup CG2D
// (the late join) its fourth wave per SIMD costs the solve's hand-offs more than it gains:
// LLC-90 1.81 ms/step uncapped, 1.715 at 3, 1.714 at 2, 1.79 at 1 (profiles/r03/wpe/)
#ifndef MGCM_TRM_WPE
#define MGCM_TRM_WPE 2
#endif
#define TRM_ATTR __attribute__((amdgpu_waves_per_eu(1, MGCM_TRM_WPE)))
__global__ void __launch_bounds__(256) TRM_ATTR k_tracer_march(Dims d, Params p, Fields f, TracerArgs a, const int *iterPtr, int KC,
                                                     int nkc, int ntx, int nty) {
  int b = mg_xcd_block();
  const int kc = b % nkc;
  b /= nkc;
  const int tx = b % ntx, ty = (b / ntx) % nty, t = d.t0 + b / (ntx * nty);
  const int i = 1 + tx * TRM_TX + (int)(threadIdx.x % TRM_TX), j = 1 + ty * TRM_TY + (int)(threadIdx.x / TRM_TX);
  if (i > d.sNx || j > d.sNy) return;
  const int Nr = d.Nr, k0 = 1 + kc * KC, k1 = min(Nr, k0 + KC - 1);
  const int myIter = *iterPtr;
  const long nx = d.nx, n2 = d.n2, q = MG_I2(d, i, j, t);
  const double *__restrict__ T = a.tr;
  TrCol c;
  tracer_load_col(d, f, a, q, c);
  long q3 = MG_I3(d, i, j, k0, t);
  const long qu = k0 > 1 ? q3 - n2 : q3;
  double Tu = T[qu], mCu = f.maskC[qu];
  double T0 = T[q3], mC0 = f.maskC[q3], w0 = f.wVel[q3], ivd0 = f.IVDConvCount[q3];
  for (int k = k0; k <= k1; k++, q3 += n2) {
    const long qd = k < Nr ? q3 + n2 : q3;
    TrLev o;
    o.T0 = T0; o.Tu = Tu; o.mC0 = mC0; o.mCu = mCu; o.w0 = w0; o.ivd0 = ivd0;
    o.Td = T[qd]; o.mCd = f.maskC[qd]; o.w1 = f.wVel[qd]; o.ivd1 = f.IVDConvCount[qd];
    o.Tw = T[q3 - 1]; o.Te = T[q3 + 1]; o.Ts = T[q3 - nx]; o.Tn = T[q3 + nx];
    o.u0 = f.uVel[q3]; o.u1 = f.uVel[q3 + 1]; o.v0 = f.vVel[q3]; o.v1 = f.vVel[q3 + nx];
    o.hW0 = f.hFacW[q3]; o.hW1 = f.hFacW[q3 + 1]; o.hS0 = f.hFacS[q3]; o.hS1 = f.hFacS[q3 + nx];
    o.rhC = f.recip_hFacC[q3]; o.gAdv = a.multiDim ? f.gAdv[q3] : 0.0; o.gOld = a.useAB ? a.gNm1[q3] : 0.0;
    double gN = 0.0;
    const double v = tracer_flat_arith(p, f, a, Nr, k, myIter, c, o, &gN);
    if (a.useAB) a.gNm1[q3] = gN;
    if (p.implicitDiffusion) a.scr[q3] = v;
    else a.trNext[q3] = v;
    Tu = T0; T0 = o.Td; mCu = mC0; mC0 = o.mCd; w0 = o.w1; ivd0 = o.ivd1;
  }
}

// k_tracer_march with 16-byte accesses: a thread marches two adjacent columns (i, i+1), i odd
// (with OLx even the pair starts 16-B aligned), so the level's loads of the column pair are
// double2 per lane -- T, T(j-1), T(j+1), v(j), v(j+1), hFacS(j), hFacS(j+1), w, maskC,
// IVDConvCount, recip_hFacC, the AB history, the stores of T* and the history -- and only
// T(i-1), T(i+2), u(i+2), hFacW(i+2) are single doubles.  A workgroup covers whole rows of
// the tile (sNx/2 pairs x 256/(sNx/2) rows), so a wave reads contiguous row segments.  Each
// column's arithmetic is tracer_flat_arith on its own operands: bit-identical.
// FWD (whole columns, KC = Nr): GAD_IMPLICIT_R's coefficients of each level (from the level's
// own operands, already in registers: maskC at k-1 / k+1, IVDConvCount at k / k+1,
// recip_hFacC) and SOLVE_TRIDIAGONAL's forward elimination ride in the march, in
// tracer_impl_body's expressions and order; the march stores (c', y') instead of T*, and
// k_tracer_backsub finishes the column.  No T* round trip, no second pass over the
// coefficient operands.
typedef __attribute__((ext_vector_type(2))) double trd2;
// SOLVE_TRIDIAGONAL's back substitution of one column pair (first level's offset q1) from
// the (c', y') k_tracer_march2<true> stored: all of a batch's loads issued before its part of
// the recurrence (they do not depend on it), the new tracer written level by level
__device__ __forceinline__ void tracer_backsub_pair(const Dims &d, const TracerArgs &a, long q1) {
  const int Nr = d.Nr;
  const long n2 = d.n2;
  auto L2 = [](const double *x, long o) { return *reinterpret_cast<const trd2 *>(x + o); };
  constexpr int CH = 10;   // levels per batch of loads
  trd2 below = {0.0, 0.0};
  for (int k1 = Nr; k1 >= 1; k1 -= CH) {
    const int k0 = k1 - CH + 1 > 1 ? k1 - CH + 1 : 1;
    trd2 cpv[CH], ypv[CH];
#pragma unroll
    for (int u = 0; u < CH; u++) {
      const int k = k1 - u;
      if (k >= k0) {
        const long q3 = q1 + (long)(k - 1) * n2;
        cpv[u] = L2(a.cp, q3);
        ypv[u] = L2(a.scr, q3);
      }
    }
#pragma unroll
    for (int u = 0; u < CH; u++) {
      const int k = k1 - u;
      if (k >= k0) {
        trd2 v;
        if (k == Nr) v = ypv[u];
        else { v.x = ypv[u].x - cpv[u].x * below.x; v.y = ypv[u].y - cpv[u].y * below.y; }
        *reinterpret_cast<trd2 *>(a.trNext + q1 + (long)(k - 1) * n2) = v;
        below = v;
      }
    }
  }
}
// BACK (with FWD): the back substitution too, by the same thread right after its column's
// forward sweep (tracer_backsub_pair: the (c', y') it just stored, read back from the caches)
template <bool FWD, bool BACK = false>
__global__ void __launch_bounds__(256) TRM_ATTR k_tracer_march2(Dims d, Params p, Fields f, TracerArgs a, const int *iterPtr,
                                                                int KC, int nkc, int nty) {
  int b = mg_xcd_block();
  const int kc = b % nkc;
  b /= nkc;
  const int hx = d.sNx >> 1;
  int i, j, t;
  if (nty < 0) {   // flat: -nty consecutive column pairs of the slab's interior per workgroup
    const int pw = -nty, np = hx * d.sNy;
    if ((int)threadIdx.x >= pw) return;
    const long gid = (long)b * pw + threadIdx.x;
    if (gid >= (long)np * d.nT) return;
    const int rem = (int)(gid % np);
    t = d.t0 + (int)(gid / np);
    j = 1 + rem / hx;
    i = 1 + 2 * (rem % hx);
  } else {         // whole rows of one tile: sNx/2 pairs x 256/(sNx/2) rows
    const int TY = 256 / hx;
    const int ty = b % nty;
    t = d.t0 + b / nty;
    const int px = (int)threadIdx.x % hx, jy = (int)threadIdx.x / hx;
    if (jy >= TY) return;
    i = 1 + 2 * px;
    j = 1 + ty * TY + jy;
    if (j > d.sNy) return;
  }
  const int Nr = d.Nr, k0 = 1 + kc * KC, k1 = min(Nr, k0 + KC - 1);
  const int myIter = *iterPtr;
  const long nx = d.nx, n2 = d.n2, q = MG_I2(d, i, j, t);
  const double *__restrict__ T = a.tr;
  auto L2 = [](const double *x, long o) { return *reinterpret_cast<const trd2 *>(x + o); };
  TrCol c[2];
  tracer_load_col(d, f, a, q, c[0]);
  tracer_load_col(d, f, a, q + 1, c[1]);
  long q3 = MG_I3(d, i, j, k0, t);
  const long qu = k0 > 1 ? q3 - n2 : q3;
  trd2 Tu = L2(T, qu), mCu = L2(f.maskC, qu);
  trd2 T0 = L2(T, q3), mC0 = L2(f.maskC, q3), w0 = L2(f.wVel, q3), ivd0 = L2(f.IVDConvCount, q3);
  double cpPrev[2] = {0.0, 0.0}, ypPrev[2] = {0.0, 0.0};   // FWD: the sweep's previous level
  const bool rs = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
  for (int k = k0; k <= k1; k++, q3 += n2) {
    const long qd = k < Nr ? q3 + n2 : q3;
    const trd2 Td = L2(T, qd), mCd = L2(f.maskC, qd), w1 = L2(f.wVel, qd), ivd1 = L2(f.IVDConvCount, qd);
    double rdrFk = 0.0, rdcK = 0.0, rdcP = 0.0;
    if constexpr (FWD) {
      rdrFk = f.recip_drF[k - 1];
      rdcK = f.recip_drC[k - 1];
      rdcP = f.recip_drC[(k <= Nr - 1 ? k + 1 : Nr) - 1];
    }
    const trd2 Ts = L2(T, q3 - nx), Tn = L2(T, q3 + nx);
    const double Tw = T[q3 - 1], Te = T[q3 + 2];
    const trd2 u01 = L2(f.uVel, q3), v0 = L2(f.vVel, q3), v1 = L2(f.vVel, q3 + nx);
    const double u2 = f.uVel[q3 + 2], hW2 = f.hFacW[q3 + 2];
    const trd2 hW01 = L2(f.hFacW, q3), hS0 = L2(f.hFacS, q3), hS1 = L2(f.hFacS, q3 + nx);
    const trd2 rhC = L2(f.recip_hFacC, q3);
    const trd2 gA = a.multiDim ? L2(f.gAdv, q3) : trd2{0.0, 0.0};
    const trd2 gO = a.useAB ? L2(a.gNm1, q3) : trd2{0.0, 0.0};
    double v[2], gN[2] = {0.0, 0.0}, cpo[2] = {0.0, 0.0};
#pragma unroll
    for (int e = 0; e < 2; e++) {
      TrLev o;
      o.T0 = e ? T0.y : T0.x; o.Tu = e ? Tu.y : Tu.x; o.Td = e ? Td.y : Td.x;
      o.Tw = e ? T0.x : Tw; o.Te = e ? Te : T0.y;
      o.Ts = e ? Ts.y : Ts.x; o.Tn = e ? Tn.y : Tn.x;
      o.u0 = e ? u01.y : u01.x; o.u1 = e ? u2 : u01.y;
      o.v0 = e ? v0.y : v0.x; o.v1 = e ? v1.y : v1.x;
      o.w0 = e ? w0.y : w0.x; o.w1 = e ? w1.y : w1.x;
      o.hW0 = e ? hW01.y : hW01.x; o.hW1 = e ? hW2 : hW01.y;
      o.hS0 = e ? hS0.y : hS0.x; o.hS1 = e ? hS1.y : hS1.x;
      o.mCu = e ? mCu.y : mCu.x; o.mC0 = e ? mC0.y : mC0.x; o.mCd = e ? mCd.y : mCd.x;
      o.ivd0 = e ? ivd0.y : ivd0.x; o.ivd1 = e ? ivd1.y : ivd1.x;
      o.rhC = e ? rhC.y : rhC.x; o.gAdv = e ? gA.y : gA.x; o.gOld = e ? gO.y : gO.x;
      v[e] = tracer_flat_arith(p, f, a, Nr, k, myIter, c[e], o, &gN[e]);
      if constexpr (FWD) {   // tracer_impl_body<true>'s coefficients, then its forward step
        const double rh = rs ? o.rhC / c[e].rsx : o.rhC;
        auto kappa = [&](double ivd) { return (ivd * p.ivdc_kappa + 0.0) + a.diffKr; };
        double sub = 0.0, sup = 0.0;
        if (k >= 2) sub = -(p.deltaTtracer * o.mCu * rh * rdrFk * kappa(o.ivd0) * rdcK);
        if (k <= Nr - 1) sup = -(p.deltaTtracer * o.mCd * rh * rdrFk * kappa(o.ivd1) * rdcP);
        const double diag = 1.0 - (sub + sup), y = v[e];
        double cp, yp;
        if (k == 1) {
          if (diag != 0.0) { const double rec = 1.0 / diag; cp = sup * rec; yp = y * rec; }
          else { cp = 0.0; yp = 0.0; }
        } else {
          const double tmp = diag - sub * cpPrev[e];
          if (tmp != 0.0) { const double rec = 1.0 / tmp; cp = sup * rec; yp = (y - sub * ypPrev[e]) * rec; }
          else { cp = 0.0; yp = 0.0; }
        }
        cpPrev[e] = cp; ypPrev[e] = yp;
        cpo[e] = cp; v[e] = yp;
      }
    }
    if (a.useAB) *reinterpret_cast<trd2 *>(a.gNm1 + q3) = trd2{gN[0], gN[1]};
    *reinterpret_cast<trd2 *>((p.implicitDiffusion ? a.scr : a.trNext) + q3) = trd2{v[0], v[1]};
    if constexpr (FWD) *reinterpret_cast<trd2 *>(a.cp + q3) = trd2{cpo[0], cpo[1]};
    Tu = T0; T0 = Td; mCu = mC0; mC0 = mCd; w0 = w1; ivd0 = ivd1;
  }
  if constexpr (FWD && BACK) tracer_backsub_pair(d, a, MG_I3(d, i, j, 1, t));
}


// SOLVE_TRIDIAGONAL's back substitution (tracer_impl_body's upward sweep) from the (c', y')
// k_tracer_march2<true> stored: one thread per interior column pair (16-byte accesses), all
// levels' loads issued before the recurrence (they do not depend on it), the new tracer
// written to its other buffer (CYCLE_TRACER).
__global__ void __launch_bounds__(256) k_tracer_backsub(Dims d, TracerArgs a, int nty) {
  const int b = mg_xcd_block();
  const int hx = d.sNx >> 1, TY = 256 / hx;
  const int ty = b % nty, t = d.t0 + b / nty;
  const int px = (int)threadIdx.x % hx, jy = (int)threadIdx.x / hx;
  if (jy >= TY) return;
  const int i = 1 + 2 * px, j = 1 + ty * TY + jy;
  if (j > d.sNy) return;
  tracer_backsub_pair(d, a, MG_I3(d, i, j, 1, t));
}

__global__ void __launch_bounds__(256) k_tracer_rhs_flat(Dims d, Params p, Fields f, TracerArgs a, const int *iterPtr) {
  MG_PLANE(1, d.sNx, 1, d.sNy, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  if (i > d.sNx || j > d.sNy) return;
  const long q3 = MG_I3(d, i, j, k, t);
  const double v = tracer_flat_point(d, p, f, a, i, j, k, t, *iterPtr);
  if (p.implicitDiffusion) a.scr[q3] = v;
  else a.trNext[q3] = v;
}


// GAD_IMPLICIT_R (implicitDiffusion) + SOLVE_TRIDIAGONAL (Thomas) + CYCLE_TRACER,
// one thread per interior column; writes the new tracer into its other buffer.
// GAD_IMPLICIT_R + SOLVE_TRIDIAGONAL per column (gad_implicit_r.F:96-140, the
// Thomas sweep of solve_tridiagonal.F): the coefficients and right-hand side of
// every level are formed k-parallel into LDS, one thread per column then sweeps
// down and up in LDS with the reference's operations, and the levels are
// written back k-parallel.
// UL: every coefficient operand loaded unconditionally at clamped levels (the standalone
// kernel on deep columns: LLC-90 1.226-1.241 against 1.265-1.267 ms/step with the tracer
// march's hoisted factors, profiles/r05/tracer_loads/); the fused C2 / C3 kernels keep the
// branch form (0.3-0.9 % slower there with UL, more VGPRs for the few levels each thread forms)
template <bool UL>
__device__ __forceinline__ void tracer_impl_body(const Dims &d, const Params &p, const Fields &f, const TracerArgs &a, int nc,
                                                 int lb) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  MG_COLF_LB(1, d.sNx, 1, d.sNy, nc, lb)
  const int Nr = d.Nr, NS = Nr * NC_;
  double *sSub = lds, *sSup = lds + NS, *sY = lds + 2 * NS;   // sSub holds the solution after the sweeps
#define G3(a_, ii, jj, kk_) f.a_[MG_I3(d, ii, jj, kk_, t)]
  if (valid) {
    // recip_hFacNew (thermodynamics.F:198-210): recip_hFacC/rStarExpC under r*
    const bool rs = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
    const long q2 = MG_I2(d, i, j, t);
    const double rsx = rs ? f.rStarExpC[q2] : 1.0;
    const double mIn = f.maskInC[q2];
    // KappaRT = (IVDConvCount*ivdc_kappa + BL79(=0)) + diffKrNr [+ Kwz*maskInC] (calc_3d_diffusivity.F)
    auto kappa = [&](double ivd, double kwz) {
      double kap = (ivd * p.ivdc_kappa + 0.0) + a.diffKr;
      if (p.useGMRedi) kap = kap + kwz * mIn;
      return kap;
    };
    if constexpr (!UL) MG_COLF_K(k) {
      const int me = (k - 1) * NC_ + cc;
      const long q3 = MG_I3(d, i, j, k, t);
      const double rh = rs ? f.recip_hFacC[q3] / rsx : f.recip_hFacC[q3];
      const double rdrF = f.recip_drF[k - 1];
      double sub = 0.0, sup = 0.0;
      if (k >= 2)
        sub = -(p.deltaTtracer * G3(maskC, i, j, k - 1) * rh * rdrF *
                kappa(G3(IVDConvCount, i, j, k), p.useGMRedi ? G3(Kwz, i, j, k) : 0.0) * f.recip_drC[k - 1]);
      if (k <= Nr - 1)
        sup = -(p.deltaTtracer * G3(maskC, i, j, k + 1) * rh * rdrF *
                kappa(G3(IVDConvCount, i, j, k + 1), p.useGMRedi ? G3(Kwz, i, j, k + 1) : 0.0) * f.recip_drC[k]);
      sSub[me] = sub;
      sSup[me] = sup;
      sY[me] = a.scr[q3];
    }
    else MG_COLF_K(k) {
      // every operand loaded unconditionally (the levels above / below clamped into the
      // column), then the reference's conditions select: no load waits behind a branch
      const int me = (k - 1) * NC_ + cc;
      const int km = k >= 2 ? k - 1 : 1, kp = k <= Nr - 1 ? k + 1 : Nr;
      const long q3 = MG_I3(d, i, j, k, t);
      const double rhc = f.recip_hFacC[q3], y = a.scr[q3];
      const double mM = G3(maskC, i, j, km), mP = G3(maskC, i, j, kp);
      const double ivK = G3(IVDConvCount, i, j, k), ivP = G3(IVDConvCount, i, j, kp);
      const double kwK = p.useGMRedi ? G3(Kwz, i, j, k) : 0.0, kwP = p.useGMRedi ? G3(Kwz, i, j, kp) : 0.0;
      const double rdrF = f.recip_drF[k - 1], rdcK = f.recip_drC[k - 1], rdcP = f.recip_drC[kp - 1];
      const double rh = rs ? rhc / rsx : rhc;
      double sub = 0.0, sup = 0.0;
      if (k >= 2) sub = -(p.deltaTtracer * mM * rh * rdrF * kappa(ivK, kwK) * rdcK);
      if (k <= Nr - 1) sup = -(p.deltaTtracer * mP * rh * rdrF * kappa(ivP, kwP) * rdcP);
      sSub[me] = sub;
      sSup[me] = sup;
      sY[me] = y;
    }
  }
  __syncthreads();
  if (valid && kk == 0) {
    double cpPrev = 0.0, ypPrev = 0.0;
    for (int k2 = 1; k2 <= Nr; k2++) {
      const int s2 = (k2 - 1) * NC_ + cc;
      const double sub = sSub[s2], sup = sSup[s2];
      const double diag = 1.0 - (sub + sup);
      const double y = sY[s2];
      double cp, yp;
      if (k2 == 1) {
        if (diag != 0.0) { const double rec = 1.0 / diag; cp = sup * rec; yp = y * rec; }
        else { cp = 0.0; yp = 0.0; }
      } else {
        const double tmp = diag - sub * cpPrev;
        if (tmp != 0.0) { const double rec = 1.0 / tmp; cp = sup * rec; yp = (y - sub * ypPrev) * rec; }
        else { cp = 0.0; yp = 0.0; }
      }
      sSup[s2] = cp;   // reuse: the c' coefficients
      sY[s2] = yp;
      cpPrev = cp; ypPrev = yp;
    }
    double below = 0.0;
    for (int k2 = Nr; k2 >= 1; k2--) {
      const int s2 = (k2 - 1) * NC_ + cc;
      const double v = (k2 == Nr) ? sY[s2] : sY[s2] - sSup[s2] * below;
      sSub[s2] = v;
      below = v;
    }
  }
  __syncthreads();
  if (valid) MG_COLF_K(k) a.trNext[MG_I3(d, i, j, k, t)] = sSub[(k - 1) * NC_ + cc];
#undef G3
}
#ifdef MGCM_TRI_WPE
#define TRI_ATTR __attribute__((amdgpu_waves_per_eu(1, MGCM_TRI_WPE)))
#else
#define TRI_ATTR
#endif
template <bool UL>
__global__ void __launch_bounds__(256) TRI_ATTR k_tracer_impl(Dims d, Params p, Fields f, TracerArgs a, int nc) {
  tracer_impl_body<UL>(d, p, f, a, nc, mg_xcd_block());
}

// gm = false: without GMREDI_CALC_TENSOR (it then rides in the next launch, launch_dyn_thermo)
// GMREDI_CALC_TENSOR alone (THERMODYNAMICS' first launch when it runs on its own stream)
hipError_t launch_gm_tensor(const Dims &d, const Params &p, const Fields &f, hipStream_t s) {
  if (!p.useGMRedi) return hipSuccess;
  hipLaunchKernelGGL(k_gm_tensor, dim3(mg_plane_blocks(d.nx - 2, d.ny - 2, d.nT * d.Nr)), dim3(MG_PLANE_THREADS), 0, s, d,
                     p, f);
  return hipGetLastError();
}

// The hFac THERMODYNAMICS reads, copied before UPDATE_R_STAR(.TRUE.) rewrites them (one_step's
// MG_FUSE_TCG layout): hFacC, hFacW, hFacS and their reciprocals into snap[6 x N3all]; the
// tracer kernels then get the Fields with those six pointers moved to the copy.
struct Snap6 {
  const double *src[6];
  double *dst[6];
};
__global__ void __launch_bounds__(256) k_hfac_snapshot(Snap6 sn, long n) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  if (q >= n) return;
  const int a = (int)blockIdx.y;
  sn.dst[a][q] = sn.src[a][q];
}
Fields hfac_snapshot_fields(const Dims &d, const Fields &f, double *snap) {
  Fields g = f;
  g.hFacC = snap; g.hFacW = snap + d.N3all; g.hFacS = snap + 2 * d.N3all;
  g.recip_hFacC = snap + 3 * d.N3all; g.recip_hFacW = snap + 4 * d.N3all; g.recip_hFacS = snap + 5 * d.N3all;
  return g;
}
hipError_t launch_hfac_snapshot(const Dims &d, const Fields &f, double *snap, hipStream_t s) {
  const Fields g = hfac_snapshot_fields(d, f, snap);
  Snap6 sn{{f.hFacC, f.hFacW, f.hFacS, f.recip_hFacC, f.recip_hFacW, f.recip_hFacS},
           {g.hFacC, g.hFacW, g.hFacS, g.recip_hFacC, g.recip_hFacW, g.recip_hFacS}};
  const long n = d.N3all;
  hipLaunchKernelGGL(k_hfac_snapshot, dim3((unsigned)((n + 255) / 256), 6), dim3(256), 0, s, sn, n);
  return hipGetLastError();
}

hipError_t launch_phys_ring(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s);
// ringDone non-null: the per-point form takes the VI path's halo-ring AB2 into its grid
// (k_phys_ring) and sets *ringDone; the 16-byte form does not
hipError_t launch_oceanic_phys(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s, bool gm,
                               bool *ringDone) {
  auto al = [](const void *q) { return ((uintptr_t)q & 15u) == 0; };
  const int v2Env = getenv("MGCM_PHYS_V2") ? atoi(getenv("MGCM_PHYS_V2")) : 1;
  // (large grids only: on config 2's 70 k points per level set, half the threads cost more
  // than the wider accesses save -- 12.9 against 10.1 us, the surface level's forcing
  // interpolation then serial in each thread)
  const bool big = (long)d.n2 * d.nT * d.Nr >= (1L << 21);
  const bool v2 = v2Env != 0 && (big || v2Env == 2) && (d.n2 & 1) == 0 && (d.n3 & 1) == 0 && al(f.theta) && al(f.salt) && al(f.maskC) &&
                  al(f.rhoInSitu) && al(f.IVDConvCount) && (!p.useGMRedi || al(f.sigmaR)) &&
                  (p.eosType != 1 || p.selectP_inEOS_Zc != 2 || al(f.totPhiHyd));
  if (v2) {
    const unsigned nb = (unsigned)(((d.n2 >> 1) + 255) / 256);
    hipLaunchKernelGGL(k_oceanic_phys2, dim3(nb * (unsigned)(d.nT * d.Nr)), dim3(256), 0, s, d, p, f, iterPtr);
  } else if (ringDone) {
    const hipError_t e = launch_phys_ring(d, p, f, iterPtr, s);
    if (e != hipSuccess) return e;
    *ringDone = true;
  } else
    hipLaunchKernelGGL(k_oceanic_phys, dim3(mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr)), dim3(MG_PLANE_THREADS), 0, s, d, p,
                       f, iterPtr);
  if (p.useGMRedi && gm)
    hipLaunchKernelGGL(k_gm_tensor, dim3(mg_plane_blocks(d.nx - 2, d.ny - 2, d.nT * d.Nr)), dim3(MG_PLANE_THREADS), 0,
                       s, d, p, f);
  return hipGetLastError();
}

// the implicit solve inside the whole-column march (deep grids, where the k-march runs): its
// forward sweep, then its back substitution by the same thread (k_tracer_march2<true, true>,
// the default; MGCM_TRACER_MARCH=3), or the back substitution as a kernel of its own
// (k_tracer_backsub; =2).  Round 6, LLC-90 per tracer: one kernel 216 us and 734 MB
// (rocprofv3 time, FETCH+WRITE), against 161 + 105 us and 596 + 228 MB for the chunked
// march + k_tracer_impl (=1) and 171 + 47 us for =2; step 1.2326-1.2330 ms against
// 1.2330-1.2455 (=1) and 1.2495 (=2), alternating on one box (profiles/r06/fwdback/)
static int tracer_fwd_form(const Dims &d) {
  const char *e = getenv("MGCM_TRACER_MARCH");   // read per launch (tests switch it per model)
  if (!e) return d.Nr >= 30 ? 3 : 0;
  const int v = atoi(e);
  return v == 2 || v == 3 ? v : 0;
}
static bool tracer_march_on(const Dims &d) {
  const char *e = getenv("MGCM_TRACER_MARCH");   // read per launch (tests switch it per model)
  if (e) return atoi(e) != 0;
  return d.Nr >= 30;
}

// impl = false: the right-hand side only (the implicit solve is launched by the caller)
hipError_t launch_tracer_step(const Dims &d, const Params &p, const Fields &f, const TracerArgs &a, const int *iterPtr,
                              hipStream_t s, bool impl) {
  const dim3 blk(MG_PLANE_THREADS), grd(mg_plane_blocks(d.sNx, d.sNy, d.nT * d.Nr));
  if (a.multiDim) {
    const dim3 fgrd(mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr));
    const bool cube = p.cubeCorners != 0, comp = p.multiDimCompressible != 0;
    if (!cube && !comp) {   // lat-lon, 2 passes: fused per-point X and Y passes
      hipLaunchKernelGGL(k_adv_x, fgrd, blk, 0, s, d, f, a);
      hipLaunchKernelGGL(k_adv_y, grd, blk, 0, s, d, f, a);
      hipLaunchKernelGGL(k_adv_r<false>, grd, blk, 0, s, d, p, f, a, f.advScr2, f.advScr2);
    } else {                // the general form: explicit passes over the whole slab
      hipLaunchKernelGGL(k_advg_init, fgrd, blk, 0, s, d, f, a, (int)comp);
      const unsigned cgrd = (unsigned)((4L * d.OLx * d.OLy * d.nT * d.Nr + 255) / 256);
      for (int ipass = 1; ipass <= (cube ? 3 : 2); ipass++)
        for (int ydir = 0; ydir < 2; ydir++) {
          if (cube) hipLaunchKernelGGL(k_advg_fill, dim3(cgrd), blk, 0, s, d, f, ipass, 2 * ydir);
          hipLaunchKernelGGL(k_advg_flux, fgrd, blk, 0, s, d, f, a, ipass, ydir, (int)cube);
          if (cube) hipLaunchKernelGGL(k_advg_fill, dim3(cgrd), blk, 0, s, d, f, ipass, 2 * ydir + 1);
          hipLaunchKernelGGL(k_advg_upd, fgrd, blk, 0, s, d, f, a, ipass, ydir, (int)cube, (int)comp);
        }
      if (comp) hipLaunchKernelGGL(k_adv_r<true>, grd, blk, 0, s, d, p, f, a, f.advScr1, f.advScr2);
      else hipLaunchKernelGGL(k_adv_r<false>, grd, blk, 0, s, d, p, f, a, f.advScr1, f.advScr1);
    }
  }
  // GM/Redi fluxes as a template switch: without them the kernel holds half the registers
  if (p.useGMRedi) hipLaunchKernelGGL(k_tracer_rhs<true>, grd, blk, 0, s, d, p, f, a, iterPtr);
  else if (a.scheme != 2 || p.useAB3)   // U3 / C4 and ADAMS_BASHFORTH3: the generic body only
    hipLaunchKernelGGL(k_tracer_rhs<false>, grd, blk, 0, s, d, p, f, a, iterPtr);
  else if (tracer_march_on(d)) {
    // the k-march (deep grids; MGCM_TRACER_MARCH=0|1 overrides): KC levels per workgroup, five
    // chunks (round 3: LLC-90 fastest among 1/2/5/10 chunks, profiles/r03/)
    const int KC = (d.Nr + 4) / 5;
    const int nkc = (d.Nr + KC - 1) / KC, ntx = (d.sNx + TRM_TX - 1) / TRM_TX, nty = (d.sNy + TRM_TY - 1) / TRM_TY;
    auto al = [](const void *x) { return ((uintptr_t)x & 15u) == 0; };
    // the two-column form (double2 accesses) where the slab's layout allows it; MGCM_TRACER_MARCH2=0
    // forces the one-column form the other layouts run, =1 the whole-column march with whole
    // tile rows per workgroup instead of its column pairs dealt evenly over one workgroup per
    // CU (2, the default: LLC-90 211 against 216 us per tracer, step unchanged, 1.2495-1.2500
    // against 1.2492-1.2500 ms alternating on one box, profiles/r06/trflat/; tests cover all)
    const int m2Env = getenv("MGCM_TRACER_MARCH2") ? atoi(getenv("MGCM_TRACER_MARCH2")) : 2;
    const int hx = d.sNx / 2;
    if (m2Env != 0 && (d.sNx & 1) == 0 && (d.OLx & 1) == 0 && (d.nx & 1) == 0 && (d.n3 & 1) == 0 && hx <= 256 && al(a.tr) &&
        al(a.trNext) && al(a.scr) && al(a.gNm1) && al(f.maskC) && al(f.wVel) && al(f.IVDConvCount) && al(f.uVel) &&
        al(f.vVel) && al(f.hFacW) && al(f.hFacS) && al(f.recip_hFacC) && (!a.multiDim || al(f.gAdv))) {
      const int TY = 256 / hx, nty2 = (d.sNy + TY - 1) / TY;
      // the implicit solve inside a whole-column march (tracer_fwd_form): no T* round trip
      const int fwd = tracer_fwd_form(d);
      if (impl && p.implicitDiffusion && !p.useGMRedi && fwd && !a.multiDim && a.cp && al(a.cp) && d.Nr > 1) {
        if (fwd == 3) {
          if (m2Env == 2) {   // flat: the column pairs dealt evenly over one workgroup per CU
            static int nCU = 0;
            int dev = 0;
            if (!nCU && (hipGetDevice(&dev) != hipSuccess ||
                         hipDeviceGetAttribute(&nCU, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || nCU < 1))
              nCU = 256;
            const long np = (long)hx * d.sNy * d.nT;
            const int pw = (int)std::min<long>(256, (np + nCU - 1) / nCU);
            hipLaunchKernelGGL((k_tracer_march2<true, true>), dim3((unsigned)((np + pw - 1) / pw)), blk, 0, s, d, p, f, a,
                               iterPtr, d.Nr, 1, -pw);
            return hipGetLastError();
          }
          hipLaunchKernelGGL((k_tracer_march2<true, true>), dim3((unsigned)(nty2 * d.nT)), blk, 0, s, d, p, f, a, iterPtr,
                             d.Nr, 1, nty2);
          return hipGetLastError();
        }
        hipLaunchKernelGGL((k_tracer_march2<true, false>), dim3((unsigned)(nty2 * d.nT)), blk, 0, s, d, p, f, a, iterPtr,
                           d.Nr, 1, nty2);
        hipLaunchKernelGGL(k_tracer_backsub, dim3((unsigned)(nty2 * d.nT)), blk, 0, s, d, a, nty2);
        return hipGetLastError();
      }
      hipLaunchKernelGGL((k_tracer_march2<false, false>), dim3((unsigned)(nkc * nty2 * d.nT)), blk, 0, s, d, p, f, a, iterPtr,
                         KC, nkc, nty2);
    } else
      hipLaunchKernelGGL(k_tracer_march, dim3((unsigned)(nkc * ntx * nty * d.nT)), blk, 0, s, d, p, f, a, iterPtr, KC, nkc,
                         ntx, nty);
  } else hipLaunchKernelGGL(k_tracer_rhs_flat, grd, blk, 0, s, d, p, f, a, iterPtr);
  if (p.implicitDiffusion && impl) {
    const long ncol = (long)d.sNx * d.sNy * d.nT;
    const int nc = mg_colf_nc(ncol, d.Nr, 3);
    MG_ALLOW_LDS(k_tracer_impl<false>);
    MG_ALLOW_LDS(k_tracer_impl<true>);
    if (d.Nr >= 30)
      hipLaunchKernelGGL(k_tracer_impl<true>, dim3(mg_colf_blocks(ncol, nc)), blk, mg_colf_lds(d.Nr, nc, 3), s, d, p, f, a, nc);
    else
      hipLaunchKernelGGL(k_tracer_impl<false>, dim3(mg_colf_blocks(ncol, nc)), blk, mg_colf_lds(d.Nr, nc, 3), s, d, p, f, a, nc);
  }
  return hipGetLastError();
}

}  // namespace mgcm
