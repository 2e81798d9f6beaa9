// kernels_thermo.hip -- the tracer half of the step on the MI355X.
//
//   k_oceanic_phys  DO_OCEANIC_PHYS subset (model/src/do_oceanic_phys.F:555-882):
//                   surfaceForcingT from FORCING_SURF_RELAX (forcing_surf_relax.F:52-80),
//                   rhoInSitu = FIND_RHO_2D LINEAR (find_rho.F:125-136) at every level,
//                   IVDConvCount from GRAD_SIGMA/CALC_IVDC (grad_sigma.F:103-117, calc_ivdc.F:60-71).
//   k_temp_step     TEMP_INTEGRATE (model/src/temp_integrate.F) for theta, GAD C2 advection
//                   (gad_c2_adv_x/y/r.F), Laplacian diffusion (gad_diff_x/y.F), surface forcing
//                   (apply_forcing.F:687-695), AB2 on gT (adams_bashforth2.F:81-88),
//                   TIMESTEP_TRACER, GAD_IMPLICIT_R implicit vertical diffusion
//                   (gad_implicit_r.F:96-140) solved by the Thomas sweep of
//                   SOLVE_TRIDIAGONAL (solve_tridiagonal.F, default branch), CYCLE_TRACER.
//
// One thread owns one interior (i,j) column of one tile.  The RHS pass marches
// k = Nr..1 carrying the vertical flux of the face below and rTrans(k+1) in
// registers (the fVerT(kUp/kDown) ping-pong of temp_integrate.F); horizontal
// face fluxes are recomputed from the neighbours' state with the reference's
// operand order (bit-exact under -ffp-contract=off).  The new theta goes to the
// other buffer of a ping-pong pair (neighbours still read the old one); gT and
// the Thomas coefficients live in per-column scratch that the same thread
// writes and re-reads (L2-resident).  Only the interior is produced: the halo
// of theta is refilled by the end-of-step EXCH (do_fields_blocking_exchanges.F).
#include "common.h"

namespace mgcm {

__device__ __forceinline__ double rho_linear(const Params &p, const Fields &f, int kRef, double t, double s) {
  const double refTemp = f.tRef[kRef - 1], refSalt = f.sRef[kRef - 1];
  const double dRho = p.rhoNil - p.rhoConst;
  return p.rhoNil * (p.sBeta * (s - refSalt) - p.tAlpha * (t - refTemp)) + dRho;
}

__global__ void __launch_bounds__(256) k_oceanic_phys(Dims d, Params p, Fields f) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x) + 1 - d.OLx;
  const int j = (int)(blockIdx.y * blockDim.y + threadIdx.y) + 1 - d.OLy;
  const int t = (int)blockIdx.z;
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

__global__ void __launch_bounds__(256) k_temp_step(Dims d, Params p, Fields f, const int *iterPtr) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x) + 1;
  const int j = (int)(blockIdx.y * blockDim.y + threadIdx.y) + 1;
  const int t = (int)blockIdx.z;
  if (i > d.sNx || j > d.sNy) return;
  const int Nr = d.Nr;
  const int myIter = *iterPtr;
  const double abFac = (myIter == p.nIter0 && p.nIter0 == 0) ? 0.0 : 0.5 + p.abEps;
  const double advFac = p.tempAdvection ? 1.0 : 0.0, rAdvFac = p.rkSign * advFac;
  const double *__restrict__ T = f.theta;
  const long q = MG_I2(d, i, j, t);
  const double maskInC = f.maskInC[q], recip_rA = f.recip_rA[q], rA = f.rA[q];
#define T3(ii, jj, kk) T[MG_I3(d, ii, jj, kk, t)]
#define G2(a, ii, jj) f.a[MG_I2(d, ii, jj, t)]
#define G3(a, ii, jj, kk) f.a[MG_I3(d, ii, jj, kk, t)]
  // face flux at west face of column ii (fZon(ii)), at level k
  auto fzon = [&](int ii, int k, double drF) {
    const double xA = G2(dyG, ii, j) * drF * G3(hFacW, ii, j, k);
    double fz = 0.0;
    if (p.tempAdvection) fz = fz + (G3(uVel, ii, j, k) * xA) * (T3(ii, j, k) + T3(ii - 1, j, k)) * 0.5;
    double df = 0.0;
    if (p.diffKhT != 0.0) df = -p.diffKhT * xA * G2(recip_dxC, ii, j) * (T3(ii, j, k) - T3(ii - 1, j, k));
    return fz + df;
  };
  auto fmer = [&](int jj, int k, double drF) {
    const double yA = G2(dxG, i, jj) * drF * G3(hFacS, i, jj, k);
    double fm = 0.0;
    if (p.tempAdvection) fm = fm + (G3(vVel, i, jj, k) * yA) * (T3(i, jj, k) + T3(i, jj - 1, k)) * 0.5;
    double df = 0.0;
    if (p.diffKhT != 0.0) df = -p.diffKhT * yA * G2(recip_dyC, i, jj) * (T3(i, jj, k) - T3(i, jj - 1, k));
    return fm + df;
  };

  // ---- RHS pass, k = Nr..1 (temp_integrate.F k-loop)
  double fVerDn = 0.0;   // fVerT(kDown): flux through the bottom face of level k
  double rTransKp = 0.0; // rTrans of level k+1 (calc_adv_flow.F rTransKp = rTrans)
  for (int k = Nr; k >= 1; k--) {
    const long q3 = MG_I3(d, i, j, k, t);
    const double drF = f.drF[k - 1];
    const double Tk = T[q3];
    // CALC_ADV_FLOW at (i,j),(i+1,j),(i,j+1)
    const double uT0 = G3(uVel, i, j, k) * (G2(dyG, i, j) * drF * G3(hFacW, i, j, k));
    const double uT1 = G3(uVel, i + 1, j, k) * (G2(dyG, i + 1, j) * drF * G3(hFacW, i + 1, j, k));
    const double vT0 = G3(vVel, i, j, k) * (G2(dxG, i, j) * drF * G3(hFacS, i, j, k));
    const double vT1 = G3(vVel, i, j + 1, k) * (G2(dxG, i, j + 1) * drF * G3(hFacS, i, j + 1, k));
    double rTrans = 0.0, fVerUp = 0.0;
    if (k > 1) {
      const double maskUp = G3(maskC, i, j, k - 1) * G3(maskC, i, j, k);
      rTrans = G3(wVel, i, j, k) * rA * maskUp;
      if (p.tempAdvection) {   // GAD_C2_ADV_R, kM1 = k-1
        const double wT = G3(maskC, i, j, k - 1) * rTrans * (Tk + T3(i, j, k - 1)) * 0.5;
        fVerUp = fVerUp + wT * maskInC;
      }
    }
    fVerUp = fVerUp + 0.0;   // implicitDiffusion: explicit vertical diffusive flux is 0
    const double fZi = fzon(i, k, drF), fZe = fzon(i + 1, k, drF);
    const double fMi = fmer(j, k, drF), fMn = fmer(j + 1, k, drF);
    double gT = 0.0 - f.recip_hFacC[q3] * f.recip_drF[k - 1] * recip_rA *
                          ((fZe - fZi) * maskInC + (fMn - fMi) * maskInC + (fVerDn - fVerUp) * p.rkSign -
                           Tk * ((uT1 - uT0) * advFac + (vT1 - vT0) * advFac + (rTransKp - rTrans) * rAdvFac) * maskInC);
    double gtForc = 0.0;
    if (p.tempForcing && k == 1) gtForc = gtForc + f.surfaceForcingT[q] * f.recip_drF[0] * f.recip_hFacC[q3];
    gT = gT + gtForc;
    // ADAMS_BASHFORTH2(k)
    const double ab = abFac * (gT - f.gtNm1[q3]);
    f.gtNm1[q3] = gT;
    gT = gT + ab;
    // TIMESTEP_TRACER
    f.gTscr[q3] = Tk + p.deltaTtracer * gT;
    fVerDn = fVerUp;
    rTransKp = rTrans;
  }
  // ---- GAD_IMPLICIT_R + SOLVE_TRIDIAGONAL (Thomas, forward k = 1..Nr)
  double cpPrev = 0.0, ypPrev = 0.0;
  for (int k = 1; k <= Nr; k++) {
    const long q3 = MG_I3(d, i, j, k, t);
    const double rh = f.recip_hFacC[q3], rdrF = f.recip_drF[k - 1];
    double sub = 0.0, sup = 0.0;
    if (k >= 2)
      sub = -(p.deltaTtracer * G3(maskC, i, j, k - 1) * rh * rdrF *
              ((G3(IVDConvCount, i, j, k) * p.ivdc_kappa + 0.0) + p.diffKrT) * f.recip_drC[k - 1]);
    if (k <= Nr - 1)
      sup = -(p.deltaTtracer * G3(maskC, i, j, k + 1) * rh * rdrF *
              ((G3(IVDConvCount, i, j, k + 1) * p.ivdc_kappa + 0.0) + p.diffKrT) * f.recip_drC[k]);
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
  // back substitution k = Nr..1, CYCLE_TRACER into the other theta buffer
  double below = 0.0;
  for (int k = Nr; k >= 1; k--) {
    const long q3 = MG_I3(d, i, j, k, t);
    const double v = (k == Nr) ? f.gTscr[q3] : f.gTscr[q3] - f.cpScr[q3] * below;
    f.thetaNext[q3] = v;
    below = v;
  }
#undef T3
#undef G2
#undef G3
}

hipError_t launch_oceanic_phys(const Dims &d, const Params &p, const Fields &f, hipStream_t s) {
  dim3 blk(64, 4, 1), grd((d.nx + 63) / 64, (d.ny + 3) / 4, d.nTiles);
  hipLaunchKernelGGL(k_oceanic_phys, grd, blk, 0, s, d, p, f);
  return hipGetLastError();
}

hipError_t launch_temp_step(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s) {
  dim3 blk(64, 4, 1), grd((d.sNx + 63) / 64, (d.sNy + 3) / 4, d.nTiles);
  hipLaunchKernelGGL(k_temp_step, grd, blk, 0, s, d, p, f, iterPtr);
  return hipGetLastError();
}

}  // namespace mgcm
