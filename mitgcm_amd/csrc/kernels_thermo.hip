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
// k_temp_rhs runs one thread per interior (i,j,k) point: both vertical faces of
// the level (the fVerT(kUp/kDown) ping-pong of temp_integrate.F) and the four
// horizontal faces are recomputed from the neighbours' state with the
// reference's operand order (bit-exact under -ffp-contract=off).  k_temp_impl
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

// GAD_CALC_RHS + forcing + AB2 + TIMESTEP_TRACER for one interior (i,j,k) point:
// writes gtNm1 and gTscr = theta + dTtracer*gT (the right-hand side of the
// implicit vertical solve).
__global__ void __launch_bounds__(256) k_temp_rhs(Dims d, Params p, Fields f, const int *iterPtr) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x) + 1;
  const int j = (int)(blockIdx.y * blockDim.y + threadIdx.y) + 1;
  const int t = (int)blockIdx.z / d.Nr;
  const int k = (int)blockIdx.z % d.Nr + 1;
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
  const double drF = f.drF[k - 1];
  // west / south face fluxes of the column (fZon, fMer): GAD_C2_ADV_X/Y + GAD_DIFF_X/Y
  auto fzon = [&](int ii) {
    const double xA = G2(dyG, ii, j) * drF * G3(hFacW, ii, j, k);
    double fz = 0.0;
    if (p.tempAdvection) fz = fz + (G3(uVel, ii, j, k) * xA) * (T3(ii, j, k) + T3(ii - 1, j, k)) * 0.5;
    double df = 0.0;
    if (p.diffKhT != 0.0) df = -p.diffKhT * xA * G2(recip_dxC, ii, j) * (T3(ii, j, k) - T3(ii - 1, j, k));
    return fz + df;
  };
  auto fmer = [&](int jj) {
    const double yA = G2(dxG, i, jj) * drF * G3(hFacS, i, jj, k);
    double fm = 0.0;
    if (p.tempAdvection) fm = fm + (G3(vVel, i, jj, k) * yA) * (T3(i, jj, k) + T3(i, jj - 1, k)) * 0.5;
    double df = 0.0;
    if (p.diffKhT != 0.0) df = -p.diffKhT * yA * G2(recip_dyC, i, jj) * (T3(i, jj, k) - T3(i, jj - 1, k));
    return fm + df;
  };
  // CALC_ADV_FLOW rTrans of level kk (0 at the surface and below the bottom level)
  auto rtrans = [&](int kk) {
    if (kk <= 1 || kk > Nr) return 0.0;
    const double maskUp = G3(maskC, i, j, kk - 1) * G3(maskC, i, j, kk);
    return G3(wVel, i, j, kk) * rA * maskUp;
  };
  // fVerT through the top face of level kk: GAD_C2_ADV_R (k >= 2) + explicit diffusive flux (0)
  auto fvert = [&](int kk, double rTr) {
    double fv = 0.0;
    if (kk >= 2 && kk <= Nr && p.tempAdvection) {
      const double wT = G3(maskC, i, j, kk - 1) * rTr * (T3(i, j, kk) + T3(i, j, kk - 1)) * 0.5;
      fv = fv + wT * maskInC;
    }
    return fv + 0.0;
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
#undef T3
#undef G2
#undef G3
}

// GAD_IMPLICIT_R (implicitDiffusion) + SOLVE_TRIDIAGONAL (Thomas) + CYCLE_TRACER,
// one thread per interior column; writes the new theta into thetaNext.
__global__ void __launch_bounds__(256) k_temp_impl(Dims d, Params p, Fields f) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x) + 1;
  const int j = (int)(blockIdx.y * blockDim.y + threadIdx.y) + 1;
  const int t = (int)blockIdx.z;
  if (i > d.sNx || j > d.sNy) return;
  const int Nr = d.Nr;
#define G3(a, ii, jj, kk) f.a[MG_I3(d, ii, jj, kk, t)]
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
  double below = 0.0;
  for (int k = Nr; k >= 1; k--) {
    const long q3 = MG_I3(d, i, j, k, t);
    const double v = (k == Nr) ? f.gTscr[q3] : f.gTscr[q3] - f.cpScr[q3] * below;
    f.thetaNext[q3] = v;
    below = v;
  }
#undef G3
}

hipError_t launch_oceanic_phys(const Dims &d, const Params &p, const Fields &f, hipStream_t s) {
  dim3 blk(64, 4, 1), grd((d.nx + 63) / 64, (d.ny + 3) / 4, d.nTiles);
  hipLaunchKernelGGL(k_oceanic_phys, grd, blk, 0, s, d, p, f);
  return hipGetLastError();
}

hipError_t launch_temp_step(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s) {
  dim3 blk(64, 4, 1), grd((d.sNx + 63) / 64, (d.sNy + 3) / 4, d.nTiles * d.Nr);
  hipLaunchKernelGGL(k_temp_rhs, grd, blk, 0, s, d, p, f, iterPtr);
  dim3 cgrd((d.sNx + 63) / 64, (d.sNy + 3) / 4, d.nTiles);
  hipLaunchKernelGGL(k_temp_impl, cgrd, blk, 0, s, d, p, f);
  return hipGetLastError();
}

}  // namespace mgcm
