// kernels_rstar.hip -- the r* coordinate of the non-linear free surface on the MI355X
// (nonlinFreeSurf = 4, select_rStar = 2; BASELINE config 2, global_ocean.90x40x15).
//
// Reference: model/src/calc_r_star.F:55-298   (rStarFac from etaH, EXCH, rStarExp/DhDt)
//            model/src/update_r_star.F:48-131 (hFac = h0Fac*rStarFac and reciprocals)
//            model/src/update_cg2d.F:49-199   (CG2D operator + preconditioner from hFac)
//
// Every kernel is elementwise or a short per-column sum over a 2-D field of a few
// thousand points: latency/launch bound.  Halo points are filled from their interior
// source (srcOf, the EXCH map of the tile topology) inside the same pass, because
// EXCH copies values that are computed by the same expression as the source's.
#include "common.h"

namespace mgcm {

// CALC_R_STAR part 1: keep the old factors (rStarExp = rStarFac, calc_r_star.F:101-109)
// and compute the new ones on the reference's ranges (:111-150); rStarAreaWeight = .TRUE.
__global__ void __launch_bounds__(256) k_calc_r_star_a(Dims d, Params p, Fields f) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= d.n2 * d.nTiles) return;
  const int t = (int)(q / d.n2);
  if (t < d.t0 || t >= d.t0 + d.nT) return;
  const long l = q % d.n2;
  const int i = (int)(l % d.nx) - d.OLx + 1, j = (int)(l / d.nx) - d.OLy + 1;
  f.rStarExpC[q] = f.rStarFacC[q];
  f.rStarExpW[q] = f.rStarFacW[q];
  f.rStarExpS[q] = f.rStarFacS[q];
  const double *eta = f.etaH;
  const int Nr = d.Nr;
  (void)p;
  if (i >= 0 && i <= d.sNx + 1 && j >= 0 && j <= d.sNy + 1) {
    // kSurfC <= Nr  <=>  maskInC = 1 (ini_masks_etc.F)
    f.rStarFacC[q] = (f.maskInC[q] != 0.0) ? (eta[q] + f.Ro_surf[q] - f.R_low[q]) * f.recip_Rcol[q] : 1.0;
  }
  if (i >= 1 && i <= d.sNx + 1 && j >= 1 && j <= d.sNy) {
    const long w = q - 1;
    // kSurfW <= Nr  <=>  some level of hFacW is wet  <=>  maskW(k=kSurfW) = 1; use h0FacW
    bool wet = false;
    for (int k = 1; k <= Nr && !wet; k++) wet = f.h0FacW[MG_I3(d, i, j, k, t)] != 0.0;
    if (wet) {
      const double tmp = f.rSurfW[q] - f.rLowW[q];
      f.rStarFacW[q] = (0.5 * (eta[w] * f.rA[w] + eta[q] * f.rA[q]) * f.recip_rAw[q] + tmp) / tmp;
    } else {
      f.rStarFacW[q] = 1.0;
    }
  }
  if (i >= 1 && i <= d.sNx && j >= 1 && j <= d.sNy + 1) {
    const long s = q - d.nx;
    bool wet = false;
    for (int k = 1; k <= Nr && !wet; k++) wet = f.h0FacS[MG_I3(d, i, j, k, t)] != 0.0;
    if (wet) {
      const double tmp = f.rSurfS[q] - f.rLowS[q];
      f.rStarFacS[q] = (0.5 * (eta[s] * f.rA[s] + eta[q] * f.rA[q]) * f.recip_rAs[q] + tmp) / tmp;
    } else {
      f.rStarFacS[q] = 1.0;
    }
  }
}

// CALC_R_STAR part 2: EXCH_XY_RL(rStarFacC) + EXCH_UV_XY_RL(rStarFacW,S) (halo from the
// interior source; lat-lon / single-facet: scalar copies) and the expansion ratios
// rStarDh*Dt = (Fac - Fac_old)/deltaTFreeSurf, rStarExp = Fac/Fac_old (:283-298).
__global__ void __launch_bounds__(256) k_calc_r_star_b(Dims d, Params p, Fields f, const long *__restrict__ srcOf) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= d.n2 * d.nTiles) return;
  const int t = (int)(q / d.n2);
  if (t < d.t0 || t >= d.t0 + d.nT) return;
  const long sq = srcOf[q];
  double fc = f.rStarFacC[q], fw = f.rStarFacW[q], fs = f.rStarFacS[q];
  if (sq >= 0) {
    fc = f.rStarFacC[sq]; fw = f.rStarFacW[sq]; fs = f.rStarFacS[sq];
    f.rStarFacC[q] = fc; f.rStarFacW[q] = fw; f.rStarFacS[q] = fs;
  }
  const double oc = f.rStarExpC[q], ow = f.rStarExpW[q], os = f.rStarExpS[q];
  f.rStarDhCDt[q] = (fc - oc) / p.deltaTFreeSurf;
  f.rStarDhWDt[q] = (fw - ow) / p.deltaTFreeSurf;
  f.rStarDhSDt[q] = (fs - os) / p.deltaTFreeSurf;
  f.rStarExpC[q] = fc / oc;
  f.rStarExpW[q] = fw / ow;
  f.rStarExpS[q] = fs / os;
}

// UPDATE_R_STAR(.TRUE.): hFac = h0Fac*rStarFac, recip_hFac = 1/hFac where wet
// (USE_MASK_AND_NO_IF undefined: dry points keep their reciprocal, 0).
__global__ void __launch_bounds__(256) k_update_r_star(Dims d, Fields f) {
  MG_PLANE(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, z)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  const long q3 = MG_I3(d, i, j, k, t), q2 = MG_I2(d, i, j, t);
  const double hC = f.h0FacC[q3] * f.rStarFacC[q2];
  const double hW = f.h0FacW[q3] * f.rStarFacW[q2];
  const double hS = f.h0FacS[q3] * f.rStarFacS[q2];
  f.hFacC[q3] = hC;
  f.hFacW[q3] = hW;
  f.hFacS[q3] = hS;
  if (f.maskC[q3] != 0.0) f.recip_hFacC[q3] = 1.0 / hC;
  if (f.maskW[q3] != 0.0) f.recip_hFacW[q3] = 1.0 / hW;
  if (f.maskS[q3] != 0.0) f.recip_hFacS[q3] = 1.0 / hS;
}

// UPDATE_CG2D part 1 (update_cg2d.F:82-143): aW2d, aS2d = Sum_k faceArea*recip_dx/yC on
// 1..sNx+1 x 1..sNy+1 (in k order), scaled by cg2dNorm*implicSurfPress*implicDiv2DFlow;
// 0 elsewhere.
__global__ void __launch_bounds__(256) k_update_cg2d_a(Dims d, Params p, Fields f) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= d.n2 * d.nTiles) return;
  const int t = (int)(q / d.n2);
  if (t < d.t0 || t >= d.t0 + d.nT) return;
  const long l = q % d.n2;
  const int i = (int)(l % d.nx) - d.OLx + 1, j = (int)(l / d.nx) - d.OLy + 1;
  double aW = 0.0, aS = 0.0;
  if (i >= 1 && i <= d.sNx + 1 && j >= 1 && j <= d.sNy + 1) {
    for (int k = 1; k <= d.Nr; k++) {
      const long q3 = MG_I3(d, i, j, k, t);
      double faceArea = f.dyG[q] * f.drF[k - 1] * f.hFacW[q3];
      aW = aW + faceArea * f.recip_dxC[q];
      faceArea = f.dxG[q] * f.drF[k - 1] * f.hFacS[q3];
      aS = aS + faceArea * f.recip_dyC[q];
    }
    aW = aW * p.cg2dNorm * p.implicSurfPress * p.implicDiv2DFlow;
    aS = aS * p.cg2dNorm * p.implicSurfPress * p.implicDiv2DFlow;
  }
  f.aW2d[q] = aW;
  f.aS2d[q] = aS;
}

// UPDATE_CG2D part 2 (update_cg2d.F:144-199): aC2d on the interior, EXCH_XY_RS(aC2d)
// (halo = the source's aC, recomputed here by the same expression), and the
// preconditioner pC, pW, pS on 1..sNx+1 x 1..sNy+1 (cg2dPreCondFreq = 1).
__global__ void __launch_bounds__(256) k_update_cg2d_p(Dims d, Params p, Fields f, const long *__restrict__ srcOf) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= d.n2 * d.nTiles) return;
  const int t = (int)(q / d.n2);
  if (t < d.t0 || t >= d.t0 + d.nT) return;
  const long l = q % d.n2;
  const int i = (int)(l % d.nx) - d.OLx + 1, j = (int)(l / d.nx) - d.OLy + 1;
  const long nx = d.nx;
  auto aCat = [&](long r) {   // aC2d at an interior point r
    return -(f.aW2d[r] + f.aW2d[r + 1] + f.aS2d[r] + f.aS2d[r + nx] +
             p.freeSurfFac * p.cg2dNorm * f.recip_Bo[r] * f.rA[r] / p.deltaTMom / p.deltaTFreeSurf);
  };
  auto aCx = [&](long r) {    // after EXCH: interior value, or the interior source's
    const long s = srcOf[r];
    return aCat(s >= 0 ? s : r);
  };
  const bool interior = i >= 1 && i <= d.sNx && j >= 1 && j <= d.sNy;
  const long sq = srcOf[q];
  if (interior || sq >= 0) f.aC2d[q] = aCat(sq >= 0 ? sq : q);
  if (i >= 1 && i <= d.sNx + 1 && j >= 1 && j <= d.sNy + 1) {
    const double aC = aCx(q), aCw = aCx(q - 1), aCs = aCx(q - nx);
    f.pC[q] = (aC == 0.0) ? 1.0 : 1.0 / aC;
    const double pWt = aC + aCw;
    if (pWt == 0.0) f.pW[q] = 0.0;
    else { const double dd = 0.51 * pWt; f.pW[q] = -f.aW2d[q] / (dd * dd); }   // cg2dpcOffDFac = 0.51
    const double pSt = aC + aCs;
    if (pSt == 0.0) f.pS[q] = 0.0;
    else { const double dd = 0.51 * pSt; f.pS[q] = -f.aS2d[q] / (dd * dd); }
  }
}

hipError_t launch_calc_r_star(const Dims &d, const Params &p, const Fields &f, const long *srcOf, hipStream_t s) {
  const long n = d.n2 * d.nTiles;
  const unsigned nb = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_calc_r_star_a, dim3(nb), dim3(256), 0, s, d, p, f);
  hipLaunchKernelGGL(k_calc_r_star_b, dim3(nb), dim3(256), 0, s, d, p, f, srcOf);
  return hipGetLastError();
}

hipError_t launch_update_r_star_cg2d(const Dims &d, const Params &p, const Fields &f, const long *srcOf, hipStream_t s) {
  hipLaunchKernelGGL(k_update_r_star, dim3(mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr)), dim3(MG_PLANE_THREADS), 0, s, d, f);
  if (p.nonlinFreeSurf > 2) {
    const long n = d.n2 * d.nTiles;
    const unsigned nb = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_update_cg2d_a, dim3(nb), dim3(256), 0, s, d, p, f);
    hipLaunchKernelGGL(k_update_cg2d_p, dim3(nb), dim3(256), 0, s, d, p, f, srcOf);
  }
  return hipGetLastError();
}

}  // namespace mgcm
