// ucg2d.h -- UPDATE_CG2D (update_cg2d.F:49-199) as per-point device bodies, shared by the r*
// pass's own launches (kernels_rstar.hip) and the fold into DYNAMICS' grids (kernels_step.hip,
// MG_FUSE_OPE).
//
// The operator of step n depends only on hFac = h0Fac*rStarFac (update_r_star.F:60-92), and
// rStarFac is the one CALC_R_STAR left at the end of step n-1: nothing between the start of
// FORWARD_STEP and UPDATE_R_STAR(.TRUE.) rewrites it, and nothing there reads the operator
// (only CG2D does).  So the operator can be built at the start of the step, beside DYNAMICS,
// from h0Fac*rStarFac -- the expression UPDATE_R_STAR stores in hFac, hence the same bits.
#pragma once
#include "common.h"

namespace mgcm {

// UPDATE_CG2D part 1 (update_cg2d.F:82-143) at one 2-D point q (flat: one thread per point,
// the levels summed in k order as the column frame's thread (c, 0) does; -ffp-contract=off
// keeps faceArea*recip_dxC a separate rounding): aW2d, aS2d on 1..sNx+1 x 1..sNy+1, 0 elsewhere
__device__ __forceinline__ void ucg2d_op_point(const Dims &d, const Params &p, const Fields &f, int lb) {
  const long q = (long)lb * blockDim.x + threadIdx.x;
  if (q >= d.n2 * d.nTiles) return;
  const int t = (int)(q / d.n2);
  if (t < d.t0 || t >= d.t0 + d.nT) return;
  const long l = q % d.n2;
  const int i = (int)(l % d.nx) - d.OLx + 1, j = (int)(l / d.nx) - d.OLy + 1;
  double aW = 0.0, aS = 0.0;
  if (i >= 1 && i <= d.sNx + 1 && j >= 1 && j <= d.sNy + 1) {
    const double fw = f.rStarFacW[q], fs = f.rStarFacS[q];
    const double dyG = f.dyG[q], dxG = f.dxG[q], rdx = f.recip_dxC[q], rdy = f.recip_dyC[q];
    for (int k = 1; k <= d.Nr; k++) {
      const long q3 = MG_I3(d, i, j, k, t);
      const double drF = f.drF[k - 1];
      const double hW = f.h0FacW[q3] * fw, hS = f.h0FacS[q3] * fs;
      double faceArea = dyG * drF * hW;
      aW = aW + faceArea * rdx;
      faceArea = dxG * drF * hS;
      aS = aS + faceArea * rdy;
    }
    aW = aW * p.cg2dNorm * p.implicSurfPress * p.implicDiv2DFlow;
    aS = aS * p.cg2dNorm * p.implicSurfPress * p.implicDiv2DFlow;
  }
  f.aW2d[q] = aW;
  f.aS2d[q] = aS;
}

// UPDATE_CG2D part 2 (update_cg2d.F:144-199): aC2d on the interior, EXCH_XY_RS(aC2d)
// (halo = the source's aC, recomputed here by the same expression), and the
// preconditioner pC, pW, pS on 1..sNx+1 x 1..sNy+1 (cg2dPreCondFreq = 1)
__device__ __forceinline__ void ucg2d_p_point(const Dims &d, const Params &p, const Fields &f,
                                              const long *__restrict__ srcOf, int lb) {
  const long q = (long)lb * blockDim.x + threadIdx.x;
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

// blocks of 256 threads over every 2-D point of the tiles (both bodies)
inline int ucg2d_blocks(const Dims &d) { return (int)((d.n2 * d.nTiles + 255) / 256); }

}  // namespace mgcm
