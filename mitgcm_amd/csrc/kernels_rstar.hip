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
#include "ucg2d.h"

namespace mgcm {

// CALC_R_STAR (calc_r_star.F:95-298) in one pass per 2-D point q: the new factors on
// the reference's ranges (:111-150, rStarAreaWeight = .TRUE.), EXCH_XY_RL(rStarFacC) +
// EXCH_UV_XY_RL(rStarFacW,S) by evaluating a halo point's factor at its interior source
// (lat-lon / single facet: scalar copies), then rStarDh*Dt = (Fac - Fac_old)/dtFS and
// rStarExp = Fac/Fac_old (:283-298).  Each thread reads and writes only its own point's
// factors, so the old values need no second buffer.
// The new etaH of k_exch_etaH at point q: EXCH_XY_RL of the eta k_corr_cont left in cg2d_b
// (the interior source of a halo point; the point itself inside; etaN where neither --
// fromX: the etaN SOLVE_FOR_PRESSURE's EXCH(cg2d_x) + etaN = recip_Bo*cg2d_x leaves there,
// recip_Bo*cg2d_x of the point itself, when that launch was skipped, see one_step).
__device__ __forceinline__ double eta_exch(const Dims &d, const Fields &f, const long *srcOf, long q, int fromX) {
  const long sq = srcOf[q];
  if (sq >= 0) return f.cg2d_b[sq];
  const long l = q % d.n2;
  const int i = (int)(l % d.nx) - d.OLx + 1, j = (int)(l / d.nx) - d.OLy + 1;
  if (i >= 1 && i <= d.sNx && j >= 1 && j <= d.sNy) return f.cg2d_b[q];
  return fromX ? f.recip_Bo[q] * f.cg2d_x[q] : f.etaN[q];
}

// fuseEtaH: k_exch_etaH in the same pass (the FORWARD_STEP order exch_etaH -> CALC_R_STAR):
// each thread stores its own point's etaN, etaH, etaHnm1 (and PmEpR) and takes the etaH of
// the neighbours it reads from eta_exch, the same values k_exch_etaH stores.  The only
// cross-thread location both read and written is etaN at points neither interior nor
// mapped, which is rewritten with the value it holds.
template <bool FUSE>
__device__ __forceinline__ void calc_r_star_body(const Dims &d, const Params &p, const Fields &f,
                                                 const long *__restrict__ srcOf, int lb, int fromX) {
  const long q = (long)lb * blockDim.x + threadIdx.x;
  if (q >= d.n2 * d.nTiles) return;
  const int t = (int)(q / d.n2);
  if (t < d.t0 || t >= d.t0 + d.nT) return;
  if constexpr (FUSE) {   // k_exch_etaH (kernels_solve.hip), atInit = 0
    if (p.nonlinFreeSurf > 0 && p.useRealFreshWaterFlux) f.PmEpR[q] = -f.EmPmR[q];
    const double x = eta_exch(d, f, srcOf, q, fromX);
    f.etaHnm1[q] = f.etaH[q];
    f.etaN[q] = x;
    f.etaH[q] = x;
  }
  const long sq = srcOf[q], r = sq >= 0 ? sq : q;   // where the new value is computed
  const long l = r % d.n2;
  const int i = (int)(l % d.nx) - d.OLx + 1, j = (int)(l / d.nx) - d.OLy + 1;
  auto eta = [&](long qq) { return FUSE ? eta_exch(d, f, srcOf, qq, fromX) : f.etaH[qq]; };
  const double oc = f.rStarFacC[q], ow = f.rStarFacW[q], os = f.rStarFacS[q];
  double fc = oc, fw = ow, fs = os;
  if (i >= 0 && i <= d.sNx + 1 && j >= 0 && j <= d.sNy + 1)   // kSurfC <= Nr <=> maskInC = 1
    fc = (f.maskInC[r] != 0.0) ? (eta(r) + f.Ro_surf[r] - f.R_low[r]) * f.recip_Rcol[r] : 1.0;
  // W/S factors: at the EXCH1 source as above, or (EXCH2 topology) in place on the
  // reference's ranges, their halos then refilled through the vector map (calc_r_star())
  const long rv = p.cubeCorners ? q : r;
  const long lv = rv % d.n2;
  const int iv = (int)(lv % d.nx) - d.OLx + 1, jv = (int)(lv / d.nx) - d.OLy + 1;
  if (iv >= 1 && iv <= d.sNx + 1 && jv >= 1 && jv <= d.sNy) {
    if (f.maskInW[rv] != 0.0) {
      const double tmp = f.rSurfW[rv] - f.rLowW[rv];
      fw = (0.5 * (eta(rv - 1) * f.rA[rv - 1] + eta(rv) * f.rA[rv]) * f.recip_rAw[rv] + tmp) / tmp;
    } else {
      fw = 1.0;
    }
  }
  if (iv >= 1 && iv <= d.sNx && jv >= 1 && jv <= d.sNy + 1) {
    if (f.maskInS[rv] != 0.0) {
      const double tmp = f.rSurfS[rv] - f.rLowS[rv];
      fs = (0.5 * (eta(rv - d.nx) * f.rA[rv - d.nx] + eta(rv) * f.rA[rv]) * f.recip_rAs[rv] + tmp) / tmp;
    } else {
      fs = 1.0;
    }
  }
  f.rStarFacC[q] = fc;
  f.rStarFacW[q] = fw;
  f.rStarFacS[q] = fs;
  f.rStarDhCDt[q] = (fc - oc) / p.deltaTFreeSurf;
  f.rStarDhWDt[q] = (fw - ow) / p.deltaTFreeSurf;
  f.rStarDhSDt[q] = (fs - os) / p.deltaTFreeSurf;
  f.rStarExpC[q] = fc / oc;
  f.rStarExpW[q] = fw / ow;
  f.rStarExpS[q] = fs / os;
}
template <bool FUSE>
__global__ void __launch_bounds__(256) k_calc_r_star(Dims d, Params p, Fields f, const long *__restrict__ srcOf, int fromX) {
  calc_r_star_body<FUSE>(d, p, f, srcOf, (int)blockIdx.x, fromX);
}
// The end of FORWARD_STEP in one grid: CALC_R_STAR (with EXCH(eta) + UPDATE_ETAH, FUSE) on
// the first nbR blocks and DO_FIELDS_BLOCKING_EXCHANGES (k_exchange_multi's nbX x nz x nF
// grid, flattened) on the rest -- independent: CALC_R_STAR reads eta and writes the 2-D r*
// factors, the exchanges copy the 3-D state's halos.
template <bool FUSE>
__global__ void __launch_bounds__(256) k_rstar_exch(Dims d, Params p, Fields f, const long *__restrict__ srcOf, int nbR,
                                                    XFields x, const long *__restrict__ map, int nHalo, int *ctr, int nbX,
                                                    int nzMax, int fromX) {
  const int b = (int)blockIdx.x;
  if (b < nbR) { calc_r_star_body<FUSE>(d, p, f, srcOf, b, fromX); return; }
  const int r = b - nbR;
  exchange_multi_body(d, x, map, nHalo, ctr, r % nbX, (r / nbX) % nzMax, r / (nbX * nzMax));
}

// CALC_R_STAR (with EXCH(eta) + UPDATE_ETAH, FUSE) on the first nbR blocks and
// DO_STAGGER_FIELDS_EXCHANGES (k_exchange_mixed's nbH x nz x (1 + x.n) grid, flattened: the
// vector pair u, v and the scalar fields) on the rest, in one grid -- independent: CALC_R_STAR
// reads eta and writes the 2-D r* factors, the exchanges copy u, v, w's halos
template <bool FUSE>
__global__ void __launch_bounds__(256) k_rstar_exmix(Dims d, Params p, Fields f, const long *__restrict__ srcOf, int nbR,
                                                     int fromX, double *u, double *v, int nzUV,
                                                     const long *__restrict__ uvMap, int nU, int nV, XFields x,
                                                     const long *__restrict__ map, int nHalo, int nbH, int nzMax) {
  const int b = (int)blockIdx.x;
  if (b < nbR) { calc_r_star_body<FUSE>(d, p, f, srcOf, b, fromX); return; }
  const int r = b - nbR;
  exchange_mixed_body(d, u, v, nzUV, uvMap, nU, nV, x, map, nHalo, nullptr, r % nbH, (r / nbH) % nzMax, r / (nbH * nzMax));
}

// UPDATE_R_STAR(.TRUE.) (update_r_star.F:60-92) and UPDATE_CG2D part 1
// (update_cg2d.F:82-143) in one pass over the columns of every 2-D point (column frame,
// common.h MG_COLF): each thread rewrites hFac = h0Fac*rStarFac and recip_hFac = 1/hFac
// (where wet; USE_MASK_AND_NO_IF undefined) at its levels, k-parallel and coalesced over i,
// and stages the operator terms faceArea*recip_dx/yC of its levels in LDS; thread (c, 0)
// then sums aW2d, aS2d in k order on 1..sNx+1 x 1..sNy+1 and scales them by
// cg2dNorm*implicSurfPress*implicDiv2DFlow (0 elsewhere).
// SFP: SOLVE_FOR_PRESSURE's right-hand side (k_sfp_rhs, kernels_solve.hip) in the same
// column pass (FORWARD_STEP: UPDATE_R_STAR + UPDATE_CG2D, then CALC_DIV_GHAT): the flux terms
// read hFacW(i+1) / hFacS(j+1) of the neighbouring columns, which this pass is rewriting, so
// they are formed from h0Fac*rStarFac there (the expression that column stores: same bits).
// opIn = 0: the operator was built at the start of the step (ucg2d.h, MG_FUSE_OPE) -- hFac only.
// nbPc > 0: the operator was built in an earlier launch of the step (opIn = 0) and UPDATE_CG2D's
// preconditioner rides here, on the first nbPc logical blocks (ucg2d_p_point; the column
// frame on the rest)
template <bool SFP>
__global__ void __launch_bounds__(256) k_update_r_star_cg2d_a(Dims d, Params p, Fields f, int nc, int opIn,
                                                              const long *__restrict__ srcOf, int nbPc) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  int lb = mg_xcd_block();
  if (lb < nbPc) { ucg2d_p_point(d, p, f, srcOf, lb); return; }
  lb -= nbPc;
  MG_COLF_LB(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, nc, lb)
  const int NS = d.Nr * NC_;
  double *sW = lds, *sS = lds + NS;
  double *fE = lds + 2 * NS, *fW = lds + 3 * NS, *fN = lds + 4 * NS, *fS = lds + 5 * NS;   // SFP only
  const long q = MG_I2(d, i, j, t);
  const bool op = opIn && p.nonlinFreeSurf > 2 && i >= 1 && i <= d.sNx + 1 && j >= 1 && j <= d.sNy + 1;
  const bool inner = i >= 1 && i <= d.sNx && j >= 1 && j <= d.sNy;
  if (valid) {
    const double fc = f.rStarFacC[q], fw = f.rStarFacW[q], fs = f.rStarFacS[q];
    double fwE = 0.0, fsN = 0.0;
    if (SFP && inner) { fwE = f.rStarFacW[MG_I2(d, i + 1, j, t)]; fsN = f.rStarFacS[MG_I2(d, i, j + 1, t)]; }
    MG_COLF_K(k) {
      const long q3 = MG_I3(d, i, j, k, t);
      const double hC = f.h0FacC[q3] * fc, hW = f.h0FacW[q3] * fw, hS = f.h0FacS[q3] * fs;
      f.hFacC[q3] = hC;
      f.hFacW[q3] = hW;
      f.hFacS[q3] = hS;
      if (f.maskC[q3] != 0.0) f.recip_hFacC[q3] = 1.0 / hC;
      if (f.maskW[q3] != 0.0) f.recip_hFacW[q3] = 1.0 / hW;
      if (f.maskS[q3] != 0.0) f.recip_hFacS[q3] = 1.0 / hS;
      const int me = (k - 1) * NC_ + cc;
      if (op) {
        double faceArea = f.dyG[q] * f.drF[k - 1] * hW;
        sW[me] = faceArea * f.recip_dxC[q];
        faceArea = f.dxG[q] * f.drF[k - 1] * hS;
        sS[me] = faceArea * f.recip_dyC[q];
      }
      if (SFP) {
        if (p.useCDscheme) {
          f.uNM1[q3] = f.uVel[q3];
          f.vNM1[q3] = f.vVel[q3];
        }
        if (inner) {   // k_sfp_rhs's CALC_DIV_GHAT flux terms of level k
          const double drF = f.drF[k - 1];
          const long qE = MG_I3(d, i + 1, j, k, t), qN = MG_I3(d, i, j + 1, k, t);
          fE[me] = f.dyG[MG_I2(d, i + 1, j, t)] * drF * (f.h0FacW[qE] * fwE) * f.gU[qE] / p.deltaTMom;
          fW[me] = f.dyG[q] * drF * hW * f.gU[q3] / p.deltaTMom;
          fN[me] = f.dxG[MG_I2(d, i, j + 1, t)] * drF * (f.h0FacS[qN] * fsN) * f.gV[qN] / p.deltaTMom;
          fS[me] = f.dxG[q] * drF * hS * f.gV[q3] / p.deltaTMom;
        }
      }
    }
  }
  __syncthreads();
  if (!valid || kk != 0) return;
  if (opIn && p.nonlinFreeSurf > 2) {
    double aW = 0.0, aS = 0.0;
    if (op) {
      for (int k = 1; k <= d.Nr; k++) {
        const int me = (k - 1) * NC_ + cc;
        aW = aW + sW[me];
        aS = aS + sS[me];
      }
      aW = aW * p.cg2dNorm * p.implicSurfPress * p.implicDiv2DFlow;
      aS = aS * p.cg2dNorm * p.implicSurfPress * p.implicDiv2DFlow;
    }
    f.aW2d[q] = aW;
    f.aS2d[q] = aS;
  }
  if (SFP) sfp_rhs_column(d, p, f, q, inner, fE, fW, fN, fS, NC_, cc);
}

// UPDATE_CG2D part 2 (ucg2d.h ucg2d_p_point)
__global__ void __launch_bounds__(256) k_update_cg2d_p(Dims d, Params p, Fields f, const long *__restrict__ srcOf) {
  ucg2d_p_point(d, p, f, srcOf, (int)blockIdx.x);
}

hipError_t launch_calc_r_star(const Dims &d, const Params &p, const Fields &f, const long *srcOf, hipStream_t s,
                              bool fuseEtaH, int fromX) {
  const long n = d.n2 * d.nTiles;
  hipLaunchKernelGGL(fuseEtaH ? k_calc_r_star<true> : k_calc_r_star<false>, dim3((unsigned)((n + 255) / 256)), dim3(256),
                     0, s, d, p, f, srcOf, fromX);
  return hipGetLastError();
}

hipError_t launch_rstar_exch(const Dims &d, const Params &p, const Fields &f, const long *srcOf, bool fuseEtaH,
                             const XFields &x, const long *map, int nHalo, int *ctr, hipStream_t s, int fromX) {
  const long n = d.n2 * d.nTiles;
  const int nbR = (int)((n + 255) / 256);
  int nzMax = 1;
  for (int q = 0; q < x.n; q++) nzMax = x.nz[q] > nzMax ? x.nz[q] : nzMax;
  const int nbX = ((nHalo > 0 ? nHalo : 1) + 255) / 256;
  const unsigned nb = (unsigned)(nbR + nbX * nzMax * (x.n > 0 ? x.n : 1));
  hipLaunchKernelGGL(fuseEtaH ? k_rstar_exch<true> : k_rstar_exch<false>, dim3(nb), dim3(256), 0, s, d, p, f, srcOf, nbR, x,
                     map, nHalo, ctr, nbX, nzMax, fromX);
  return hipGetLastError();
}

hipError_t launch_rstar_exmix(const Dims &d, const Params &p, const Fields &f, const long *srcOf, bool fuseEtaH, int fromX,
                              double *u, double *v, int nzUV, const long *uvMap, int nU, int nV, const XFields &x,
                              const long *map, int nHalo, hipStream_t s) {
  const long n = d.n2 * d.nTiles;
  const int nbR = (int)((n + 255) / 256);
  int nzMax = nzUV;
  for (int q = 0; q < x.n; q++) nzMax = x.nz[q] > nzMax ? x.nz[q] : nzMax;
  const int nh = (nU + nV) > nHalo ? nU + nV : nHalo;
  const int nbH = ((nh > 0 ? nh : 1) + 255) / 256;
  const unsigned nb = (unsigned)(nbR + nbH * nzMax * (1 + x.n));
  hipLaunchKernelGGL(fuseEtaH ? k_rstar_exmix<true> : k_rstar_exmix<false>, dim3(nb), dim3(256), 0, s, d, p, f, srcOf, nbR,
                     fromX, u, v, nzUV, uvMap, nU, nV, x, map, nHalo, nbH, nzMax);
  return hipGetLastError();
}

// opEarly: the operator and preconditioner were built beside DYNAMICS (launch_dyn_thermo);
// pcHere (with opEarly): only the operator was, the preconditioner rides in this launch
hipError_t launch_update_r_star_cg2d(const Dims &d, const Params &p, const Fields &f, const long *srcOf, hipStream_t s,
                                     bool sfp, bool opEarly, bool pcHere) {
  const long n = d.n2 * d.nTiles;
  const unsigned nb = (unsigned)((n + 255) / 256);
  const long ncol = (long)d.nx * d.ny * d.nT;
  const int nArr = sfp ? 6 : 2;
  const int nc = mg_colf_nc(ncol, d.Nr, nArr);
  MG_ALLOW_LDS(k_update_r_star_cg2d_a<false>);
  MG_ALLOW_LDS(k_update_r_star_cg2d_a<true>);
  const int nbPc = (opEarly && pcHere && p.nonlinFreeSurf > 2) ? (int)nb : 0;
  hipLaunchKernelGGL(sfp ? k_update_r_star_cg2d_a<true> : k_update_r_star_cg2d_a<false>,
                     dim3(mg_colf_blocks(ncol, nc) + (unsigned)nbPc), dim3(256), mg_colf_lds(d.Nr, nc, nArr), s, d, p, f, nc,
                     opEarly ? 0 : 1, srcOf, nbPc);
  if (p.nonlinFreeSurf > 2 && !opEarly) hipLaunchKernelGGL(k_update_cg2d_p, dim3(nb), dim3(256), 0, s, d, p, f, srcOf);
  return hipGetLastError();
}

}  // namespace mgcm
