// common.h -- shared device-side definitions for the MI355X hot-path kernels.
//
// Layout in HBM (one allocation per field, all tiles of this GPU):
//   2-D  a[t][j][i]      i in 1-OLx..sNx+OLx fastest  (reference layout, GRID.h)
//   3-D  a[t][k][j][i]   one level = one (sNx+2OLx)(sNy+2OLy) slab
// i fastest keeps every host<->device hand-off a plain memcpy of the
// reference's Fortran arrays; each thread owns an (i,j) column and marches k
// in registers (the fVerU/V ping-pong of dynamics.F:428-431).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mgcm {

struct Dims {
  int sNx, sNy, OLx, OLy, Nr, nSx, nSy, nTiles;
  int t0, nT;   // tiles this process steps (tile-sharded runs); 0, nTiles otherwise
  int nx, ny;
  long n2, n3;
};

// Run-time parameters needed on device (PARAMS.h names).
struct Params {
  double deltaTMom, deltaTFreeSurf, deltaTClock, abEps, rhoConst, gBaro;
  double viscAhD, viscAhZ, viscA4D, viscA4Z, viscAr, sideDragFactor;
  double freeSurfFac, implicSurfPress, implicDiv2DFlow, rkSign;
  double afFacMom, vfFacMom, pfFacMom, cfFacMom, foFacMom, mtFacMom;
  double cg2dNorm, cg2dTolerance_sq;
  int momAdvection, momViscosity, momForcing, useCoriolis, no_slip_sides, no_slip_bottom;
  int selectCoriScheme, momForcingOutAB, momDissip_In_AB, implicitViscosity;
  int cg2dMaxIters, cg2dUseMinResSol, cg2dNormaliseRHS, nIter0;
  // 3-D / tracer path
  double gravity, gravitySign, rhoNil, tAlpha, sBeta, ivdc_kappa, diffKhT, diffKrT, deltaTtracer;
  double recip_rSphere;
  int exactConserv, tempStepping, tempAdvection, tempForcing, implicitDiffusion, tempAdvScheme;
  int metricSphere;   // usingSphericalPolarGrid && selectMetricTerms >= 1
  double diffKhS, diffKrS;
  int saltStepping, saltAdvection, saltForcing, saltAdvScheme, multiDimAdvection, momStepping;
  // lat-lon ocean physics (tutorial_global_oce_latlon / global_ocean.90x40x15)
  int eosType;   // 0 LINEAR, 1 JMD95Z
  int allowFreezing, useRealFreshWaterFlux, useCDscheme, useGMRedi, periodicExternalForcing, nForcRec;
  double HeatCapacity_Cp, convertFW2Salt, temp_EvPrRn, salt_EvPrRn, rCD, epsAB_CD;
  double externForcingPeriod, externForcingCycle;
  double GM_background_K, GM_isopycK, GM_skewflx, GM_maxSlope, GM_Kmin_horiz, GM_Small_Number, GM_slopeSqCutoff;
  int GM_AdvForm, GM_ExtraDiag;   // bolus advective form (gmredi_calc_psi_b.F) + extra-diagonal Redi terms
  // global_ocean.90x40x15: r* non-linear free surface, JMD95P, QH / NH metric, 3-D Coriolis
  int nonlinFreeSurf, select_rStar, quasiHydrostatic, useNHMTerms, select3dCoriScheme, selectP_inEOS_Zc;
  int storePhiHyd4Phys;
  double hFacInf;
  // cubed sphere (pkg/exch2) + vector-invariant momentum (pkg/mom_vecinv)
  int vectorInvariantMomentum, selectVortScheme, selectKEscheme, upwindShear, cubeCorners;
  int staggerTimeStep, tracForcingOutAB;   // forward_step.F:1003-1036; temp_integrate.F:373-410
};

// Device pointers of every field the kernels touch.
struct Fields {
  // 1-D vertical grid
  const double *drF, *drC, *recip_drF, *recip_drC, *rF, *rC, *tRef, *sRef;
  // 2-D grid
  const double *dxF, *dyF, *dxG, *dyG, *dxC, *dyC, *dxV, *dyU, *rA, *rAw, *rAs;
  const double *recip_dxF, *recip_dyF, *recip_dxC, *recip_dyC, *recip_dxV, *recip_dyU;
  const double *recip_rA, *recip_rAw, *recip_rAs, *fCori, *Bo_surf, *recip_Bo;
  const double *tanPhiAtU, *tanPhiAtV, *maskInC, *lambdaThetaClimRelax;
  double *SST;   // interpolated by k_fields_load
  // 3-D masks
  // (hFac and the CG2D operator are rewritten every step under r*: UPDATE_R_STAR, UPDATE_CG2D)
  double *hFacC, *hFacW, *hFacS, *recip_hFacC, *recip_hFacW, *recip_hFacS;
  const double *maskC, *maskW, *maskS;
  // CG2D operator
  double *aW2d, *aS2d, *aC2d, *pW, *pS, *pC;
  // state
  double *uVel, *vVel, *wVel, *theta, *salt, *etaN;
  double *gU, *gV, *guNm1, *gvNm1;
  double *fu, *fv;
  double *etaH, *surfaceForcingT, *rhoInSitu, *IVDConvCount, *gtNm1;
  double *thetaNext, *gTscr, *cpScr;   // tracer ping-pong buffer and per-column scratch
  double *phiHydC;                     // CALC_PHI_HYD output at cell centres (k_phi_hyd)
  double *saltNext, *gsNm1, *surfaceForcingS;
  double *advScr1, *advScr2, *gAdv;     // multi-dim advection passes and its tendency
  // lat-lon ocean physics
  const double *pRef4EOS;                  // [Nr] reference pressure for the EOS (set_ref_state.F)
  const double *forcRec;                   // [6][nForcRec][tiles*n2]: SST, SSS, taux, tauy, Qnet, EmPmR
  double *Qnet, *EmPmR, *SSS, *lambdaSaltClimRelax, *etaNm1;   // 2-D
  double *sigmaR, *Kwx, *Kwy, *Kwz, *Kux, *Kvy;                // 3-D GM/Redi
  double *Kuz, *Kvz, *GM_PsiX, *GM_PsiY;                       // 3-D GM_ExtraDiag / GM_AdvForm
  double *uVelD, *vVelD, *uNM1, *vNM1, *cdU, *cdV;             // 3-D CD scheme (+ gUtmp/gVtmp scratch)
  // r* coordinate (global_ocean.90x40x15): rest-state hFac, column geometry, the r* factors
  const double *h0FacC, *h0FacW, *h0FacS;                                  // 3-D
  const double *fCoriCos, *recip_Rcol, *rSurfW, *rSurfS, *rLowW, *rLowS, *Ro_surf, *R_low;   // 2-D
  const double *phiRefC;                                                   // [Nr]: phiRef(2k)
  double *totPhiHyd, *alphaRho, *del2u, *del2v;                            // 3-D
  double *rStarFacC, *rStarFacW, *rStarFacS, *rStarExpC, *rStarExpW, *rStarExpS;   // 2-D
  double *rStarDhCDt, *rStarDhWDt, *rStarDhSDt, *PmEpR, *dEtaHdt;          // 2-D
  const double *maskInW, *maskInS;                                         // 2-D: kSurfW/S <= Nr
  double *dWtC, *dWtU, *dWtV;   // 3-D: MOM_CALC_RTRANS's dWtransC/U/V at each level (k_phi_hyd)
  // vector-invariant momentum on curvilinear / cube grids
  const double *fCoriG, *recip_rAz, *recip_dxG, *recip_dyG;   // 2-D
  const int *tileFace, *tileEdge;   // per tile: exch2_myFace, edge bits N=1 S=2 E=4 W=8
  // solver work
  double *cg2d_b, *cg2d_x;
};

#define MG_I2(d, i, j, t) \
  ((long)((i) + (d).OLx - 1) + (long)((j) + (d).OLy - 1) * (d).nx + (long)(t) * (d).n2)
#define MG_I3(d, i, j, k, t)                                                                \
  ((long)((i) + (d).OLx - 1) + (long)((j) + (d).OLy - 1) * (d).nx + (long)((k) - 1) * (d).n2 + \
   (long)(t) * (d).n3)

// Flattened, XCD-aware launch geometry.  A launch covers nz planes of ni*nj points
// (i fastest, so a wave reads contiguous memory whatever the tile width); the
// hardware deals workgroups round-robin over the 8 XCDs, so the linear block id
// is remapped to give each XCD (own L2) one contiguous run of blocks: neighbouring
// rows/levels, whose halos overlap, then hit the same L2.
#define MG_NXCD 8
__device__ __forceinline__ int mg_xcd_block() {
  const int b = (int)blockIdx.x, n = (int)gridDim.x;
  const int x = b % MG_NXCD, per = n / MG_NXCD, rem = n % MG_NXCD;
  return x * per + (x < rem ? x : rem) + b / MG_NXCD;
}
#define MG_PLANE(i0, ni, j0, nj, zvar)                                                  \
  int i, j, zvar;                                                                       \
  {                                                                                     \
    const int np_ = (ni) * (nj), nb_ = (np_ + (int)blockDim.x - 1) / (int)blockDim.x; \
    const int lb_ = mg_xcd_block();                                                     \
    const int q_ = (lb_ % nb_) * (int)blockDim.x + (int)threadIdx.x;                    \
    zvar = lb_ / nb_;                                                                   \
    if (q_ >= np_) return;                                                              \
    i = (i0) + q_ % (ni);                                                               \
    j = (j0) + q_ / (ni);                                                               \
  }
#define MG_PLANE_THREADS 256

// Column blocks for the vertical recurrences (implicit solves, column sums, scans):
// a 256-thread workgroup holds NC = 256/KP columns x KP >= Nr levels, thread
// (c, kk) = threadIdx.x = kk*NC + c, so the k-parallel loads/stores of a level are
// NC consecutive i (coalesced) and the serial part of a column runs out of LDS.
// Threads past the last column stay resident (valid = false) for the barriers.
__host__ __device__ inline int mg_col_kp(int Nr) { int kp = 1; while (kp < Nr) kp <<= 1; return kp; }
#define MG_COLS(i0, ni, j0, nj, Nr)                                                    \
  const int KP_ = mg_col_kp(Nr), NC_ = 256 / KP_;                                        \
  const int cc = (int)threadIdx.x % NC_, kk = (int)threadIdx.x / NC_;                   \
  const long col_ = (long)mg_xcd_block() * NC_ + cc;                                    \
  const long npl_ = (long)(ni) * (nj);                                                  \
  const bool valid = col_ < npl_ * d.nT;                                                \
  const int t = d.t0 + (int)(valid ? col_ / npl_ : 0);                                  \
  const int i = (i0) + (int)((valid ? col_ % npl_ : 0) % (ni));                         \
  const int j = (j0) + (int)((valid ? col_ % npl_ : 0) / (ni));
inline unsigned mg_col_blocks(int ni, int nj, int nT, int Nr) {
  const int nc = 256 / mg_col_kp(Nr);
  return (unsigned)(((long)ni * nj * nT + nc - 1) / nc);
}
inline unsigned mg_plane_blocks(int ni, int nj, int nz) {
  return (unsigned)(((ni) * (nj) + MG_PLANE_THREADS - 1) / MG_PLANE_THREADS * (nz));
}

// One tracer of TEMP_INTEGRATE / SALT_INTEGRATE (temp_integrate.F, salt_integrate.F).
struct TracerArgs {
  const double *tr;     // tracer at the start of the step (halo-exchanged)
  double *trNext;       // where CYCLE_TRACER writes the new tracer (ping-pong partner)
  double *gNm1;         // AB2 history of the tendency
  const double *sfc;    // surface forcing (surfaceForcingT/S), or null
  double diffKh, diffKr, dT;
  int advection, multiDim, useAB, forcing;
};

// Fields exchanged together by k_exchange_multi.
#define MG_XMAX 8
struct XFields {
  double *p[MG_XMAX];
  int nz[MG_XMAX];
  int n;
};

// Multi-workgroup CG2D (kernels_cg2d_mwg.hip): tables of every part (a row strip of a tile,
// one workgroup), built by build_mwg (model.hip); slot s = p*NT + tid.
struct MwgTables {
  const int *ownG;        // [G][OPT*NT] 2-D offset of the owned point (-1: none)
  const int *ownC;        // [G][OPT*NT] compact point index (exchange buffer slot)
  const unsigned *ownNb;  // [G][OPT*NT][2] LDS slots (W | E<<16), (S | N<<16)
  const unsigned *ownExp; // [G][NT] bit p set: owned point p is in another part's rings
  const int *ringG;       // [G][RPT*NT] 2-D offset of the ring-1 point (-1: none)
  const unsigned *ringNb; // [G][RPT*NT][2]
  const int *impC;        // [G][IMAX] compact index of ring-1 then ring-2 point (LDS slot NO + q)
  const int *impG;        // [G][IMAX] its 2-D offset
  const int *nImp;        // [G]
  int G, IMAX, SZ;        // parts, import capacity, LDS slots before the ZERO slot
  int pinned;             // 1: only blockIdx.x % 8 == 0 work (all parts on one XCD)
  double *xs;             // [nPts] exchange buffer of s (sc1 stores / loads)
  double *part;           // [2][3][G] workgroup partials (sc1)
  unsigned *ctr;          // [0] arrival counter, [1] timeout word (zeroed before each launch)
};

// Per-solve record written by the device CG2D (one slot per time step).
struct SolveRecord {
  double firstResidual, lastResidual, minResidualSq, rhsMax, sumRHS;
  int numIters, nIterMin;
};

}  // namespace mgcm
