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
#include <stdlib.h>

namespace mgcm {

struct Dims {
  int sNx, sNy, OLx, OLy, Nr, nSx, nSy, nTiles;
  int t0, nT;   // tiles this process steps (tile-sharded runs); 0, nTiles otherwise
  int nx, ny;
  long n2, n3;
  long N2all, N3all;   // n2 * nTiles, n3 * nTiles: the stride of one field in its arena
};

// Every 2-D and 3-D field of the model in one list each (X-macros): the order of the
// per-kind arenas model.hip allocates (field n of a kind lives at arena + n * N2all / N3all),
// so a kernel can address any field from ONE base pointer (AR2 / AR3 below) instead of
// holding a pointer per field in scalar registers.  theta / salt and their ping-pong
// partners swap pointers every step: address them through Fields, never by arena index.
#define MG_F2D_LIST(X) X(dxF) X(dyF) X(dxG) X(dyG) X(dxC) X(dyC) X(dxV) X(dyU) X(rA) X(rAw) X(rAs) X(recip_dxF) \
    X(recip_dyF) X(recip_dxC) X(recip_dyC) X(recip_dxV) X(recip_dyU) X(recip_rA) X(recip_rAw) X(recip_rAs) \
    X(fCori) X(Bo_surf) X(recip_Bo) X(tanPhiAtU) X(tanPhiAtV) X(maskInC) X(SST) X(lambdaThetaClimRelax) X(aW2d) \
    X(aS2d) X(aC2d) X(pW) X(pS) X(pC) X(etaN) X(fu) X(fv) X(etaH) X(surfaceForcingT) X(surfaceForcingS) \
    X(cg2d_b) X(cg2d_x) X(Qnet) X(EmPmR) X(SSS) X(lambdaSaltClimRelax) X(etaNm1) X(fCoriCos) X(recip_Rcol) \
    X(rSurfW) X(rSurfS) X(rLowW) X(rLowS) X(Ro_surf) X(R_low) X(rStarFacC) X(rStarFacW) X(rStarFacS) \
    X(rStarExpC) X(rStarExpW) X(rStarExpS) X(rStarDhCDt) X(rStarDhWDt) X(rStarDhSDt) X(PmEpR) X(dEtaHdt) \
    X(maskInW) X(maskInS) X(fCoriG) X(recip_rAz) X(recip_dxG) X(recip_dyG) X(etaHnm1) X(cg2d_r) X(cg2d_s) X(cg2d_q) \
    X(cg2d_min) X(cg2d_y) X(cg2d_v)
#define MG_F3D_LIST(X) X(hFacC) X(hFacW) X(hFacS) X(recip_hFacC) X(recip_hFacW) X(recip_hFacS) X(maskC) X(maskW) \
    X(maskS) X(uVel) X(vVel) X(wVel) X(theta) X(salt) X(gU) X(gV) X(guNm1) X(gvNm1) X(rhoInSitu) X(IVDConvCount) \
    X(gtNm1) X(thetaNext) X(gTscr) X(cpScr) X(phiHydC) X(saltNext) X(gsNm1) X(advScr1) X(advScr2) X(gAdv) \
    X(sigmaR) X(Kwx) X(Kwy) X(Kwz) X(Kux) X(Kvy) X(uVelD) X(vVelD) X(uNM1) X(vNM1) X(cdU) X(cdV) X(h0FacC) \
    X(h0FacW) X(h0FacS) X(totPhiHyd) X(alphaRho) X(del2u) X(del2v) X(dWtC) X(dWtU) X(dWtV) X(Kuz) X(Kvz) \
    X(GM_PsiX) X(GM_PsiY) X(gtNm2) X(gsNm2)
#define MG_ENUM2(n) F2_##n,
#define MG_ENUM3(n) F3_##n,
enum F2Id { MG_F2D_LIST(MG_ENUM2) F2_COUNT };
enum F3Id { MG_F3D_LIST(MG_ENUM3) F3_COUNT };
#undef MG_ENUM2
#undef MG_ENUM3

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
  int cg2dUseFMA;   // CG2D in fused multiply-adds (device-order oracle: the same fma chains)
  int useSRCGSolver;   // CG2D_SR (cg2d_sr.F): single-reduction CG, k_cg2d_bxy only
  int cg2dRefOrder;    // CG2D sums in the reference's order (per-tile sequential, tile order): parity mode
  // 3-D / tracer path
  double gravity, gravitySign, rhoNil, tAlpha, sBeta, ivdc_kappa, diffKhT, diffKrT, deltaTtracer;
  double recip_rSphere;
  int exactConserv, tempStepping, tempAdvection, tempForcing, implicitDiffusion, tempAdvScheme;
  int metricSphere;   // usingSphericalPolarGrid && selectMetricTerms >= 1
  double diffKhS, diffKrS;
  int saltStepping, saltAdvection, saltForcing, saltAdvScheme, multiDimAdvection, momStepping;
  int multiDimCompressible;   // GAD_MULTIDIM_COMPRESSIBLE (GAD_OPTIONS.h)
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
  // ALLOW_ADAMSBASHFORTH_3 for the tracers (adams_bashforth3.F; momStepping off, init refuses the rest)
  double alph_AB, beta_AB;
  int useAB3;
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
  double *gtNm2, *gsNm2;                // ADAMS_BASHFORTH3's second tendency history (gtNm(:,:,:,2))
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
  double *etaHnm1;   // 2-D: etaH before UPDATE_ETAH (update_etah.F:49-53), WRITE_PICKUP's EtaH record
  const double *maskInW, *maskInS;                                         // 2-D: kSurfW/S <= Nr
  double *dWtC, *dWtU, *dWtV;   // 3-D: MOM_CALC_RTRANS's dWtransC/U/V at each level (k_phi_hyd)
  // vector-invariant momentum on curvilinear / cube grids
  const double *fCoriG, *recip_rAz, *recip_dxG, *recip_dyG;   // 2-D
  const int *tileFace, *tileEdge;   // per tile: exch2_myFace, edge bits N=1 S=2 E=4 W=8
  // solver work
  double *cg2d_b, *cg2d_x;
  double *cg2d_r, *cg2d_s, *cg2d_q;   // distributed CG2D work vectors (kernels_cg2d_dist.hip)
  double *cg2d_min;                   // its lowest-residual solution (cg2dUseMinResSol, cg2d.F:148-155, 338-369)
  double *cg2d_y, *cg2d_v;            // CG2D_SR's y = M r and v = A y (cg2d_sr.F:102-104)
  // the 2-D and 3-D arenas (MG_F2D_LIST / MG_F3D_LIST order)
  double *a2, *a3;
};
// field x at flat offset q of its kind's arena (one base pointer for every field), addressed as
// global memory: a kernel that launders the arena bases through an asm statement (k_mom_vi_m2)
// would otherwise reach them with flat instructions, which count on the LDS counter too, so
// every LDS wait after such a store waits for the store
typedef __attribute__((address_space(1))) double mg_gdouble;
#define AR2(x, q) ((mg_gdouble *)f.a2)[(long)F2_##x * d.N2all + (q)]
#define AR3(x, q) ((mg_gdouble *)f.a3)[(long)F3_##x * d.N3all + (q)]

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
// MG_PLANE with an explicit logical block id (kernels that split their grid between bodies)
#define MG_PLANE_LB(i0, ni, j0, nj, zvar, LB)                                           \
  int i, j, zvar;                                                                       \
  {                                                                                     \
    const int np_ = (ni) * (nj), nb_ = (np_ + (int)blockDim.x - 1) / (int)blockDim.x; \
    const int lb_ = (LB);                                                               \
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
// Column frame with a run-time column count: a 256-thread workgroup holds NC consecutive
// columns (NC = 16, 32 or 64) and KW = 256/NC level slots; thread (c, w) = threadIdx.x =
// w*NC + c stages levels k = w+1, w+1+KW, ... of column c (MG_COLF_K loop) into LDS slot
// (k-1)*NC + c -- coalesced over i -- and thread (c, 0) runs column c's serial recurrence
// out of LDS.  With NC = 64 the serial part of 64 columns runs in one full wave (MG_COLS
// puts 4 columns per workgroup at Nr = 50, so its serial part ran on 4 lanes of 256).
// The LDS arrays are dynamic: nArr slices of Nr*NC doubles (mg_colf_lds).
#define MG_COLF(i0, ni, j0, nj, NCv)                                                   \
  const int NC_ = (NCv), KW_ = 256 / NC_;                                              \
  const int cc = (int)threadIdx.x % NC_, kk = (int)threadIdx.x / NC_;                  \
  const long col_ = (long)mg_xcd_block() * NC_ + cc;                                   \
  const long npl_ = (long)(ni) * (nj);                                                 \
  const bool valid = col_ < npl_ * d.nT;                                               \
  const int t = d.t0 + (int)(valid ? col_ / npl_ : 0);                                 \
  const int i = (i0) + (int)((valid ? col_ % npl_ : 0) % (ni));                        \
  const int j = (j0) + (int)((valid ? col_ % npl_ : 0) / (ni));
// MG_COLF with an explicit logical block id (kernels that split their grid between bodies)
#define MG_COLF_LB(i0, ni, j0, nj, NCv, LB)                                            \
  const int NC_ = (NCv), KW_ = 256 / NC_;                                              \
  const int cc = (int)threadIdx.x % NC_, kk = (int)threadIdx.x / NC_;                  \
  const long col_ = (long)(LB) * NC_ + cc;                                             \
  const long npl_ = (long)(ni) * (nj);                                                 \
  const bool valid = col_ < npl_ * d.nT;                                               \
  const int t = d.t0 + (int)(valid ? col_ / npl_ : 0);                                 \
  const int i = (i0) + (int)((valid ? col_ % npl_ : 0) % (ni));                        \
  const int j = (j0) + (int)((valid ? col_ % npl_ : 0) / (ni));
// (the bodies keep global stores out of these loops, so that nothing orders a level's
// loads behind the previous level's stores)
#define MG_COLF_K(kvar) for (int kvar = kk + 1; kvar <= d.Nr; kvar += KW_)
// NC for a launch: 16 columns x 16 level slots (measured on LLC-90, Nr = 50: the implicit
// tracer solve 119 us at NC = 16, 201 at 32, 168 with MG_COLS' 4 columns x 64 levels; wider
// column runs cost occupancy through their LDS)
inline int mg_colf_nc(long ncols, int Nr, int nArr) {
  (void)ncols; (void)Nr; (void)nArr;
  return 16;
}
inline size_t mg_colf_lds(int Nr, int nc, int nArr) { return (size_t)nArr * Nr * nc * sizeof(double); }
// dynamic LDS above the 64 KB default needs the per-kernel attribute (set once)
#define MG_ALLOW_LDS(kern)                                                                              \
  do {                                                                                                  \
    static const bool set_ = (hipFuncSetAttribute((const void *)(kern),                                 \
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess); \
    (void)set_;                                                                                         \
  } while (0)
inline unsigned mg_colf_blocks(long ncols, int nc) { return (unsigned)((ncols + nc - 1) / nc); }
// Launch fusions of FORWARD_STEP, each switchable for A/B runs: MGCM_STEP_FUSE = bit mask of
// the enabled ones (default SFP | PHI | END | DT | ETAX): MG_FUSE_SFP CALC_DIV_GHAT in the r* column pass,
// MG_FUSE_ETA EXCH(cg2d_x) + etaN in the single-workgroup CG2D, MG_FUSE_PHI CALC_PHI_HYD +
// del2uv in one grid, MG_FUSE_END CALC_R_STAR + the blocking exchanges in one grid,
// MG_FUSE_PHYS DO_OCEANIC_PHYS + CALC_PHI_HYD in one column pass (bit-identical, but on LLC-90
// 226-313 us against 75 + 77 for the two launches: the per-point EOS loads lose their
// plane-wide parallelism inside the column frame; profiles/r03/phys/), MG_FUSE_ETAA
// SOLVE_FOR_PRESSURE's EXCH(cg2d_x) + etaN off the critical path (exactConserv: beside the
// correction step, which derives the eta it needs from cg2d_x itself; bit-identical, but the
// third stream's fork and join cost more than the launch they hide: config 2 0.343 against
// 0.330 ms/step, config 3 0.454 against 0.429; profiles/r03/fuseab/), MG_FUSE_TREX the
// tracers' halo exchange on their own stream beside the pressure solve (late join only;
// bit-identical, no measurable change on LLC-90: 1.851 against 1.851-1.854 ms/step).
// MG_FUSE_DT THERMODYNAMICS' tracer kernels folded into DYNAMICS' launches instead of a
// second stream beside them (kernels_step.hip; early fork only, small grids), MG_FUSE_ETAX
// no separate EXCH(cg2d_x) + etaN under exactConserv (one_step), MG_FUSE_OPE UPDATE_CG2D's
// operator and preconditioner in the fold's first two grids (ucg2d.h; r*, with MG_FUSE_DT),
// MG_FUSE_RING the VI path's halo-ring AB2 on the tracers' stream (late fork, one_step),
// MG_FUSE_RINGP that ring in DO_OCEANIC_PHYS's grid instead where there is no late fork
// (k_phys_ring: the staggered cube), MG_FUSE_ENDS CALC_R_STAR and
// DO_STAGGER_FIELDS_EXCHANGES' u, v, w in one grid (k_rstar_exmix: the staggered cube).
enum { MG_FUSE_SFP = 1, MG_FUSE_ETA = 2, MG_FUSE_PHI = 4, MG_FUSE_END = 8, MG_FUSE_PHYS = 16, MG_FUSE_ETAA = 32,
       MG_FUSE_TREX = 64, MG_FUSE_DT = 128, MG_FUSE_ETAX = 256, MG_FUSE_TCG = 512, MG_FUSE_OPE = 1024,
       MG_FUSE_RING = 2048, MG_FUSE_RINGP = 4096, MG_FUSE_ENDS = 8192 };
inline bool mg_fuse_on(int bit) {
  // read per call (tests switch it per model)
  const int mask = getenv("MGCM_STEP_FUSE") ? atoi(getenv("MGCM_STEP_FUSE"))
                                            : MG_FUSE_SFP | MG_FUSE_PHI | MG_FUSE_END | MG_FUSE_DT | MG_FUSE_ETAX |
                                                MG_FUSE_OPE | MG_FUSE_RING | MG_FUSE_RINGP | MG_FUSE_ENDS;
  return (mask & bit) != 0;
}
// Horizontal launch fusion of two independent latency-bound kernels into one grid: on the
// small configurations only (up to 2^21 grid points), where each launch is a few us of latency
inline bool mg_hfuse(int bit, long nx, long ny, long nT, long Nr) {
  return mg_fuse_on(bit) && nx * ny * nT * Nr <= (1L << 21);
}
inline unsigned mg_plane_blocks(int ni, int nj, int nz) {
  return (unsigned)(((ni) * (nj) + MG_PLANE_THREADS - 1) / MG_PLANE_THREADS * (nz));
}

// The serial end of SOLVE_FOR_PRESSURE's right-hand side for one column (k_sfp_rhs and the
// fused r* pass k_update_r_star_cg2d_a<SFP>): etaNm1 (CD scheme), cg2d_x = Bo_surf*etaN and
// cg2d_b = CALC_DIV_GHAT's k = Nr..1 sum of the staged flux terms + the free-surface term.
__device__ __forceinline__ void sfp_rhs_column(const Dims &d, const Params &p, const Fields &f, long q, bool inner,
                                               const double *sE, const double *sW, const double *sN, const double *sS,
                                               int NC_, int cc) {
  if (p.useCDscheme) f.etaNm1[q] = f.etaN[q];
  f.cg2d_x[q] = f.Bo_surf[q] * f.etaN[q];
  double b = 0.0;
  if (inner) {
    if (p.useRealFreshWaterFlux) {
      const double tmpFac = p.freeSurfFac * (1.0 / p.rhoConst) * p.implicDiv2DFlow;
      b = tmpFac * f.rA[q] * f.EmPmR[q] / p.deltaTMom * f.maskInC[q];
    }
    for (int k2 = d.Nr; k2 >= 1; k2--) {
      const int s2 = (k2 - 1) * NC_ + cc;
      b = b + sE[s2] - sW[s2];
      b = b + sN[s2] - sS[s2];
    }
    // solve_for_pressure.F:214-236 (linear free surface): etaH with exactConserv, else etaN
    b = b - p.freeSurfFac * f.rA[q] / p.deltaTMom / p.deltaTFreeSurf * (p.exactConserv ? f.etaH[q] : f.etaN[q]);
  }
  f.cg2d_b[q] = b;
}

// One tracer of TEMP_INTEGRATE / SALT_INTEGRATE (temp_integrate.F, salt_integrate.F).
struct TracerArgs {
  const double *tr;     // tracer at the start of the step (halo-exchanged)
  double *trNext;       // where CYCLE_TRACER writes the new tracer (ping-pong partner)
  double *gNm1;         // AB2 history of the tendency
  double *scr;          // T* for the implicit vertical solve (gTscr for theta, cpScr for salt)
  double *cp;           // the Thomas sweep's c' (k_tracer_march2<true>; advScr1 / advScr2, unused without
                        // multi-dimensional advection), or null
  const double *sfc;    // surface forcing (surfaceForcingT/S), or null
  double diffKh, diffKr, dT;
  int advection, multiDim, useAB, forcing;
  int limiter;          // multi-dim face fluxes: 1 DST3FL (scheme 33), 0 DST3 (scheme 30)
  int scheme;           // the advection scheme (2 C2, 3 U3, 4 C4 inside GAD_CALC_RHS; 30/33 multi-dim)
  double *gNm2;         // ADAMS_BASHFORTH3: gtNm(:,:,:,2) (gNm1 is slot 1)
};

// Fields exchanged together by k_exchange_multi.
#define MG_XMAX 8
struct XFields {
  double *p[MG_XMAX];
  int nz[MG_XMAX];
  int n;
};

// DO_FIELDS_BLOCKING_EXCHANGES' copies for one (halo block hb, level k, field fi) of
// k_exchange_multi's grid; the block (0,0,0) also advances the step counters (the last
// kernel of a step: nothing later in the step reads them).
__device__ __forceinline__ void exchange_multi_body(const Dims &d, const XFields &x, const long *__restrict__ map,
                                                    int nHalo, int *ctr, int hb, int k, int fi) {
  const int h = hb * (int)blockDim.x + (int)threadIdx.x;
  if (ctr && h == 0 && k == 0 && fi == 0) { ctr[0] += 1; ctr[1] += 1; }
  if (h >= nHalo || fi >= x.n || k >= x.nz[fi]) return;
  const long dst = map[2 * h], src = map[2 * h + 1];
  const long dt = dst / d.n2, dl = dst % d.n2, st = src / d.n2, sl = src % d.n2;
  const long lvl = (long)d.n2 * x.nz[fi];
  double *a = x.p[fi];
  a[dt * lvl + (long)k * d.n2 + dl] = a[st * lvl + (long)k * d.n2 + sl];
}

// k_exchange_mixed's copies for one (halo block hb, level k, slice z) of its grid: z = 0 the
// vector pair u, v through the vector map (codes: +-(source+1), v's sources offset by the
// 2-D size of every tile), z = 1.. the scalar field z-1 through the scalar map; the block
// (0,0,0) advances the step counters when ctr is given.
__device__ __forceinline__ void exchange_mixed_body(const Dims &d, double *u, double *v, int nzUV,
                                                    const long *__restrict__ uvMap, int nU, int nV, const XFields &x,
                                                    const long *__restrict__ map, int nHalo, int *ctr, int hb, int k,
                                                    int z) {
  const int h = hb * (int)blockDim.x + (int)threadIdx.x;
  if (ctr && h == 0 && k == 0 && z == 0) { ctr[0] += 1; ctr[1] += 1; }
  if (z == 0) {
    if (h >= nU + nV || k >= nzUV) return;
    const long dst = uvMap[2 * h], code = uvMap[2 * h + 1];
    const long N2 = d.n2 * d.nTiles, s = (code > 0 ? code : -code) - 1;
    const long n3 = d.n2 * nzUV, lvl = (long)k * d.n2;
    auto at = [&](long g) -> long { return (g / d.n2) * n3 + lvl + g % d.n2; };
    const double val = s < N2 ? u[at(s)] : v[at(s - N2)];
    (h < nU ? u : v)[at(dst)] = code > 0 ? val : -val;
    return;
  }
  const int fi = z - 1;
  if (h >= nHalo || fi >= x.n || k >= x.nz[fi]) return;
  const long dst = map[2 * h], src = map[2 * h + 1];
  const long dt = dst / d.n2, dl = dst % d.n2, st = src / d.n2, sl = src % d.n2;
  const long lvl = (long)d.n2 * x.nz[fi];
  double *a = x.p[fi];
  a[dt * lvl + (long)k * d.n2 + dl] = a[st * lvl + (long)k * d.n2 + sl];
}

// Multi-workgroup CG2D (kernels_cg2d_mwg.hip): tables of every part (a row strip of a tile,
// one workgroup), built by build_mwg (model.hip); slot s = p*NT + tid.
struct MwgTables {
  const int *ownG;        // [G][OPT*NT] 2-D offset of the owned point (-1: none)
  const int *ownC;        // [G][OPT*NT] compact point index (exchange buffer slot)
  const unsigned *ownNb;  // [G][OPT*NT][2] LDS slots (W | E<<16), (S | N<<16)
  const unsigned *ownExp; // [G][NT] bit p set: owned point p is in another part's rings
  const int *ringG;       // [G][RPT*NT] 2-D offset of the ring-1 point (-1: none)
  const unsigned *ringNb; // [G][RPT*NT][2]
  const int *impC;        // [G][IMAX] export slot of ring-1 then ring-2 point (LDS slot NO + q)
  const int *impG;        // [G][IMAX] its 2-D offset
  const int *nImp;        // [G]
  int G, IMAX, SZ;        // parts, import capacity, LDS slots before the ZERO slot
  int nExp;               // exported points (the xs granule pairs of one export buffer)
  int pinned;             // 1: only blockIdx.x % 8 == 0 work (all parts on one XCD)
  int sys;                // 1: the hand-off block is shared across processes (system scope)
  int partsPerTile;       // parts of tile t: t*partsPerTile .. (t+1)*partsPerTile - 1
  int exclusive;          // 1: every part claims its CU's whole LDS (no co-resident workgroups)
  // hand-off state, one block zeroed before each launch (hsBytes from ctr): granules of
  // {tag = phase + 1 (32 bits), half of an f64 (32 bits)}, two per value
  unsigned *ctr;          // [1] timeout word (hand-off block, shared by every launch of the solve)
  unsigned *epoch;        // launch epoch of THIS process's launches (its own memory, never shared):
                          // read by its parts at their start, advanced by its first part at the end
  unsigned long long *part;   // [2 parities][3 values][G][2] workgroup partials
  unsigned long long *xs;     // [2 buffers][exported points][2] q = M r (CG2D_SR: r, q, v) of the points
                              // other parts' rings hold (the standard solve uses buffer 0 only)
  size_t hsBytes;
};

// MONITOR dynstat on the device (kernels_monitor.hip): one field's arrays; arr3d / hf3d:
// 3-D (tile stride n3, level stride n2) or 2-D (tile stride n2)
struct MonSpec {
  const double *arr, *hfac, *mask, *area, *dr;
  int nz, arr3d, hf3d;
};
constexpr int MON_NF = 6, MON_NV = 6;   // eta, u, v, w, theta, salt; plane values nb, del2, vol, sum, min, max
struct MonSpecs {
  MonSpec s[MON_NF];
  double mean[MON_NF];
};

// Per-solve record written by the device CG2D (one slot per time step).
struct SolveRecord {
  double firstResidual, lastResidual, minResidualSq, rhsMax, sumRHS;
  int numIters, nIterMin;
};

}  // namespace mgcm
