// kernels_step.hip -- DYNAMICS and THERMODYNAMICS in one translation unit, and the launches
// that fold the two into shared grids.
//
// forward_step.F:732-760 runs THERMODYNAMICS then DYNAMICS; neither reads what the other
// writes (THERMODYNAMICS: the tracers' other buffers, their AB histories and T* scratch;
// DYNAMICS: phiHyd, gU/gV, the momentum AB histories, the CD-scheme fields), so on a small
// grid -- where every launch is a few microseconds of latency and one kernel cannot fill the
// chip -- their kernels of the same depth share one grid (horizontal launch fusion, split by
// logical block id as k_phi_del2 does) instead of running on two streams joined by events.
// The default layout (k_dt_l1..l3, config 2: 0.3097 against 0.3218 ms/step for the layout
// below it and 0.334 for two streams):
//
//   1: GMREDI_CALC_TENSOR | CALC_PHI_HYD | MOM del2 (biharmonic)
//   2: MOM_FLUXFORM+TIMESTEP (U and V halves) | GAD_CALC_RHS+AB2+TIMESTEP (theta) | (salt)
//   3: CD_CODE_SCHEME | GAD_IMPLICIT_R + SOLVE_TRIDIAGONAL (theta) | (salt)
//
// and the front/back layout (k_dt_front / k_dt_back, MGCM_DT_LAYOUT=2): [CALC_PHI_HYD | del2 |
// rhs theta | rhs salt], [MOM U | V | implicit theta | salt], then the CD scheme.  Outside the
// fold, on the small grids: GMREDI_CALC_TENSOR beside CALC_PHI_HYD (launch_gm_phi) and both
// tracers per launch (launch_tracer_hpair) for the staggered step.
//
// Every body is the same device function the separate kernels run, so the results are the
// same bits.  The two source files are included rather than linked: hipcc builds without
// relocatable device code, and the fused kernels need both files' bodies.
#include "kernels_dyn.hip"
#include "kernels_thermo.hip"
#include "ucg2d.h"

namespace mgcm {

// CALC_PHI_HYD | del2uv | rhs(theta) | rhs(salt): logical blocks [0, nbPhi) phi's column frame,
// then nbDel del2uv planes, then nbTr planes of each tracer (barriers stay block-uniform)
template <bool GM>
__global__ void __launch_bounds__(256) k_dt_front(Dims d, Params p, Fields f, TracerArgs aT, TracerArgs aS,
                                                  const int *iterPtr, int nc, int nbPhi, int nbDel, int nbTr) {
  int lb = mg_xcd_block();
  if (lb < nbPhi) { phi_hyd_body(d, p, f, nc, lb); return; }
  lb -= nbPhi;
  if (lb < nbDel) { del2uv_body(d, p, f, lb); return; }
  lb -= nbDel;
  if (lb < nbTr) tracer_rhs_body_br<GM>(d, p, f, aT, iterPtr, lb);
  else tracer_rhs_body_br<GM>(d, p, f, aS, iterPtr, lb - nbTr);
}

// MOM_FLUXFORM U | V (k_mom_step_uv's split: even logical blocks U, odd V) | implicit solve
// (theta) | (salt)
__global__ void __launch_bounds__(256) k_dt_back(Dims d, Params p, Fields f, TracerArgs aT, TracerArgs aS,
                                                 const int *iterPtr, int nc, int nbMom, int nbImp) {
  int lb = mg_xcd_block();
  if (lb < nbMom) {
    if (lb & 1) mom_step_point<false, 2>(d, p, f, iterPtr, lb >> 1);
    else mom_step_point<false, 1>(d, p, f, iterPtr, lb >> 1);
    return;
  }
  lb -= nbMom;
  if (lb < nbImp) tracer_impl_body<false>(d, p, f, aT, nc, lb);
  else tracer_impl_body<false>(d, p, f, aS, nc, lb - nbImp);
}

// The default layout (MGCM_DT_LAYOUT=3; 2 = front/back above): GMREDI_CALC_TENSOR leaves
// DO_OCEANIC_PHYS' launch for the first grid (it and CALC_PHI_HYD both read only DO_OCEANIC_PHYS'
// rhoInSitu / sigmaR), the right-hand sides (which read the tensor) move one grid later beside
// the momentum tendencies, the implicit solves beside the CD scheme:
//   1: GMREDI_CALC_TENSOR | CALC_PHI_HYD | del2uv
//   2: MOM_FLUXFORM U | V | rhs(theta) | rhs(salt)
//   3: CD_CODE_SCHEME | implicit solve (theta) | (salt)
// and under r* with MG_FUSE_OPE UPDATE_CG2D's operator (nbOp blocks, ucg2d.h) and its
// preconditioner (nbPc blocks) at the head of 2 and 3 (MGCM_OPE_AT=1: 1 and 2) -- the
// operator of the step, built early
// the fused grids' logical-block order: the longest bodies (CALC_PHI_HYD's and the implicit
// solves' column sweeps, the tracers' right-hand sides) first, so they are not the dispatch's
// tail (config 2: 0.2893-0.2897 against 0.2906-0.2911 ms/step for the order listed above,
// alternating on one box, the fused grids 54.4 against 55.8 us; rocprofv3 on another box, the
// three grids 51.7-52.5 against 53.8-54.0 us, each grid faster, profiles/r06/dtorder/);
// MGCM_DT_LAYOUT=4 runs the listed order
static int dt_long_first() {
  const char *e = getenv("MGCM_DT_LAYOUT");   // read per launch (A/B runs)
  return !(e && atoi(e) == 4);
}
__global__ void __launch_bounds__(256) k_dt_l1(Dims d, Params p, Fields f, int nc, int nbGm, int nbPhi, int nbOp, int lf) {
  int lb = mg_xcd_block();
  if (lf) {   // long first: CALC_PHI_HYD's column sweeps at the head of the dispatch
    if (lb < nbPhi) { phi_hyd_body(d, p, f, nc, lb); return; }
    lb -= nbPhi;
    if (lb < nbOp) { ucg2d_op_point(d, p, f, lb); return; }
    lb -= nbOp;
    if (lb < nbGm) { gm_tensor_body(d, p, f, lb); return; }
    del2uv_body(d, p, f, lb - nbGm);
    return;
  }
  if (lb < nbOp) { ucg2d_op_point(d, p, f, lb); return; }
  lb -= nbOp;
  if (lb < nbGm) { gm_tensor_body(d, p, f, lb); return; }
  lb -= nbGm;
  if (lb < nbPhi) { phi_hyd_body(d, p, f, nc, lb); return; }
  del2uv_body(d, p, f, lb - nbPhi);
}
static void phi_frame(const Dims &d, const Params &p, int &nc, int &nArr, int &nb);
// k_dt_l1 with CALC_PHI_HYD's flat per-column pass (kernels_dyn.hip phi_flat_body)
template <bool RS, bool QH>
__global__ void __launch_bounds__(256) k_dt_l1f(Dims d, Params p, Fields f, int nbGm, int nbPhi, int nbOp) {
  int lb = mg_xcd_block();
  if (lb < nbOp) { ucg2d_op_point(d, p, f, lb); return; }
  lb -= nbOp;
  if (lb < nbGm) { gm_tensor_body(d, p, f, lb); return; }
  lb -= nbGm;
  if (lb < nbPhi) { phi_flat_body<RS, QH>(d, p, f, lb); return; }
  del2uv_body(d, p, f, lb - nbPhi);
}
// launch [UPDATE_CG2D operator (nbOp blocks, 0 = none) | GMREDI_CALC_TENSOR | CALC_PHI_HYD |
// del2uv (nbDel blocks, 0 = none)]
static void launch_l1(const Dims &d, const Params &p, const Fields &f, int nbDel, hipStream_t s, int nbOp = 0) {
  const int nbGm = (int)mg_plane_blocks(d.nx - 2, d.ny - 2, d.nT * d.Nr);
  if (phi_flat_on(p)) {
    const bool rs = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
    const bool qh = p.quasiHydrostatic && (p.select3dCoriScheme >= 1 || p.useNHMTerms);
    auto kern = rs ? (qh ? k_dt_l1f<true, true> : k_dt_l1f<true, false>)
                   : (qh ? k_dt_l1f<false, true> : k_dt_l1f<false, false>);
    const int nbPhi = phi_flat_blocks(d, p);
    hipLaunchKernelGGL(kern, dim3((unsigned)(nbOp + nbGm + nbPhi + nbDel)), dim3(256), 0, s, d, p, f, nbGm, nbPhi,
                       nbOp);
    return;
  }
  int nc, nArr, nbPhi;
  phi_frame(d, p, nc, nArr, nbPhi);
  MG_ALLOW_LDS(k_dt_l1);
  hipLaunchKernelGGL(k_dt_l1, dim3((unsigned)(nbOp + nbGm + nbPhi + nbDel)), dim3(256), mg_colf_lds(d.Nr, nc, nArr), s, d, p,
                     f, nc, nbGm, nbPhi, nbOp, dt_long_first());
}
template <bool GM, bool FF4>
__global__ void __launch_bounds__(256) k_dt_l2(Dims d, Params p, Fields f, TracerArgs aT, TracerArgs aS,
                                               const int *iterPtr, int nbMom, int nbTr, const long *__restrict__ srcOf,
                                               int nbPc, int nbOp, int lf) {
  int lb = mg_xcd_block();
  if (lf) {   // long first: the tracers' right-hand sides at the head of the dispatch
    if (lb < 2 * nbTr) {
      if (lb < nbTr) tracer_rhs_body_br<GM>(d, p, f, aT, iterPtr, lb);
      else tracer_rhs_body_br<GM>(d, p, f, aS, iterPtr, lb - nbTr);
      return;
    }
    lb -= 2 * nbTr;
  }
  if (lb < nbPc) { ucg2d_p_point(d, p, f, srcOf, lb); return; }
  lb -= nbPc;
  if (lb < nbOp) { ucg2d_op_point(d, p, f, lb); return; }
  lb -= nbOp;
  if (lb < nbMom) {
    if constexpr (FF4) mom_ff4_body(d, p, f, iterPtr, lb);
    else if (lb & 1) mom_step_point<false, 2>(d, p, f, iterPtr, lb >> 1);
    else mom_step_point<false, 1>(d, p, f, iterPtr, lb >> 1);
    return;
  }
  lb -= nbMom;
  if (lb < nbTr) tracer_rhs_body_br<GM>(d, p, f, aT, iterPtr, lb);
  else tracer_rhs_body_br<GM>(d, p, f, aS, iterPtr, lb - nbTr);
}
__global__ void __launch_bounds__(256) k_dt_l3(Dims d, Params p, Fields f, TracerArgs aT, TracerArgs aS,
                                               const int *iterPtr, int nc, int nbCd, int nbImp, const long *__restrict__ srcOf,
                                               int nbPc, int lf) {
  int lb = mg_xcd_block();
  if (lf) {   // long first: the implicit solves' column sweeps at the head of the dispatch
    if (lb < 2 * nbImp) {
      if (lb < nbImp) tracer_impl_body<false>(d, p, f, aT, nc, lb);
      else tracer_impl_body<false>(d, p, f, aS, nc, lb - nbImp);
      return;
    }
    lb -= 2 * nbImp;
    if (lb < nbPc) { ucg2d_p_point(d, p, f, srcOf, lb); return; }
    cd_scheme_body(d, p, f, iterPtr, lb - nbPc);
    return;
  }
  if (lb < nbPc) { ucg2d_p_point(d, p, f, srcOf, lb); return; }
  lb -= nbPc;
  if (lb < nbCd) { cd_scheme_body(d, p, f, iterPtr, lb); return; }
  lb -= nbCd;
  if (lb < nbImp) tracer_impl_body<false>(d, p, f, aT, nc, lb);
  else tracer_impl_body<false>(d, p, f, aS, nc, lb - nbImp);
}
// whether launch_dyn_thermo runs GMREDI_CALC_TENSOR itself (one_step then launches
// DO_OCEANIC_PHYS without it)
bool dyn_thermo_takes_gm(const Params &p) {
  const char *e = getenv("MGCM_DT_LAYOUT");   // read per call (A/B runs)
  return p.useGMRedi && p.useCDscheme && !(p.implicitViscosity) && !(e && atoi(e) == 2);
}

// Where the fold is exact and applies: both tracers stepped with the per-point right-hand
// side (GM/Redi; no multi-dimensional advection) and the implicit vertical solve, flux-form
// momentum split into U and V halves, on the small grids (mg_hfuse: <= 2^21 points), and
// MGCM_STEP_FUSE bit MG_FUSE_DT
bool dyn_thermo_fusable(const Dims &d, const Params &p, const TracerArgs &aT, const TracerArgs &aS) {
  return mg_hfuse(MG_FUSE_DT, d.nx, d.ny, d.nT, d.Nr) && p.momStepping && p.tempStepping && p.saltStepping &&
         p.useGMRedi && p.implicitDiffusion && !aT.multiDim && !aS.multiDim && !p.vectorInvariantMomentum &&
         aT.scr != aS.scr && aT.scheme == 2 && aS.scheme == 2 && !p.useAB3;   // (tracer_rhs_body_br: C2, AB2)
}

// CALC_PHI_HYD's column frame as launch_phi_hyd sizes it
static void phi_frame(const Dims &d, const Params &p, int &nc, int &nArr, int &nb) {
  const long ncol = (long)(d.sNx + 3) * (d.sNy + 3) * d.nT;
  nArr = (p.nonlinFreeSurf > 0 && p.select_rStar > 0) ? 6 : 3;
  nc = mg_colf_nc(ncol, d.Nr, nArr);
  nb = (int)mg_colf_blocks(ncol, nc);
}

// Outside the fold (e.g. the staggered step): GMREDI_CALC_TENSOR beside CALC_PHI_HYD (+ del2uv
// where it shares phi's grid, phi_del2_fused) in k_dt_l1 -- both read only DO_OCEANIC_PHYS'
// output -- on the small grids; DO_OCEANIC_PHYS then launches without the tensor
bool gm_phi_fusable(const Dims &d, const Params &p) {
  return mg_hfuse(MG_FUSE_DT, d.nx, d.ny, d.nT, d.Nr) && p.useGMRedi && p.momStepping;
}
// op: UPDATE_CG2D's operator in the same grid (ucg2d.h; its preconditioner then rides in the r*
// pass, launch_update_r_star_cg2d pcHere)
hipError_t launch_gm_phi(const Dims &d, const Params &p, const Fields &f, hipStream_t s, bool op) {
  launch_l1(d, p, f, phi_del2_fused(d, p) ? (int)mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr) : 0, s, op ? ucg2d_blocks(d) : 0);
  return hipGetLastError();
}

// Both tracers of THERMODYNAMICS in two launches instead of four (small grids, outside the
// fold, e.g. after the pressure solve in the staggered step): [rhs(theta) | rhs(salt)], then
// [implicit solve (theta) | (salt)]; theta's T* in gTscr, salt's in cpScr
template <bool GM>
__global__ void __launch_bounds__(256) k_tr_rhs_pair(Dims d, Params p, Fields f, TracerArgs aT, TracerArgs aS,
                                                     const int *iterPtr, int nbTr) {
  const int lb = mg_xcd_block();
  if (lb < nbTr) tracer_rhs_body<GM>(d, p, f, aT, iterPtr, lb);
  else tracer_rhs_body<GM>(d, p, f, aS, iterPtr, lb - nbTr);
}
__global__ void __launch_bounds__(256) k_tr_impl_pair(Dims d, Params p, Fields f, TracerArgs aT, TracerArgs aS, int nc,
                                                      int nbImp) {
  const int lb = mg_xcd_block();
  if (lb < nbImp) tracer_impl_body<false>(d, p, f, aT, nc, lb);
  else tracer_impl_body<false>(d, p, f, aS, nc, lb - nbImp);
}
bool tracer_hpair_ok(const Dims &d, const Params &p, const TracerArgs &aT, const TracerArgs &aS) {
  return mg_hfuse(MG_FUSE_DT, d.nx, d.ny, d.nT, d.Nr) && p.tempStepping && p.saltStepping && p.implicitDiffusion &&
         !aT.multiDim && !aS.multiDim && aT.scr != aS.scr && !tracer_march_on(d);
}
hipError_t launch_tracer_hpair(const Dims &d, const Params &p, const Fields &f, const TracerArgs &aT, const TracerArgs &aS,
                               const int *iterPtr, hipStream_t s) {
  const int nbTr = (int)mg_plane_blocks(d.sNx, d.sNy, d.nT * d.Nr);
  // (without GM/Redi k_tracer_rhs<false>'s body: bit-identical to the flat kernel the single
  // path runs)
  if (p.useGMRedi) hipLaunchKernelGGL(k_tr_rhs_pair<true>, dim3((unsigned)(2 * nbTr)), dim3(256), 0, s, d, p, f, aT, aS,
                                      iterPtr, nbTr);
  else hipLaunchKernelGGL(k_tr_rhs_pair<false>, dim3((unsigned)(2 * nbTr)), dim3(256), 0, s, d, p, f, aT, aS, iterPtr, nbTr);
  const long ncol = (long)d.sNx * d.sNy * d.nT;
  const int nc = mg_colf_nc(ncol, d.Nr, 3);
  const int nbImp = (int)mg_colf_blocks(ncol, nc);
  MG_ALLOW_LDS(k_tr_impl_pair);
  hipLaunchKernelGGL(k_tr_impl_pair, dim3((unsigned)(2 * nbImp)), dim3(256), mg_colf_lds(d.Nr, nc, 3), s, d, p, f, aT, aS, nc,
                     nbImp);
  return hipGetLastError();
}

// CALC_PHI_HYD + THERMODYNAMICS' tracers + DYNAMICS in three launches on one stream
// (after DO_OCEANIC_PHYS; dyn_thermo_fusable must hold).  srcOf != nullptr (default layout,
// nonlinFreeSurf > 2, every tile): UPDATE_CG2D in the first two grids as well (ucg2d.h), and
// launch_update_r_star_cg2d then runs with opEarly
hipError_t launch_dyn_thermo(const Dims &d, const Params &p, const Fields &f, const TracerArgs &aT, const TracerArgs &aS,
                             const int *iterPtr, hipStream_t s, const long *srcOf) {
  const dim3 blk(256);
  // front: phi's column frame (launch_phi_hyd's columns and LDS), del2uv's and the tracers' planes
  int ncPhi, nArrPhi, nbPhi;
  phi_frame(d, p, ncPhi, nArrPhi, nbPhi);
  const int nbDel = del2_needed(p) ? (int)mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr) : 0;
  const int nbTr = (int)mg_plane_blocks(d.sNx, d.sNy, d.nT * d.Nr);
  if (dyn_thermo_takes_gm(p)) {
    // UPDATE_CG2D's operator in grid 2, its preconditioner in grid 3 (config 2 0.2821-0.2832
    // ms/step; the operator in grid 1 and the preconditioner in grid 2 0.2852-0.2857 on the same
    // box, profiles/r04/ope_at/; the preconditioner in the r* pass 0.2825-0.2829 against
    // 0.2815-0.2819, profiles/r04/ope_at3/) -- the longest grid (the momentum chain) hides the
    // operator's blocks best
    const int nbU = srcOf ? ucg2d_blocks(d) : 0;
    const int nbOp1 = 0, nbPc2 = 0, nbOp2 = nbU, nbPc3 = nbU;
    launch_l1(d, p, f, nbDel, s, nbOp1);
    const bool ff4 = mom_ff4_on(true);
    const int nbMom = ff4 ? mom_ff4_blocks(d) : 2 * (int)mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr);
    auto l2 = ff4 ? k_dt_l2<true, true> : k_dt_l2<true, false>;
    hipLaunchKernelGGL(l2, dim3((unsigned)(nbPc2 + nbOp2 + nbMom + 2 * nbTr)), blk, 0, s, d, p, f, aT, aS, iterPtr, nbMom, nbTr,
                       srcOf, nbPc2, nbOp2, dt_long_first());
    const long ncolTr = (long)d.sNx * d.sNy * d.nT;
    const int ncTr = mg_colf_nc(ncolTr, d.Nr, 3);
    const int nbImp = (int)mg_colf_blocks(ncolTr, ncTr);
    const int nbCd = (int)mg_plane_blocks(d.nx - 2, d.ny - 2, d.nT * d.Nr);
    MG_ALLOW_LDS(k_dt_l3);
    hipLaunchKernelGGL(k_dt_l3, dim3((unsigned)(nbPc3 + nbCd + 2 * nbImp)), blk, mg_colf_lds(d.Nr, ncTr, 3), s, d, p, f, aT,
                       aS, iterPtr, ncTr, nbCd, nbImp, srcOf, nbPc3, dt_long_first());
    return hipGetLastError();
  }
  if (srcOf) return hipErrorInvalidValue;   // (the operator rides only in the default layout)
  MG_ALLOW_LDS(k_dt_front<true>);
  hipLaunchKernelGGL(k_dt_front<true>, dim3((unsigned)(nbPhi + nbDel + 2 * nbTr)), blk,
                     mg_colf_lds(d.Nr, ncPhi, nArrPhi), s, d, p, f, aT, aS, iterPtr, ncPhi, nbPhi, nbDel, nbTr);
  // back: the momentum halves and the implicit solves (k_tracer_impl's columns and LDS)
  const int nbMom = 2 * (int)mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr);
  const long ncolTr = (long)d.sNx * d.sNy * d.nT;
  const int ncTr = mg_colf_nc(ncolTr, d.Nr, 3);
  const int nbImp = (int)mg_colf_blocks(ncolTr, ncTr);
  MG_ALLOW_LDS(k_dt_back);
  hipLaunchKernelGGL(k_dt_back, dim3((unsigned)(nbMom + 2 * nbImp)), blk, mg_colf_lds(d.Nr, ncTr, 3), s, d, p, f, aT, aS,
                     iterPtr, ncTr, nbMom, nbImp);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_mom_tail(d, p, f, iterPtr, s);
}

}  // namespace mgcm
