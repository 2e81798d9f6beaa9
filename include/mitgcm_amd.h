/*
 * mitgcm_amd.h -- C-ABI of the MI355X-native MITgcm dynamical hot path.
 *
 * Plain C: opaque handles, pointers and sizes only (no torch / HIP types).
 * Two families of entry points:
 *
 *  1. Model-handle API (mgcm_*): a tile set resident in HBM, driven step by step.
 *     Every array crossing the boundary uses the reference's layout: fp64,
 *     halo-inclusive (1-OLx:sNx+OLx, 1-OLy:sNy+OLy[, 1:Nr], tile), i fastest
 *     (model/inc/DYNVARS.h:36-152, model/inc/GRID.h:311-523).
 *
 *  2. Fortran-callable drop-ins with the reference's own argument lists
 *     (lower-case + trailing underscore, all arguments by reference, as
 *     genmake2's FC_NAMEMANGLE produces for amdflang), e.g. cg2d_amd_ replaces
 *     SUBROUTINE CG2D of model/src/cg2d.F:13-17.  See INTEGRATION.md for the
 *     MODS-directory shims that bind them.
 *
 * Errors: entry points returning int give 0 on success and a negative code on
 * failure (mgcm_last_error() has the message).  The Fortran entry points have
 * no return channel (the reference has none either): they
 * print the error and abort(), the equivalent of STOP 'ABNORMAL END'.
 */
#ifndef MITGCM_AMD_H
#define MITGCM_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mgcm_model mgcm_model;

/* ------------------------------------------------------------ lifecycle */
/* Allocate a device-resident tile set of nSx*nSy tiles of (sNx+2OLx)(sNy+2OLy)Nr
 * points on HIP device `device`.  Replaces the per-tile COMMON-block storage of
 * DYNVARS.h / GRID.h / CG2D.h for the tiles this GPU owns. */
mgcm_model *mgcm_create(int sNx, int sNy, int OLx, int OLy, int Nr, int nSx, int nSy, int device);
void mgcm_destroy(mgcm_model *m);
const char *mgcm_last_error(void);

/* pkg/exch2 halo maps from the W2_EXCH2_TOPOLOGY.h arrays W2_E2SETUP fills (host only, no
 * model, no device): the copies of EXCH2_3D_RL (exch2_3d_rx.template) and
 * EXCH2_UV_CGRID_3D_RL with (u1, v1) and without (u0, v0) signs, as the gather maps of
 * mgcm_set_halo_map / mgcm_set_uv_map, over nTiles tiles of sNx x sNy with overlap OL.
 * Per-neighbour arrays in Fortran layout (ldNb = W2_maxNeighbours, ldT = W2_maxNbTiles), pij
 * (4, ldNb, ldT); tile ids 1-based as W2 numbers them.  Outputs hold nTiles*(sNx+2OL)*(sNy+2OL)
 * entries.  useCubedSphereExchange (EEPARAMS.h, 0/1) gates the cube-corner u/v fix-ups as
 * the reference's IF does (exch2_uv_3d_rx.template:79).  Returns -1 on an inconsistent
 * topology.  (exch2_maps.hip) */
int mgcm_exch2_maps(int sNx, int sNy, int OL, int nTiles, int ldNb, int ldT, const int *tBasex, const int *tBasey,
                    const int *isNedge, const int *isSedge, const int *isEedge, const int *isWedge,
                    const int *nNeighbours, const int *neighbourId, const int *opposingSend, const int *pij,
                    const int *oi, const int *oj, const int *iLo, const int *iHi, const int *jLo, const int *jHi,
                    int useCubedSphereExchange, long *src, long *u1, long *v1, long *u0, long *v0);

/* Run-time parameters (PARAMS.h names, already resolved as ini_parms.F does). */
int mgcm_set_param(mgcm_model *m, const char *name, double value);
double mgcm_get_param(mgcm_model *m, const char *name);

/* The device's iteration counter (myIter: AB2's first step, the CD scheme's start),
 * written in stream order without a host synchronisation (mgcm_set_param("myIter")
 * synchronises). */
int mgcm_set_iter(mgcm_model *m, int myIter);
/* myIter += inc on the device, in stream order: FORWARD_STEP's advance of myIter
 * (forward_step.F:806) inside a captured step, where mgcm_set_iter's value would be baked in
 * (fortran_abi.hip's multi-model step replay). */
int mgcm_add_iter(mgcm_model *m, int inc);
/* Which of the theta / salt ping-pong buffers are current (CYCLE_TRACER is a pointer swap,
 * cycle_tracer.F): bit 0 theta, bit 1 salt, 0 = the first-allocated buffer.  set < 0 returns
 * the current parity; set = 0..3 makes that parity current (a replayed step whose capture
 * already ran the host-side swaps: fortran_abi.hip). */
int mgcm_tracer_parity(mgcm_model *m, int set);

/* Host <-> device copies of named fields (DYNVARS/GRID/CG2D/FFIELDS names,
 * e.g. "uVel", "hFacW", "aW2d", "fu").  count = number of doubles. */
int mgcm_put(mgcm_model *m, const char *name, const double *host, long count);
int mgcm_get(mgcm_model *m, const char *name, double *host, long count);
/* mgcm_put in stream order, without a host synchronisation: the host arrays are staged in
 * pinned memory (two slots) and may be reused as soon as the call returns; a batch of n
 * fields goes up as one copy and one scatter launch. */
int mgcm_put_async(mgcm_model *m, const char *name, const double *host, long count);
int mgcm_put_batch_async(mgcm_model *m, int n, const char *const *names, const double *const *hosts,
                         const long *counts);
/* Device pointer of a named field (for zero-copy interop, e.g. torch tensors). */
double *mgcm_device_ptr(mgcm_model *m, const char *name);

/* Halo topology.  Default (set by mgcm_create): EXCH1 lat-lon, periodic over the
 * nSx x nSy tile layout (eesupp/src/exch1_rx.template:8-276).  A caller with a
 * cube/LLC topology (pkg/exch2) passes, for every halo point, the flat source
 * offset (tile,j,i) it copies from, or -1 to leave it untouched. */
int mgcm_set_halo_map(mgcm_model *m, const long *src_of_point, long count);

/* EXCH2 C-grid vector maps (pkg/exch2/exch2_uv_3d_rx.template), for EXCH_UV_XY(Z)_RL with
 * withSigns = .TRUE. (u1, v1) and .FALSE. (u0, v0): per point of u and of v, 0 = untouched,
 * +(src+1) / -(src+1) = copy (minus) the value at src, which indexes [u | v] (2*count);
 * tileFace/tileEdge (exch2_myFace, edge bits N=1 S=2 E=4 W=8) drive the cube-corner
 * vorticity of MOM_CALC_RELVORT3.  Built by mitgcm_amd/exch2.py. */
int mgcm_set_uv_map(mgcm_model *m, const long *u1, const long *v1, const long *u0, const long *v0,
                    const int *tileFace, const int *tileEdge, long count);

/* Finish set-up after grid/mask/operator fields are in place: builds the CG2D
 * neighbour tables and checks that the option set is one the kernels support. */
int mgcm_init(mgcm_model *m);

/* --------------------------------------------------------- hot path ops */
/* DO_OCEANIC_PHYS subset (model/src/do_oceanic_phys.F:555-882: surface
 * relaxation forcing, FIND_RHO_2D, IVDC) followed by THERMODYNAMICS
 * (model/src/thermodynamics.F:25 -> temp_integrate.F: GAD advection/diffusion,
 * AB2, implicit vertical diffusion) for theta.  No-op unless tempStepping. */
int mgcm_thermodynamics(mgcm_model *m);
/* DYNAMICS (model/src/dynamics.F:21): MOM_FLUXFORM + TIMESTEP + AB2 for every
 * tile and level; writes gU/gV (= u*, v*) and updates guNm1/gvNm1. */
int mgcm_dynamics(mgcm_model *m);
/* SOLVE_FOR_PRESSURE (model/src/solve_for_pressure.F:7): CALC_DIV_GHAT RHS,
 * CG2D, EXCH, etaN = recip_Bo * x. */
int mgcm_solve_for_pressure(mgcm_model *m);
/* MOMENTUM_CORRECTION_STEP (model/src/momentum_correction_step.F:7). */
int mgcm_momentum_correction_step(mgcm_model *m);
/* INTEGR_CONTINUITY (model/src/integr_continuity.F:13): wVel (r* included), and with
 * exactConserv the new etaN, EXCH, UPDATE_ETAH. */
int mgcm_integr_continuity(mgcm_model *m);
/* UPDATE_R_STAR(.TRUE.) + UPDATE_CG2D (update_r_star.F:6, update_cg2d.F:7;
 * forward_step.F:838-868); no-op unless nonlinFreeSurf > 0. */
int mgcm_update_r_star(mgcm_model *m);
/* CALC_R_STAR(etaH) (calc_r_star.F:10; forward_step.F:976); no-op unless nonlinFreeSurf > 0. */
int mgcm_calc_r_star(mgcm_model *m);
/* DO_FIELDS_BLOCKING_EXCHANGES (model/src/do_fields_blocking_exchanges.F:54): the set
 * FORWARD_STEP exchanges (u, v through the vector map on EXCH2, w, the stepped tracers,
 * uVelD/vVelD with the CD scheme); does not advance the step counter. */
int mgcm_blocking_exchanges(mgcm_model *m);
/* DO_OCEANIC_PHYS (model/src/do_oceanic_phys.F:43) alone: forcing records (when
 * periodicExternalForcing), FREEZE_SURFACE, surface forcing, FIND_RHO_2D, GRAD_SIGMA,
 * CALC_IVDC, the GM/Redi tensor. */
int mgcm_oceanic_phys(mgcm_model *m);
/* THERMODYNAMICS (model/src/thermodynamics.F:25) alone: TEMP/SALT_INTEGRATE + CYCLE_TRACER. */
int mgcm_tracer_step(mgcm_model *m);
/* DO_STAGGER_FIELDS_EXCHANGES (model/src/do_stagger_fields_exchanges.F:7; forward_step.F:1010,
 * staggerTimeStep): EXCH_UV_3D_RL(uVel, vVel, .TRUE.) + EXCH_3D_RL(wVel) before the staggered
 * THERMODYNAMICS. */
int mgcm_stagger_exchanges(mgcm_model *m);
/* EXCH_XY(Z)_RL / EXCH_UV_XY(Z)_RL (eesupp/src/exch_*_rx.template) on caller-owned host
 * arrays of nz levels (u alone for a scalar; u, v with vector = 1 for a C-grid pair,
 * withSigns as the reference's LOGICAL), with this model's halo maps. */
int mgcm_exchange_host(mgcm_model *m, double *u, double *v, int nz, int vector, int withSigns);
/* Name of run-time parameter i (0-based) that mgcm_set_param accepts; NULL past the end. */
const char *mgcm_param_name(int i);
/* Number of doubles of a named field (-1: unknown name). */
long mgcm_field_count(mgcm_model *m, const char *name);
/* Capture the hipGraph that mgcm_forward_step replays (two steps per graph) for
 * the current state, so that a timed region does not include the capture. */
int mgcm_prepare(mgcm_model *m);
/* FORWARD_STEP subset: the six ops above (+ surface forcing), nsteps times,
 * asynchronously on the model's stream (captured once into a hipGraph). */
int mgcm_forward_step(mgcm_model *m, int nsteps);
/* ---- tile-sharded runs (one process per GPU, mitgcm_amd/parallel.py; or several models
 * of one Fortran host process, fortran_abi.hip) -------------------------------------------
 * Every process holds the whole domain's arrays; the 3-D kernels step only tiles
 * [t0, t0+nT) (the reference's myBxLo..myBxHi / process tile set).
 * The 2-D pressure solve runs either as the device CG2D -- the multi-workgroup solver's
 * parts of each process's tiles on one shared hand-off block (phase 10, mgcm_cg2d_shared_*)
 * -- or replicated on every process over the gathered right-hand side (phase 2); either way
 * its sums are the single-GPU sums and results are bit-identical at any N. */
int mgcm_set_tile_range(mgcm_model *m, int t0, int nT);
/* Run on `stream` (a hipStream_t, e.g. the caller's collective stream); NULL = own. */
int mgcm_set_stream(mgcm_model *m, void *stream);
/* Number of fields DO_FIELDS_BLOCKING_EXCHANGES moves (u, v, w[, theta][, salt]). */
int mgcm_exchange_nfields(mgcm_model *m);
/* Gather (unpack=0) / scatter (unpack=1) those fields at n device-resident 2-D
 * offsets idx (t*n2 + j*nx + i), all levels: buf[(f*Nr + k)*n + h]. */
int mgcm_halo_pack(mgcm_model *m, const long *idx, long n, double *buf, int unpack);
/* The same for a group of them: 0 all, 1 the tracers (final after THERMODYNAMICS, so their
 * exchange can overlap DYNAMICS and the solve: pkg/exch2/exch2_rx1_cube.template:118-247's
 * PUT/send ... recv/GET split), 2 the rest; -1 from the count for a bad group. */
int mgcm_exchange_nfields_group(mgcm_model *m, int group);
int mgcm_halo_pack_group(mgcm_model *m, int group, const long *idx, long n, double *buf, int unpack);
/* Order the model's stream against a caller's stream `other` (a hipStream_t): direction 0
 * = `other` waits for the model's work so far (its outputs are then readable there), 1 =
 * the model waits for `other`'s work so far (e.g. a received buffer).  No-op when they are
 * the same stream. */
int mgcm_stream_handoff(mgcm_model *m, void *other, int direction);
/* Device-to-device copy of tiles [t0, t0+nT) of a 2-D/3-D field to (toField=0) or
 * from (toField=1) the device buffer buf, on the model's stream. */
int mgcm_tile_copy(mgcm_model *m, const char *name, int t0, int nT, void *buf, int toField);
/* Reset the per-step solve records before a sequence of mgcm_step_phase steps. */
int mgcm_begin_steps(mgcm_model *m);
/* After replaying caller-captured steps: the batch recorded nsteps solve records. */
int mgcm_end_steps(mgcm_model *m, int nsteps);
/* One FORWARD_STEP split at its exchange points (model.hip): 1 = 8 + 9; 8 DO_OCEANIC_PHYS +
 * THERMODYNAMICS; 9 DYNAMICS + UPDATE_R_STAR/CG2D + CALC_DIV_GHAT; 2 CG2D + correction +
 * continuity; 10 the device CG2D over this process's parts; 6 = 2 after a CG2D done
 * outside phase 2; 3 r*; 5 staggered tracers; 4 exchanges. */
int mgcm_step_phase(mgcm_model *m, int phase);
/* Distributed CG2D (mitgcm_amd/parallel.py, cg2dMode = "distributed"): one operation of
 * model/src/cg2d.F:100-415 over this process's tiles (op 0 normalise + max, 1 scale by a0,
 * 2 initial residual, 3 preconditioner, 4 s = q + a0*s, 5 A s, 6 x/r update with a0,
 * 7 un-normalise, 8 save x as the lowest-residual solution, 9 restore it: cg2dUseMinResSol;
 * CG2D_SR, cg2d_sr.F: 10 y = M r, s = y, 11 x/r update with a0, 12 y = M r, 13 v = A y,
 * 14 sum r*r, 15 s/q update with a0),
 * per-tile partials to the device buffer part[2*nTiles] -- the per-tile
 * values GLOBAL_SUM_TILE_RL (eesupp/src/global_sum_tile.F:14-17,161-191) sums in tile order.
 * Phase 6 of mgcm_step_phase finishes phase 2 after such a solve. */
int mgcm_cg2d_op(mgcm_model *m, int op, double a0, double *part);
/* The tile-sharded device CG2D (parallel.py cg2d="device", phase 10 of mgcm_step_phase):
 * the multi-workgroup solver's parts of this process's tiles, on one hand-off block shared
 * by all processes -- exported (IPC handle of mgcm_cg2d_shared_bytes bytes) by one process
 * and mapped by the others; the solve's sums are the single-process sums, no host step
 * inside an iteration.  Needs whole-domain multi-workgroup tables (param cg2dForceMwg on
 * grids the single-workgroup kernels would take). */
int mgcm_cg2d_shared_bytes(mgcm_model *m);
int mgcm_cg2d_shared_export(mgcm_model *m, void *handle);
int mgcm_cg2d_shared_import(mgcm_model *m, const void *handle);
/* Several models stepped by ONE host process (fortran_abi.hip: the Fortran drop-ins with
 * MGCM_AMD_MODELS = N), each over its own tile range:
 *   mgcm_get_stream    the model's current hipStream_t (cross-model ordering by events);
 *   mgcm_halo_sources  the interior points outside tiles [t0, t0+nT) that their halos copy
 *                      (scalar map + EXCH2 vector maps), sorted; returns the count (writes at
 *                      most cap) -- what the models stepping those points deliver;
 *   mgcm_cg2d_tiles    the device CG2D's parts of tiles [t0, t0+nT) on this model's arrays;
 *   mgcm_cg2d_share    m polls owner's hand-off block (uncached, system scope; peer access
 *                      between GPUs) -- the in-process form of mgcm_cg2d_shared_export/import.
 * mgcm_step_phase adds the routine-level phases 11 (CALC_DIV_GHAT right-hand side), 12 (CG2D
 * on the gathered domain + EXCH(cg2d_x) + etaN), 13 (EXCH(cg2d_x) + etaN), 14 (INTEGR_CONTINUITY's
 * column pass after MOMENTUM_CORRECTION_STEP) and 15 (EXCH(eta) + UPDATE_ETAH). */
void *mgcm_get_stream(mgcm_model *m);
long mgcm_halo_sources(mgcm_model *m, int t0, int nT, long *out, long cap);
int mgcm_cg2d_tiles(mgcm_model *m, int t0, int nT);
int mgcm_cg2d_share(mgcm_model *m, mgcm_model *owner);
/* Store CG2D's output arguments (cg2d.F:13-17) as this step's solve record (minResidualSq,
 * nIterMin: -1, -1 without cg2dUseMinResSol). */
int mgcm_cg2d_record(mgcm_model *m, double firstResidual, double lastResidual, double rhsMax, double sumRHS,
                     int numIters, double minResidualSq, int nIterMin);
/* Gather (unpack=0) / scatter (1) a 2-D field at n device-resident flat offsets idx. */
int mgcm_field_pack(mgcm_model *m, const char *name, const long *idx, long n, double *buf, int unpack);
/* EXCH of one field from this process's copy of the domain (EXCH_XY_RL / EXCH_S3D_RL with
 * the model's halo map; the cross-process sources must have been delivered first). */
int mgcm_exchange_field(mgcm_model *m, const char *name);

/* Wait for all queued device work. */
int mgcm_sync(mgcm_model *m);

/* Device CG2D on fields of this model (cg2d.F:13 semantics; b is normalised in
 * place).  b and x are host arrays of nTiles*(sNx+2OLx)*(sNy+2OLy) doubles. */
int mgcm_cg2d(mgcm_model *m, double *cg2d_b, double *cg2d_x, double *firstResidual,
              double *minResidualSq, double *lastResidual, int *numIters, int *nIterMin);

/* The summation order of the device CG2D's global sums (the GLOBAL_SUM_TILE_RL it
 * replaces, eesupp/src/global_sum_tile.F:161-191, sums tile partials in tile order): NG
 * workgroups of NT threads; thread tid of workgroup g accumulates, from 0.0, the per-point
 * terms at plan[(g*PPT + p)*NT + tid] (2-D flat offsets, -1 = none) for p = 0..PPT-1; a
 * workgroup's partial is the pairwise tree over its threads in thread order; lane l then
 * adds the partials l, l+64, ... in order and the total is the pairwise tree over the 64
 * lanes.  The oracle restates it (oracle_set_sum_plan) so that a device solve can be
 * checked bit for bit.  capacity = length of plan. */
int mgcm_cg2d_sum_plan(mgcm_model *m, int *plan, long capacity, int *NT, int *PPT, int *NG);

/* Statistics of the most recent solve (what SOLVE_FOR_PRESSURE prints,
 * solve_for_pressure.F:333-351) for step `back` (0 = latest) of the last
 * mgcm_forward_step call. */
int mgcm_solve_stats(mgcm_model *m, int back, double *firstResidual, double *lastResidual,
                     int *numIters, double *rhsMax);
/* The box's reference HBM rate: a STREAM triad a = b + s*c over three fp64 arrays of n
 * doubles on `device` (16 B per lane), best of `reps`, in GB/s (24 bytes per element). */
int mgcm_stream_triad(int device, long n, int reps, double *gbs);

/* The same step's min-residual bookkeeping (cg2dUseMinResSol, cg2d.F:190-193, 338-347):
 * minResidualSq and nIterMin (both -1 when the option is off). */
int mgcm_solve_minres(mgcm_model *m, int back, double *minResidualSq, int *nIterMin);
/* The same records for the last n steps of the last batch in one device-to-host copy,
 * oldest first (any output pointer may be NULL). */
int mgcm_solve_history(mgcm_model *m, int n, int *numIters, double *firstResidual, double *lastResidual);

/* MONITOR's dynstat block (pkg/monitor/monitor.F:103-129 -> MON_CALC_STATS_RL,
 * mon_calc_stats_rl.F / mon_stats_rl.F:104-107) computed on the device, no field download:
 * out[6*5] = (max, min, mean, sd, del2) of eta, uvel, vvel, wvel, theta, salt over this
 * process's tiles (per-plane tree partials added in tile, level order). */
int mgcm_monitor(mgcm_model *m, double *out);

/* Average device time (ms) of each kernel family over the last timed region,
 * measured with hipEvents on the model's stream.  name: "mom_step", "cg2d", ... */
double mgcm_kernel_ms(mgcm_model *m, const char *name, int *launches);
void mgcm_kernel_timing(mgcm_model *m, int enable);

/* ------------------------------------------- Fortran drop-in (reference ABI) */
/* Bound by the MODS-directory shims of mitgcm_amd/fortran/mods; all
 * arguments by reference, CHARACTER lengths appended as size_t.  Implementation:
 * mitgcm_amd/csrc/fortran_abi.hip. */
/* SIZE.h tile set; nProcs = nPx*nPy and nThreads = nTx*nTy must be 1. */
void mgcm_amd_setup_(const int *sNx, const int *sNy, const int *OLx, const int *OLy, const int *Nr,
                     const int *nSx, const int *nSy, const int *nProcs, const int *nThreads);
/* Halo maps given point by point: ids = source index per point, u1/v1/u0/v0 = +-(source+1)
 * codes, per-tile face and edges (a host that derives them itself). */
void mgcm_amd_set_maps_(const double *ids, const double *u1, const double *v1, const double *u0, const double *v0,
                        const int *tFace, const int *tEdge, const int *nPts);
/* The halo maps of a pkg/exch2 topology from the W2_EXCH2_TOPOLOGY.h COMMON arrays
 * W2_E2SETUP fills (mods/mgcm_amd_exch2.F; derived by mgcm_exch2_maps): one process holding
 * every tile in W2's order; ldNb = W2_maxNeighbours, ldT = W2_maxNbTiles; useCS = the host's
 * useCubedSphereExchange (0/1). */
void mgcm_amd_set_w2_(const int *nTiles, const int *ldNb, const int *ldT, const int *myFace, const int *tBasex,
                      const int *tBasey, const int *isN, const int *isS, const int *isE, const int *isW, const int *nNb,
                      const int *nbId, const int *opp, const int *pij, const int *oi, const int *oj, const int *iLo,
                      const int *iHi, const int *jLo, const int *jHi, const int *useCS);
/* One PARAMS.h parameter (LOGICAL as 0/1). */
void mgcm_amd_param_(const char *name, const double *value, size_t len);
/* Register a COMMON-block array of `count` doubles as device field `name`; kind 1 static
 * (uploaded once at init), 0 state, 2 host input (uploaded before every DO_OCEANIC_PHYS);
 * phiRef(2Nr+1) binds the device's phiRefC. */
void mgcm_amd_bind_(const char *name, double *array, const int *count, const int *kind, size_t len);
/* Upload the bound arrays and finish the device set-up. */
void mgcm_amd_init_(const int *myIter);
/* The device-authoritative mirror (fortran_abi.hip): bring the state down for a host
 * reader / push a host-modified state up; whole-array copies made so far. */
void mgcm_amd_host_sync_(const int *myThid);
void mgcm_amd_device_sync_(const int *myThid);
void mgcm_amd_transfer_stats_(int *nUploads, int *nDownloads, double *bytesUp, double *bytesDown);
/* Wait for the device work issued so far (hosts that clock their steps). */
void mgcm_amd_step_fence_(const int *myThid);
/* Routine drop-ins: during initialisation the bound state is uploaded before and
 * downloaded after each; from the first DO_OCEANIC_PHYS / THERMODYNAMICS / DYNAMICS on, the
 * device copy is authoritative (forcing up every step, state down for host readers). */
void do_oceanic_phys_amd_(const double *myTime, const int *myIter, const int *myThid);     /* do_oceanic_phys.F:43 */
void thermodynamics_amd_(const double *myTime, const int *myIter, const int *myThid);      /* thermodynamics.F:25 */
void dynamics_amd_(const double *myTime, const int *myIter, const int *myThid);            /* dynamics.F:21 */
void update_r_star_amd_(const int *useLatest, const double *myTime, const int *myIter,
                        const int *myThid);                                          /* update_r_star.F:6 */
void update_cg2d_amd_(const double *myTime, const int *myIter, const int *myThid);        /* update_cg2d.F:7 */
void calc_r_star_amd_(const double *etaFld, const double *myTime, const int *myIter,
                      const int *myThid);                                            /* calc_r_star.F:10 */
void solve_for_pressure_amd_(const double *myTime, const int *myIter, const int *myThid);  /* solve_for_pressure.F:7 */
void momentum_correction_step_amd_(const double *myTime, const int *myIter,
                                   const int *myThid);                   /* momentum_correction_step.F:7 */
void integr_continuity_amd_(const double *uFld, const double *vFld, const double *myTime, const int *myIter,
                            const int *myThid);                          /* integr_continuity.F:13 */
void do_fields_blocking_exchanges_amd_(const int *myThid);             /* do_fields_blocking_exchanges.F:7 */
void do_stagger_fields_exchanges_amd_(const double *myTime, const int *myIter,
                                       const int *myThid);              /* do_stagger_fields_exchanges.F:7 */
/* Exchanges and the tile-ordered global sum on host arrays. */
void exch_xy_rl_amd_(double *phi, const int *myThid);                          /* exch_xy_rx.template:9 */
void exch_xyz_rl_amd_(double *phi, const int *myThid);                         /* exch_xyz_rx.template:8 */
void exch_uv_xy_rl_amd_(double *u, double *v, const int *withSigns, const int *myThid);  /* exch_uv_xy_rx.template:11 */
void exch_uv_xyz_rl_amd_(double *u, double *v, const int *withSigns,
                         const int *myThid);                                   /* exch_uv_xyz_rx.template:12 */
void global_sum_tile_rl_amd_(const double *phiTile, double *sumPhi, const int *myThid);  /* global_sum_tile.F:14 */
/* Registers the CG2D operator of CG2D.h (ini_cg2d.F:61-237 outputs) for the
 * drop-in CG2D below.  Arrays are (1-OLx:sNx+OLx,1-OLy:sNy+OLy,nSx,nSy). */
void ini_cg2d_amd_(const int *sNx, const int *sNy, const int *OLx, const int *OLy,
                   const int *nSx, const int *nSy, const double *aW2d, const double *aS2d,
                   const double *aC2d, const double *pW, const double *pS, const double *pC,
                   const double *cg2dNorm, const double *cg2dTolerance_sq,
                   const int *cg2dNormaliseRHS);
/* SUBROUTINE CG2D(cg2d_b,cg2d_x,firstResidual,minResidualSq,lastResidual,
 *                 numIters,nIterMin,myThid)   -- model/src/cg2d.F:13-17 */
void cg2d_amd_(double *cg2d_b, double *cg2d_x, double *firstResidual, double *minResidualSq,
               double *lastResidual, int *numIters, int *nIterMin, const int *myThid);

#ifdef __cplusplus
}
#endif
#endif
