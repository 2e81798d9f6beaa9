// model.hip -- host runtime of the MI355X hot path and its C-ABI (include/mitgcm_amd.h).
//
// Owns the device mirror of the reference's per-tile COMMON blocks (DYNVARS.h,
// GRID.h, SURFACE.h, FFIELDS.h, CG2D.h) for the tiles on one GPU, the halo
// topology (EXCH1 lat-lon by default, any EXCH2 map via mgcm_set_halo_map), and
// the launch sequence of FORWARD_STEP's device-resident subset.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <utility>
#include <string>
#include <vector>

#include "../../include/mitgcm_amd.h"
#include "common.h"

namespace mgcm {
// Host ranges the Fortran mirror registered for DMA (fortran_abi.hip register_host: the
// page-rounded extents of its bound COMMON arrays).  An unbound host array that shares an
// edge page is then partly registered, and the runtime refuses a copy that spans the edge of
// a registered range ("invalid argument"): mg_host_copy splits a host<->device copy at every
// registered-range edge, so each piece lies wholly inside or wholly outside one.
static std::vector<std::pair<uintptr_t, uintptr_t>> g_hostReg;
void mg_host_ranges_set(const uintptr_t *lo, const uintptr_t *hi, size_t n) {
  g_hostReg.clear();
  for (size_t i = 0; i < n; i++) g_hostReg.push_back({lo[i], hi[i]});
  std::sort(g_hostReg.begin(), g_hostReg.end());
}
hipError_t mg_host_copy(void *dst, const void *src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
  if (g_hostReg.empty() || bytes == 0) return hipMemcpyAsync(dst, src, bytes, kind, s);
  const uintptr_t h = (uintptr_t)(kind == hipMemcpyHostToDevice ? src : dst), end = h + bytes;
  size_t off = 0;
  while (h + off < end) {
    const uintptr_t cur = h + off;
    uintptr_t cut = end;
    for (const auto &r : g_hostReg) {
      if (r.first > cur && r.first < cut) cut = r.first;
      if (r.second > cur && r.second < cut) cut = r.second;
    }
    const hipError_t e = hipMemcpyAsync((char *)dst + off, (const char *)src + off, cut - cur, kind, s);
    if (e != hipSuccess) return e;
    off += cut - cur;
  }
  return hipSuccess;
}
}  // namespace mgcm

namespace mgcm {
hipError_t launch_mom_step(const Dims &, const Params &, const Fields &, const int *, hipStream_t, bool ring = true);
bool mom_ring_separable(const Dims &, const Params &);
hipError_t launch_mom_ring(const Dims &, const Params &, const Fields &, const int *, hipStream_t);
hipError_t launch_phi_hyd(const Dims &, const Params &, const Fields &, hipStream_t);
bool phys_phi_fusable(const Dims &, const Params &);
hipError_t launch_phys_phi(const Dims &, const Params &, const Fields &, const int *, hipStream_t);
hipError_t launch_sfp_rhs(const Dims &, const Params &, const Fields &, hipStream_t);
hipError_t launch_cg2d_block(const Dims &, const Params &, const Fields &, const unsigned *, const int *, int, int, int,
                             SolveRecord *, int *, hipStream_t);
int cg2d_block_ppt(int nPts);
int cg2d_ref_max_points();
hipError_t launch_cg2d_bxy(int, const Dims &, const Params &, const Fields &, const unsigned *, const int *, int, int,
                           int, SolveRecord *, int *, const int *, const long *, hipStream_t);
int cg2d_bxy_geometry(int, int *, int *, int *);
int cg2d_bxy_variants();
hipError_t launch_cg2d_blk2(const Dims &, const Params &, const Fields &, const unsigned *, const int *, int, int, int,
                            SolveRecord *, int *, hipStream_t);
int cg2d_block_max_points();
hipError_t launch_exchange(const Dims &, double *, const long *, int, int, hipStream_t);
hipError_t launch_cgd(const Dims &, const Params &, const Fields &, int, double, double *, hipStream_t);
hipError_t launch_cgd_record(SolveRecord *, const int *, double, double, double, double, int, double, int, hipStream_t);
hipError_t launch_field_pack(double *, const long *, long, double *, int, hipStream_t);
hipError_t launch_correction(const Dims &, const Params &, const Fields &, hipStream_t);
hipError_t launch_bump_counter(int *, int, hipStream_t);
hipError_t launch_exchange_multi(const Dims &, const XFields &, const long *, int, int *, hipStream_t);
hipError_t launch_exchange_uv(const Dims &, double *, double *, const long *, int, int, int, hipStream_t);
hipError_t launch_exchange_mixed(const Dims &, double *, double *, int, const long *, int, int, const XFields &,
                                 const long *, int, int *, hipStream_t);
hipError_t launch_exchange_uv_pairs(const Dims &, double *const *, double *const *, int, const long *, int, int,
                                   hipStream_t);
hipError_t launch_exch_eta(const Dims &, const Params &, const Fields &, const long *, bool, int, hipStream_t,
                           int fromX = 0);
hipError_t launch_corr_cont(const Dims &, const Params &, const Fields &, int, hipStream_t, const long *etaSrc = nullptr);
hipError_t launch_calc_r_star(const Dims &, const Params &, const Fields &, const long *, hipStream_t, bool fuseEtaH = false,
                              int fromX = 0);
hipError_t launch_rstar_exmix(const Dims &, const Params &, const Fields &, const long *, bool, int, double *, double *, int,
                              const long *, int, int, const XFields &, const long *, int, hipStream_t);
hipError_t launch_rstar_exch(const Dims &, const Params &, const Fields &, const long *, bool, const XFields &, const long *,
                             int, int *, hipStream_t, int fromX = 0);
hipError_t launch_update_r_star_cg2d(const Dims &, const Params &, const Fields &, const long *, hipStream_t, bool sfp = false,
                                     bool opEarly = false, bool pcHere = false);
hipError_t launch_halo_pack(const Dims &, const XFields &, const long *, long, double *, int, hipStream_t);
hipError_t launch_oceanic_phys(const Dims &, const Params &, const Fields &, const int *, hipStream_t, bool gm = true,
                               bool *ringDone = nullptr);
hipError_t launch_tracer_step(const Dims &, const Params &, const Fields &, const TracerArgs &, const int *, hipStream_t,
                              bool impl = true);
bool dyn_thermo_fusable(const Dims &, const Params &, const TracerArgs &, const TracerArgs &);
hipError_t launch_dyn_thermo(const Dims &, const Params &, const Fields &, const TracerArgs &, const TracerArgs &, const int *,
                             hipStream_t, const long *srcOf = nullptr);
bool dyn_thermo_takes_gm(const Params &);
hipError_t launch_gm_tensor(const Dims &, const Params &, const Fields &, hipStream_t);
hipError_t launch_hfac_snapshot(const Dims &, const Fields &, double *, hipStream_t);
Fields hfac_snapshot_fields(const Dims &, const Fields &, double *);
bool gm_phi_fusable(const Dims &, const Params &);
hipError_t launch_gm_phi(const Dims &, const Params &, const Fields &, hipStream_t, bool op = false);
bool tracer_hpair_ok(const Dims &, const Params &, const TracerArgs &, const TracerArgs &);
hipError_t launch_tracer_hpair(const Dims &, const Params &, const Fields &, const TracerArgs &, const TracerArgs &,
                               const int *, hipStream_t);
hipError_t launch_mon_stats(const Dims &, const MonSpecs &, int, double *, int, hipStream_t);
int cg2d_mwg_geometry(int *, int *, int *);
hipError_t launch_cg2d_mwg(const Dims &, const Params &, const Fields &, const MwgTables &, int, int, SolveRecord *, int *,
                           hipStream_t, int g0 = 0, int gN = -1);
}  // namespace mgcm

using namespace mgcm;

static thread_local std::string g_err;
static int set_err(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return -1;
}
#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return set_err("%s:%d %s: %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
  } while (0)

enum FieldKind { F1D, F2D, F3D, FREC };   // FREC: 6 forcing fields x MG_MAXREC records of 2-D
#define MG_MAXREC 12
struct FieldDesc {
  const char *name;
  FieldKind kind;
  size_t off;  // offset of the pointer inside Fields
};

#define FD(n, k) {#n, k, offsetof(Fields, n)}
static const FieldDesc FIELDS[] = {
    FD(drF, F1D), FD(drC, F1D), FD(recip_drF, F1D), FD(recip_drC, F1D), FD(rF, F1D), FD(rC, F1D), FD(tRef, F1D), FD(sRef, F1D), FD(pRef4EOS, F1D), FD(phiRefC, F1D),
#define FD2(n) FD(n, F2D),
#define FD3(n) FD(n, F3D),
    MG_F2D_LIST(FD2)
    MG_F3D_LIST(FD3)
#undef FD2
#undef FD3
    FD(forcRec, FREC),
};
#undef FD

struct PDesc {
  const char *name;
  size_t off;
  bool isint;
};
#define PD(n) {#n, offsetof(Params, n), false}
#define PI_(n) {#n, offsetof(Params, n), true}
static const PDesc PARAMS[] = {
    PD(deltaTMom), PD(deltaTFreeSurf), PD(deltaTClock), PD(abEps), PD(alph_AB), PD(beta_AB), PI_(useAB3), PD(rhoConst), PD(gBaro), PD(viscAhD), PD(viscAhZ),
    PD(viscA4D), PD(viscA4Z), PD(viscAr), PD(sideDragFactor), PD(freeSurfFac), PD(implicSurfPress),
    PD(implicDiv2DFlow), PD(rkSign), PD(afFacMom), PD(vfFacMom), PD(pfFacMom), PD(cfFacMom), PD(foFacMom),
    PD(mtFacMom), PD(cg2dNorm), PD(cg2dTolerance_sq),
    PI_(momAdvection), PI_(momViscosity), PI_(momForcing), PI_(useCoriolis), PI_(no_slip_sides),
    PI_(no_slip_bottom), PI_(selectCoriScheme), PI_(momForcingOutAB), PI_(momDissip_In_AB),
    PI_(implicitViscosity), PI_(cg2dMaxIters), PI_(cg2dUseMinResSol), PI_(cg2dNormaliseRHS), PI_(nIter0), PI_(cg2dUseFMA), PI_(useSRCGSolver), PI_(cg2dRefOrder),
    PD(gravity), PD(gravitySign), PD(rhoNil), PD(tAlpha), PD(sBeta), PD(ivdc_kappa), PD(diffKhT), PD(diffKrT),
    PD(deltaTtracer), PI_(exactConserv), PI_(tempStepping), PI_(tempAdvection), PI_(tempForcing),
    PI_(implicitDiffusion), PI_(tempAdvScheme), PI_(saltStepping), PI_(saltAdvection), PI_(saltForcing),
    PI_(saltAdvScheme), PD(diffKhS), PD(diffKrS), PI_(multiDimAdvection), PI_(multiDimCompressible), PI_(momStepping),
    PI_(eosType), PI_(allowFreezing), PI_(useRealFreshWaterFlux), PI_(useCDscheme), PI_(useGMRedi),
    PI_(periodicExternalForcing), PI_(nForcRec), PD(HeatCapacity_Cp), PD(convertFW2Salt), PD(temp_EvPrRn),
    PD(salt_EvPrRn), PD(rCD), PD(epsAB_CD), PD(externForcingPeriod), PD(externForcingCycle), PD(GM_background_K),
    PD(GM_isopycK), PD(GM_skewflx), PD(GM_maxSlope), PD(GM_Kmin_horiz), PD(GM_Small_Number), PD(GM_slopeSqCutoff),
    PI_(GM_AdvForm), PI_(GM_ExtraDiag),
    PI_(nonlinFreeSurf), PI_(select_rStar), PI_(quasiHydrostatic), PI_(useNHMTerms), PI_(select3dCoriScheme),
    PI_(selectP_inEOS_Zc), PI_(storePhiHyd4Phys), PD(hFacInf),
    PI_(vectorInvariantMomentum), PI_(selectVortScheme), PI_(selectKEscheme), PI_(upwindShear),
    PI_(staggerTimeStep), PI_(tracForcingOutAB),
};
#undef PD
#undef PI_

// kernel families timed with hipEvents when timing is enabled
enum Kern { K_MOM, K_RHS, K_CG2D, K_EXCH, K_ETA, K_CORR, K_CONT, K_PHYS, K_TEMP, K_RSTAR, K_PHI, K_N };
static const char *KNAMES[K_N] = {"mom_step",   "sfp_rhs",    "cg2d",         "exchange",  "eta_update",
                                  "correction", "continuity", "oceanic_phys", "temp_step", "r_star", "phi_hyd"};

struct mgcm_model {
  Dims d{};
  Params p{};
  Fields f{};
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t ownStream = nullptr;   // created by mgcm_create; `stream` may be a caller's
  // THERMODYNAMICS runs on a second stream concurrently with DYNAMICS (fork after
  // DO_OCEANIC_PHYS, join before UPDATE_R_STAR / SOLVE_FOR_PRESSURE; MGCM_NO_OVERLAP=1 off)
  hipStream_t stream2 = nullptr;
  hipEvent_t evFork = nullptr, evJoin = nullptr;
  hipEvent_t evSnap = nullptr;   // the hFac snapshot of THERMODYNAMICS beside the solve under r* (MG_FUSE_TCG)
  double *snapH = nullptr;        // hFacC, hFacW, hFacS, recip_hFacC, recip_hFacW, recip_hFacS (6 x N3all)
  hipStream_t stream3 = nullptr;                  // EXCH(cg2d_x) + etaN beside the correction step
  hipEvent_t evEta0 = nullptr, evEta1 = nullptr;
  hipEvent_t evHand = nullptr;   // mgcm_stream_handoff
  bool overlap = true;
  std::vector<void *> allocs;
  // extra parameters kept on host only
  std::map<std::string, double> extra;
  // halo map (2*nHalo longs) and CG2D neighbour table
  long *d_halo = nullptr;
  long *d_srcOf = nullptr;    // per 2-D point: interior source of a halo point, -1 otherwise
  int nHalo = 0;
  long *d_haloAll = nullptr;  // the map of EVERY tile's halo when this model steps a tile subset
  int nHaloAll = 0;           // (EXCH_*_RL on host arrays, mgcm_exchange_host, covers the domain)
  std::vector<long> h_halo;
  unsigned *d_nbr = nullptr;  // packed (W|E<<16),(S|N<<16) compact neighbour indices, padded
  int *d_gofs = nullptr;      // 2-D flat offset of each (padded) interior point
  int nPts = 0;
  // 2x2-blocked solver tables (even sNx, sNy; <= 1024 blocks)
  unsigned *d_nb4 = nullptr;
  int *d_blk = nullptr;
  int nBlk = 0;
  // BX x BY-blocked solver tables (k_cg2d_bxy; preferred when the global grid tiles into them)
  unsigned *d_nbx = nullptr;
  int *d_blkx = nullptr;
  int nBlkX = 0;
  int bxyVar = -1;              // k_cg2d_bxy geometry (kernels_solve.hip CGX[])
  int *d_slot2 = nullptr;       // per 2-D point: k_cg2d_bxy's LDS slot of its value after EXCH, or -1
  bool latlonTopology = true;   // false once a custom halo map (e.g. EXCH2 cube) is installed
  // multi-workgroup CG2D (kernels_cg2d_mwg.hip): tables of every part, device buffers
  bool useMwg = false;
  MwgTables mwg{};
  std::vector<void *> mwgAllocs;
  void *mwgShared = nullptr;   // another process's hand-off block, opened by IPC (mgcm_cg2d_shared_import)
  void *mwgBlock = nullptr;    // this model's own hand-off block (hipMalloc, or uncached once shared)
  std::vector<int> mwgPlan;   // summation plan for mgcm_cg2d_sum_plan: [(g*OPT + p)*NT + tid]
  // EXCH2 C-grid vector maps (mgcm_set_uv_map): [withSigns] -> (dst, code) pairs of this
  // process's tiles, u entries first; code = +-(src+1), src indexing [u | v]
  bool uvMap = false;
  std::vector<long> h_uv[2];
  long *d_uv[2] = {nullptr, nullptr};
  int nUvU[2] = {0, 0}, nUvV[2] = {0, 0};
  // the same maps over every tile (tile-sharded runs recompute the 2-D r* state of the whole
  // domain redundantly: CALC_R_STAR's EXCH_UV of the W/S factors covers remote tiles too)
  long *d_uvAll[2] = {nullptr, nullptr};
  int nUvUAll[2] = {0, 0}, nUvVAll[2] = {0, 0};
  int *d_tileInfo = nullptr;
  // device scratch of mgcm_exchange_host (EXCH_*_RL on caller arrays)
  double *exchBuf[2] = {nullptr, nullptr};
  long exchCap = 0;
  // hipGraphs of two FORWARD_STEPs, one per theta/salt ping-pong parity
  bool useGraph = true;
  hipGraphExec_t graphExec[2][4] = {};   // [THERMODYNAMICS overlap off/on][tracer buffer parity]
  hipGraphExec_t graph1Exec[2][4] = {};  // ONE step (callers that step one at a time: the Fortran drop-ins)
  double *graph1Tr[2][4][4] = {};        // its tracer pointers after the step: theta, thetaNext, salt, saltNext
  // overlap auto-selection (ovl_trial): both graphs timed on a copy of the state
  bool ovlAuto = false, ovlDecided = false;
  float ovlMs[2] = {0.f, 0.f};
  hipEvent_t ovlEv[2] = {nullptr, nullptr};
  double *thetaA = nullptr, *saltA = nullptr;
  int stepLayout = 0;   // one_step's launch layout (mgcm_get_param "stepLayout")
  // THERMODYNAMICS of a sharded step on the second stream (mgcm_step_phase 16): 1 forked after
  // DO_OCEANIC_PHYS (joined before UPDATE_R_STAR), 2 to fork after CALC_DIV_GHAT, 3 forked
  // after it (joined before the correction step), 0 none pending
  int shardFork = 0;
  // mgcm_put_batch_async: two pinned host slots (each with the event of its last copy) and
  // one device buffer; a batch travels as [header | values] in one copy, then one scatter
  char *stHost[2] = {nullptr, nullptr};
  hipEvent_t stEv[2] = {nullptr, nullptr};    // slot q's scatter done (its pinned and device buffers free)
  hipEvent_t stCopied[2] = {nullptr, nullptr};   // slot q's copy done (the scatter may read it)
  size_t stCap = 0;
  int stNext = 0;
  char *stDev[2] = {nullptr, nullptr};
  hipStream_t stCopy = nullptr;   // the uploads' copy stream: a step's copy overlaps the step before
  // step counters: [0] = myIter, [1] = record slot
  int *d_ctr = nullptr;
  SolveRecord *d_rec = nullptr;
  int maxRec = 4096;
  int lastBatch = 0;
  double *monBuf = nullptr;   // MONITOR plane partials (mgcm_monitor)
  size_t monCap = 0;
  bool ready = false;
  // timing
  bool timing = false;
  std::vector<hipEvent_t> evPool;            // created once, reused
  size_t evUsed = 0;
  std::vector<std::pair<int, int>> evPairs;  // (kernel, start event index)
  double kms[K_N] = {0};
  int kcnt[K_N] = {0};
};

static void drop_graphs(mgcm_model *m);

static long field_count(const mgcm_model *m, FieldKind k) {
  if (k == F1D) return m->d.Nr + 1;
  if (k == F2D) return m->d.n2 * m->d.nTiles;
  if (k == FREC) return 6L * MG_MAXREC * m->d.n2 * m->d.nTiles;
  return m->d.n3 * m->d.nTiles;
}
static const FieldDesc *find_field(const char *name) {
  for (auto &fd : FIELDS)
    if (!strcmp(fd.name, name)) return &fd;
  return nullptr;
}
static double *&field_ptr(mgcm_model *m, const FieldDesc *fd) {
  return *reinterpret_cast<double **>(reinterpret_cast<char *>(&m->f) + fd->off);
}

// ------------------------------------------------------------------ timing
static int ev_next(mgcm_model *m) {
  if (m->evUsed == m->evPool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    m->evPool.push_back(e);
  }
  return (int)m->evUsed++;
}
static int ev_begin(mgcm_model *m, int k) {
  (void)k;
  if (!m->timing) return -1;
  const int i = ev_next(m);
  if (i < 0) return -1;
  hipEventRecord(m->evPool[i], m->stream);
  return i;
}
static void ev_end(mgcm_model *m, int k, int startIdx) {
  if (!m->timing || startIdx < 0) return;
  const int i = ev_next(m);
  if (i < 0) return;
  hipEventRecord(m->evPool[i], m->stream);
  m->evPairs.push_back({k, startIdx});
}
// call with the stream drained
static void ev_collect(mgcm_model *m) {
  for (auto &pr : m->evPairs) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, m->evPool[pr.second], m->evPool[pr.second + 1]) == hipSuccess) {
      m->kms[pr.first] += ms;
      m->kcnt[pr.first] += 1;
    }
  }
  m->evPairs.clear();
  m->evUsed = 0;
}
static void ev_free(mgcm_model *m) {
  for (auto e : m->evPool) hipEventDestroy(e);
  m->evPool.clear();
  m->evUsed = 0;
}

// ------------------------------------------------------------------ topology
// EXCH1 lat-lon periodic halo map (eesupp/src/exch1_rx.template:170-198): every
// halo point copies the interior point with the wrapped global index.
static void build_latlon_halo(mgcm_model *m) {
  const Dims &d = m->d;
  const int Nx = d.sNx * d.nSx, Ny = d.sNy * d.nSy;
  m->h_halo.clear();
  for (int t = 0; t < d.nTiles; t++) {
    const int bi = t % d.nSx, bj = t / d.nSx;
    for (int j = 1 - d.OLy; j <= d.sNy + d.OLy; j++)
      for (int i = 1 - d.OLx; i <= d.sNx + d.OLx; i++) {
        if (i >= 1 && i <= d.sNx && j >= 1 && j <= d.sNy) continue;
        int iG = ((bi * d.sNx + i - 1) % Nx + Nx) % Nx, jG = ((bj * d.sNy + j - 1) % Ny + Ny) % Ny;
        int st = (jG / d.sNy) * d.nSx + iG / d.sNx;
        m->h_halo.push_back(MG_I2(d, i, j, t));
        m->h_halo.push_back(MG_I2(d, iG % d.sNx + 1, jG % d.sNy + 1, st));
      }
  }
}

static int upload_halo(mgcm_model *m) {
  if (m->d_halo) { hipFree(m->d_halo); m->d_halo = nullptr; }
  if (m->d_srcOf) { hipFree(m->d_srcOf); m->d_srcOf = nullptr; }
  const long N2 = m->d.n2 * m->d.nTiles;
  std::vector<long> srcOf(N2, -1);
  for (size_t h = 0; h + 1 < m->h_halo.size(); h += 2) srcOf[m->h_halo[h]] = m->h_halo[h + 1];
  HIPCHK(hipMalloc(&m->d_srcOf, N2 * sizeof(long)));
  HIPCHK(hipMemcpy(m->d_srcOf, srcOf.data(), N2 * sizeof(long), hipMemcpyHostToDevice));
  // the 3-D exchange kernels refresh the halos of this process's tiles only
  // (tile-sharded runs receive the remote sources first, mgcm_halo_unpack)
  std::vector<long> loc;
  const long lo = (long)m->d.t0 * m->d.n2, hi = (long)(m->d.t0 + m->d.nT) * m->d.n2;
  for (size_t h = 0; h + 1 < m->h_halo.size(); h += 2)
    if (m->h_halo[h] >= lo && m->h_halo[h] < hi) { loc.push_back(m->h_halo[h]); loc.push_back(m->h_halo[h + 1]); }
  m->nHalo = (int)(loc.size() / 2);
  if (m->d_haloAll) { hipFree(m->d_haloAll); m->d_haloAll = nullptr; }
  m->nHaloAll = 0;
  if (m->d.nT < m->d.nTiles && !m->h_halo.empty()) {
    HIPCHK(hipMalloc(&m->d_haloAll, m->h_halo.size() * sizeof(long)));
    HIPCHK(hipMemcpy(m->d_haloAll, m->h_halo.data(), m->h_halo.size() * sizeof(long), hipMemcpyHostToDevice));
    m->nHaloAll = (int)(m->h_halo.size() / 2);
  }
  if (m->uvMap) {
    const long N2 = m->d.n2 * m->d.nTiles;
    for (int all = 0; all < 2; all++)
      for (int w = 0; w < 2; w++) {
        long *&dm = all ? m->d_uvAll[w] : m->d_uv[w];
        if (dm) { hipFree(dm); dm = nullptr; }
        const long l0 = all ? 0 : lo, l1 = all ? N2 : hi;
        std::vector<long> e;
        int nu = 0, nv = 0;
        for (int c = 0; c < 2; c++)
          for (long q = l0; q < l1; q++) {
            const long code = m->h_uv[w][(size_t)c * N2 + q];
            if (code == 0) continue;
            e.push_back(q); e.push_back(code);
            (c ? nv : nu)++;
          }
        (all ? m->nUvUAll : m->nUvU)[w] = nu;
        (all ? m->nUvVAll : m->nUvV)[w] = nv;
        if (!e.empty()) {
          HIPCHK(hipMalloc(&dm, e.size() * sizeof(long)));
          HIPCHK(hipMemcpy(dm, e.data(), e.size() * sizeof(long), hipMemcpyHostToDevice));
        }
      }
  }
  if (m->nHalo == 0) return 0;
  HIPCHK(hipMalloc(&m->d_halo, loc.size() * sizeof(long)));
  HIPCHK(hipMemcpy(m->d_halo, loc.data(), loc.size() * sizeof(long), hipMemcpyHostToDevice));
  return 0;
}

// CG2D neighbour table: compact interior index of the value found at the W,E,S,N
// neighbour (through the halo map when the neighbour is a halo point), packed as
// two 16-bit indices per word; points are padded to PPT*1024 and padding /
// missing neighbours point at the ZERO slot (index NP).
static int build_nbr(mgcm_model *m) {
  const Dims &d = m->d;
  const long N2 = d.n2 * d.nTiles;
  std::vector<long> srcOf(N2, -1);
  for (size_t h = 0; h + 1 < m->h_halo.size(); h += 2) srcOf[m->h_halo[h]] = m->h_halo[h + 1];
  m->nPts = d.nTiles * d.sNx * d.sNy;
  const int ppt = cg2d_block_ppt(m->nPts);
  if (!ppt) return 0;  // too large for the single-workgroup solver (checked by mgcm_init)
  const int NP = ppt * 1024;
  const unsigned ZERO = (unsigned)NP;
  auto compact = [&](long g) -> unsigned {
    if (g < 0) return ZERO;
    long t = g / d.n2, l = g % d.n2;
    int i = (int)(l % d.nx) - d.OLx + 1, j = (int)(l / d.nx) - d.OLy + 1;
    if (i < 1 || i > d.sNx || j < 1 || j > d.sNy) return ZERO;
    return (unsigned)(t * d.sNx * d.sNy + (long)(j - 1) * d.sNx + (i - 1));
  };
  std::vector<unsigned> nb(2 * (size_t)NP, ZERO | (ZERO << 16));
  std::vector<int> gofs(NP, (int)MG_I2(d, 1, 1, 0));
  for (int t = 0; t < d.nTiles; t++)
    for (int j = 1; j <= d.sNy; j++)
      for (int i = 1; i <= d.sNx; i++) {
        const int pidx = t * d.sNx * d.sNy + (j - 1) * d.sNx + (i - 1);
        const int di[4] = {-1, 1, 0, 0}, dj[4] = {0, 0, -1, 1};
        unsigned c4[4];
        for (int c = 0; c < 4; c++) {
          const int ii = i + di[c], jj = j + dj[c];
          long g = MG_I2(d, ii, jj, t);
          if (ii < 1 || ii > d.sNx || jj < 1 || jj > d.sNy) g = srcOf[g];
          c4[c] = compact(g);
        }
        nb[2 * (size_t)pidx] = c4[0] | (c4[1] << 16);
        nb[2 * (size_t)pidx + 1] = c4[2] | (c4[3] << 16);
        gofs[pidx] = (int)MG_I2(d, i, j, t);
      }
  if (m->d_nbr) (void)hipFree(m->d_nbr);
  if (m->d_gofs) (void)hipFree(m->d_gofs);
  HIPCHK(hipMalloc(&m->d_nbr, nb.size() * sizeof(unsigned)));
  HIPCHK(hipMemcpy(m->d_nbr, nb.data(), nb.size() * sizeof(unsigned), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&m->d_gofs, gofs.size() * sizeof(int)));
  HIPCHK(hipMemcpy(m->d_gofs, gofs.data(), gofs.size() * sizeof(int), hipMemcpyHostToDevice));
  // 2x2 blocks (k_cg2d_blk2), formed on the global lat-lon index space so that odd
  // tile sizes work: needs the default EXCH1 lat-lon topology, even global Nx and Ny,
  // and <= 1024 blocks; the ZERO slot is 4*1024.
  m->nBlk = 0;
  const int Nx = d.sNx * d.nSx, Ny = d.sNy * d.nSy;
  const int nBk = (Nx / 2) * (Ny / 2);
  if (m->latlonTopology && Nx % 2 == 0 && Ny % 2 == 0 && nBk <= 1024 && !getenv("MGCM_CG2D_NOBLOCKED")) {
    const unsigned Z = 4096u;
    auto cmp = [&](long g) -> unsigned {
      unsigned c = compact(g);
      return c == ZERO ? Z : c;
    };
    auto nbv = [&](int i, int j, int t) -> unsigned {  // value slot of the point (i,j,t), via halo map
      long g = MG_I2(d, i, j, t);
      if (i < 1 || i > d.sNx || j < 1 || j > d.sNy) g = srcOf[g];
      return cmp(g);
    };
    // global (I, J), 1-based -> tile-local point
    auto gpt = [&](int I, int J, int &i, int &j, int &t) {
      const int bi = (I - 1) / d.sNx, bj = (J - 1) / d.sNy;
      t = bj * d.nSx + bi; i = (I - 1) % d.sNx + 1; j = (J - 1) % d.sNy + 1;
    };
    std::vector<unsigned> nb4(4 * 1024, Z | (Z << 16));
    std::vector<int> blk(4 * 1024, (int)MG_I2(d, 1, 1, 0));
    int q = 0;
    for (int J0 = 1; J0 <= Ny; J0 += 2)
      for (int I0 = 1; I0 <= Nx; I0 += 2, q++) {
        int ii[2][2], jj[2][2], tt[2][2];
        for (int b = 0; b < 2; b++)
          for (int a = 0; a < 2; a++) gpt(I0 + a, J0 + b, ii[b][a], jj[b][a], tt[b][a]);
        for (int b = 0; b < 2; b++)
          for (int a = 0; a < 2; a++) blk[4 * q + 2 * b + a] = (int)MG_I2(d, ii[b][a], jj[b][a], tt[b][a]);
        // out-of-block neighbours, through each boundary point's own halo map
        nb4[4 * q + 0] = nbv(ii[0][0] - 1, jj[0][0], tt[0][0]) | (nbv(ii[1][0] - 1, jj[1][0], tt[1][0]) << 16);
        nb4[4 * q + 1] = nbv(ii[0][1] + 1, jj[0][1], tt[0][1]) | (nbv(ii[1][1] + 1, jj[1][1], tt[1][1]) << 16);
        nb4[4 * q + 2] = nbv(ii[0][0], jj[0][0] - 1, tt[0][0]) | (nbv(ii[0][1], jj[0][1] - 1, tt[0][1]) << 16);
        nb4[4 * q + 3] = nbv(ii[1][0], jj[1][0] + 1, tt[1][0]) | (nbv(ii[1][1], jj[1][1] + 1, tt[1][1]) << 16);
      }
    if (m->d_nb4) (void)hipFree(m->d_nb4);
    if (m->d_blk) (void)hipFree(m->d_blk);
    HIPCHK(hipMalloc(&m->d_nb4, nb4.size() * sizeof(unsigned)));
    HIPCHK(hipMemcpy(m->d_nb4, nb4.data(), nb4.size() * sizeof(unsigned), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&m->d_blk, blk.size() * sizeof(int)));
    HIPCHK(hipMemcpy(m->d_blk, blk.data(), blk.size() * sizeof(int), hipMemcpyHostToDevice));
    m->nBlk = nBk;
  }
  // BX x BY blocks (k_cg2d_bxy), same global-index construction; the first geometry of
  // the preference list the grid tiles into
  m->nBlkX = 0;
  int BX = 0, BY = 0, NT = 0, nBx = 0;
  m->bxyVar = -1;
  {
    static const int pref[] = {0, 1};
    for (int v : pref) {
      int bx, by, nt;
      if (cg2d_bxy_geometry(v, &bx, &by, &nt)) continue;
      const int n = (Nx % bx == 0 && Ny % by == 0) ? (Nx / bx) * (Ny / by) : 0;
      if (n > 0 && n <= nt) { m->bxyVar = v; BX = bx; BY = by; NT = nt; nBx = n; break; }
    }
  }
  if (m->latlonTopology && m->bxyVar >= 0 && !getenv("MGCM_CG2D_NOBLOCKED")) {
    const int NPT = BX * BY, NB = 2 * (BX + BY);
    const unsigned Z = (unsigned)(NPT * NT);
    // LDS slot of an interior point: point-in-block major, block minor (p*NT + block),
    // so that consecutive threads touch consecutive doubles (no LDS bank conflicts)
    std::vector<unsigned> slotOf((size_t)m->nPts, Z);
    {
      int qb = 0;
      for (int J0 = 1; J0 <= Ny; J0 += BY)
        for (int I0 = 1; I0 <= Nx; I0 += BX, qb++)
          for (int b = 0; b < BY; b++)
            for (int a = 0; a < BX; a++) {
              const int I = I0 + a, J = J0 + b, bi = (I - 1) / d.sNx, bj = (J - 1) / d.sNy;
              const int t = bj * d.nSx + bi, i = (I - 1) % d.sNx + 1, j = (J - 1) % d.sNy + 1;
              slotOf[(size_t)t * d.sNx * d.sNy + (size_t)(j - 1) * d.sNx + (i - 1)] = (unsigned)((b * BX + a) * NT + qb);
            }
    }
    auto cmp = [&](long g) -> unsigned {
      unsigned c = compact(g);
      return c == ZERO ? Z : slotOf[c];
    };
    auto nbv = [&](int i, int j, int t) -> unsigned {
      long g = MG_I2(d, i, j, t);
      if (i < 1 || i > d.sNx || j < 1 || j > d.sNy) g = srcOf[g];
      return cmp(g);
    };
    auto gpt = [&](int I, int J, int &i, int &j, int &t) {
      const int bi = (I - 1) / d.sNx, bj = (J - 1) / d.sNy;
      t = bj * d.nSx + bi; i = (I - 1) % d.sNx + 1; j = (J - 1) % d.sNy + 1;
    };
    std::vector<unsigned> nbx((size_t)(NB / 2) * NT, Z | (Z << 16));
    std::vector<int> blkx((size_t)NPT * NT, (int)MG_I2(d, 1, 1, 0));
    int q = 0;
    for (int J0 = 1; J0 <= Ny; J0 += BY)
      for (int I0 = 1; I0 <= Nx; I0 += BX, q++) {
        std::vector<int> ii(NPT), jj(NPT), tt(NPT);
        for (int b = 0; b < BY; b++)
          for (int a = 0; a < BX; a++) {
            gpt(I0 + a, J0 + b, ii[b * BX + a], jj[b * BX + a], tt[b * BX + a]);
            blkx[(size_t)NPT * q + b * BX + a] = (int)MG_I2(d, ii[b * BX + a], jj[b * BX + a], tt[b * BX + a]);
          }
        std::vector<unsigned> v(NB);
        for (int b = 0; b < BY; b++) {
          const int w = b * BX, e = b * BX + BX - 1;
          v[b] = nbv(ii[w] - 1, jj[w], tt[w]);
          v[BY + b] = nbv(ii[e] + 1, jj[e], tt[e]);
        }
        for (int a = 0; a < BX; a++) {
          const int so = a, no = (BY - 1) * BX + a;
          v[2 * BY + a] = nbv(ii[so], jj[so] - 1, tt[so]);
          v[2 * BY + BX + a] = nbv(ii[no], jj[no] + 1, tt[no]);
        }
        for (int k = 0; k < NB / 2; k++) nbx[(size_t)(NB / 2) * q + k] = v[2 * k] | (v[2 * k + 1] << 16);
      }
    // the epilogue's EXCH_XY_RL(cg2d_x): every 2-D point's value is the slot of itself
    // (interior) or of its interior source (halo), -1 where neither (kept as it is)
    std::vector<int> slot2((size_t)d.n2 * d.nTiles, -1);
    for (int J = 1; J <= Ny; J++)
      for (int I = 1; I <= Nx; I++) {
        int i, j, t;
        gpt(I, J, i, j, t);
        slot2[(size_t)MG_I2(d, i, j, t)] = (int)slotOf[(size_t)t * d.sNx * d.sNy + (size_t)(j - 1) * d.sNx + (i - 1)];
      }
    for (size_t g = 0; g < slot2.size(); g++)
      if (srcOf[g] >= 0) slot2[g] = slot2[(size_t)srcOf[g]];
    if (m->d_slot2) (void)hipFree(m->d_slot2);
    HIPCHK(hipMalloc(&m->d_slot2, slot2.size() * sizeof(int)));
    HIPCHK(hipMemcpy(m->d_slot2, slot2.data(), slot2.size() * sizeof(int), hipMemcpyHostToDevice));
    if (m->d_nbx) (void)hipFree(m->d_nbx);
    if (m->d_blkx) (void)hipFree(m->d_blkx);
    HIPCHK(hipMalloc(&m->d_nbx, nbx.size() * sizeof(unsigned)));
    HIPCHK(hipMemcpy(m->d_nbx, nbx.data(), nbx.size() * sizeof(unsigned), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&m->d_blkx, blkx.size() * sizeof(int)));
    HIPCHK(hipMemcpy(m->d_blkx, blkx.data(), blkx.size() * sizeof(int), hipMemcpyHostToDevice));
    m->nBlkX = nBx;
  }
  return 0;
}

// Multi-workgroup CG2D tables (kernels_cg2d_mwg.hip): every tile cut into row strips of
// <= OPT*NT points (one workgroup each), the two rings of neighbouring-part points each
// strip's stencils reach (through the halo map), LDS slot tables, export flags.
template <typename T>
static int mwg_upload(mgcm_model *m, const std::vector<T> &h, const T **out) {
  T *dptr = nullptr;
  HIPCHK(hipMalloc(&dptr, (h.empty() ? 1 : h.size()) * sizeof(T)));
  if (!h.empty()) HIPCHK(hipMemcpy(dptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  m->mwgAllocs.push_back(dptr);
  *out = dptr;
  return 0;
}

static int mwg_block_realloc(mgcm_model *m, int mem, bool sys);
static int build_mwg(mgcm_model *m) {
  for (void *q : m->mwgAllocs) (void)hipFree(q);
  m->mwgAllocs.clear();
  m->useMwg = false;
  const Dims &d = m->d;
  int NT, OPT, RPT;
  cg2d_mwg_geometry(&NT, &OPT, &RPT);
  const int NO = NT * OPT, NR = NT * RPT;
  if (d.sNx > NO) return set_err("build_mwg: sNx = %d > %d points per part", d.sNx, NO);
  const long N2 = d.n2 * d.nTiles;
  std::vector<long> srcOf(N2, -1);
  for (size_t h = 0; h + 1 < m->h_halo.size(); h += 2) srcOf[m->h_halo[h]] = m->h_halo[h + 1];
  const int ppTile = d.sNx * d.sNy;
  auto comp = [&](int i, int j, int t) { return t * ppTile + (j - 1) * d.sNx + (i - 1); };
  auto g2of = [&](int c) { const int t = c / ppTile, l = c % ppTile; return (int)MG_I2(d, l % d.sNx + 1, l / d.sNx + 1, t); };
  // neighbour (dir 0 W, 1 E, 2 S, 3 N) of compact point c, through the halo map; -1 = none
  auto nbr = [&](int c, int dir) -> int {
    const int t = c / ppTile, l = c % ppTile, i = l % d.sNx + 1, j = l / d.sNx + 1;
    const int ii = i + (dir == 0 ? -1 : dir == 1 ? 1 : 0), jj = j + (dir == 2 ? -1 : dir == 3 ? 1 : 0);
    if (ii >= 1 && ii <= d.sNx && jj >= 1 && jj <= d.sNy) return comp(ii, jj, t);
    const long src = srcOf[MG_I2(d, ii, jj, t)];
    if (src < 0) return -1;
    const int st = (int)(src / d.n2), sl = (int)(src % d.n2);
    const int si = sl % d.nx - d.OLx + 1, sj = sl / d.nx - d.OLy + 1;
    if (si < 1 || si > d.sNx || sj < 1 || sj > d.sNy) return -1;
    return comp(si, sj, st);
  };
  // parts: row strips of each tile
  int rows = NO / d.sNx;
  while (rows > 1 && 2 * (d.sNx + rows) > NR) rows--;
  if (rows > d.sNy) rows = d.sNy;
  const int nPartsTile = (d.sNy + rows - 1) / rows;
  std::vector<int> partOf((size_t)d.nTiles * ppTile);
  std::vector<std::vector<int>> own;
  for (int t = d.t0; t < d.t0 + d.nT; t++)
    for (int k = 0; k < nPartsTile; k++) {
      const int j0 = 1 + (k * d.sNy) / nPartsTile, j1 = ((k + 1) * d.sNy) / nPartsTile;
      std::vector<int> pts;
      for (int j = j0; j <= j1; j++)
        for (int i = 1; i <= d.sNx; i++) { pts.push_back(comp(i, j, t)); partOf[comp(i, j, t)] = (int)own.size(); }
      if ((int)pts.size() > NO) return set_err("build_mwg: part of %zu points > %d", pts.size(), NO);
      own.push_back(pts);
    }
  const int G = (int)own.size();
  std::vector<std::vector<int>> ring1(G), ring2(G);
  std::vector<std::vector<char>> inAnyRing(1);   // compact -> exported?
  std::vector<char> exported((size_t)d.nTiles * ppTile, 0);
  int r2max = 0;
  for (int g = 0; g < G; g++) {
    std::map<int, int> seen;   // compact -> 0 own, 1 ring1, 2 ring2
    for (int c : own[g]) seen[c] = 0;
    for (int c : own[g])
      for (int dir = 0; dir < 4; dir++) {
        const int nb = nbr(c, dir);
        if (nb >= 0 && !seen.count(nb)) { seen[nb] = 1; ring1[g].push_back(nb); }
      }
    for (int c : ring1[g])
      for (int dir = 0; dir < 4; dir++) {
        const int nb = nbr(c, dir);
        if (nb >= 0 && !seen.count(nb)) { seen[nb] = 2; ring2[g].push_back(nb); }
      }
    if ((int)ring1[g].size() > NR) return set_err("build_mwg: ring of %zu points > %d", ring1[g].size(), NR);
    for (int c : ring1[g]) exported[c] = 1;
    for (int c : ring2[g]) exported[c] = 1;
    r2max = std::max(r2max, (int)ring2[g].size());
  }
  const int IMAX = NR + ((r2max + 63) / 64) * 64, SZ = NO + IMAX;
  if (SZ >= 65535) return set_err("build_mwg: %d LDS slots exceed 16-bit indices", SZ);
  std::vector<int> ownG((size_t)G * NO, -1), ownC((size_t)G * NO, 0), ringG((size_t)G * NR, -1);
  std::vector<unsigned> ownNb((size_t)G * NO * 2, (unsigned)SZ | ((unsigned)SZ << 16)), ringNb((size_t)G * NR * 2,
                                                                                                 (unsigned)SZ | ((unsigned)SZ << 16));
  std::vector<unsigned> ownExp((size_t)G * NT, 0u);
  std::vector<int> impC((size_t)G * IMAX, 0), impG((size_t)G * IMAX, (int)MG_I2(d, 1, 1, d.t0)), nImp(G);
  m->mwgPlan.assign((size_t)G * NO, -1);
  // the exported points, numbered: their granules in the hand-off block
  std::vector<int> expSlot(exported.size(), -1);
  int nExp = 0;
  for (size_t c = 0; c < exported.size(); c++)
    if (exported[c]) expSlot[c] = nExp++;
  for (int g = 0; g < G; g++) {
    std::map<int, int> slot;
    for (size_t n = 0; n < own[g].size(); n++) {
      const int p = (int)n / NT, tid = (int)n % NT;
      slot[own[g][n]] = p * NT + tid;
    }
    for (size_t n = 0; n < ring1[g].size(); n++) slot[ring1[g][n]] = NO + (int)n;   // n = p*NT + tid
    for (size_t n = 0; n < ring2[g].size(); n++) slot[ring2[g][n]] = NO + NR + (int)n;
    auto sl = [&](int c) -> unsigned { if (c < 0) return (unsigned)SZ; auto it = slot.find(c); return it == slot.end() ? (unsigned)SZ : (unsigned)it->second; };
    for (size_t n = 0; n < own[g].size(); n++) {
      const int c = own[g][n], q = (int)n;   // slot p*NT + tid == n
      const size_t o = (size_t)g * NO + q;
      ownG[o] = g2of(c);
      ownC[o] = exported[c] ? expSlot[c] : 0;
      ownNb[2 * o] = sl(nbr(c, 0)) | (sl(nbr(c, 1)) << 16);
      ownNb[2 * o + 1] = sl(nbr(c, 2)) | (sl(nbr(c, 3)) << 16);
      if (exported[c]) ownExp[(size_t)g * NT + q % NT] |= 1u << (q / NT);
      m->mwgPlan[o] = ownG[o];
    }
    for (size_t n = 0; n < ring1[g].size(); n++) {
      const int c = ring1[g][n];
      const size_t o = (size_t)g * NR + n;
      ringG[o] = g2of(c);
      ringNb[2 * o] = sl(nbr(c, 0)) | (sl(nbr(c, 1)) << 16);
      ringNb[2 * o + 1] = sl(nbr(c, 2)) | (sl(nbr(c, 3)) << 16);
      impC[(size_t)g * IMAX + n] = expSlot[c];
      impG[(size_t)g * IMAX + n] = g2of(c);
    }
    for (size_t n = 0; n < ring2[g].size(); n++) {
      impC[(size_t)g * IMAX + NR + n] = expSlot[ring2[g][n]];
      impG[(size_t)g * IMAX + NR + n] = g2of(ring2[g][n]);
    }
    nImp[g] = NR + (int)ring2[g].size();
  }
  MwgTables &T = m->mwg;
  T = MwgTables{};
  if (mwg_upload(m, ownG, &T.ownG) || mwg_upload(m, ownC, &T.ownC) || mwg_upload(m, ownNb, &T.ownNb) ||
      mwg_upload(m, ownExp, &T.ownExp) || mwg_upload(m, ringG, &T.ringG) || mwg_upload(m, ringNb, &T.ringNb) ||
      mwg_upload(m, impC, &T.impC) || mwg_upload(m, impG, &T.impG) || mwg_upload(m, nImp, &T.nImp))
    return -1;
  T.G = G; T.IMAX = IMAX; T.SZ = SZ; T.nExp = nExp;
  T.pinned = (G <= 32 && !getenv("MGCM_CG2D_SPREAD")) ? 1 : 0;
  T.sys = 0;
  T.exclusive = 0;
  T.partsPerTile = (d.t0 == 0 && d.nT == d.nTiles) ? nPartsTile : 0;   // part ranges: whole-domain tables only
  // hand-off block: 64 B of words (launch epoch, timeout word), the partial granules, the
  // export granules; zeroed once here -- granule tags carry the launch epoch, so a launch
  // never matches an earlier launch's granules (a multiple of 16 B from the start)
  const size_t partGr = (size_t)2 * 3 * G * 2, hs = 64 + (partGr + (size_t)nExp * 4) * sizeof(unsigned long long);
  char *blk = nullptr;
  HIPCHK(hipMalloc(&blk, hs));
  HIPCHK(hipMemset(blk, 0, hs));
  m->mwgAllocs.push_back(blk);
  m->mwgBlock = blk;
  // this process's launch epoch: its own word (not in the hand-off block an IPC import replaces)
  unsigned *ep = nullptr;
  HIPCHK(hipMalloc(&ep, 64));
  HIPCHK(hipMemset(ep, 0, 64));
  m->mwgAllocs.push_back(ep);
  T.epoch = ep;
  T.ctr = (unsigned *)blk;
  T.part = (unsigned long long *)(blk + 64);
  T.xs = T.part + partGr;
  T.hsBytes = hs;
  m->useMwg = true;
  // The hand-off block's memory: where the parts spread over the XCDs (not pinned), uncached
  // device memory -- a granule store is then visible to the other XCDs' polls without an L2
  // round of its own: LLC-90 1.591 ms/step against 1.688 with the coarse-grained block, 117
  // parts, ~1 us per CG iteration (profiles/r04/mwgmem/); the XCD-pinned parts (cube, <= 32
  // parts, one XCD's L2) keep coarse-grained memory (cs32x15 0.416 against 0.421-0.455).
  // (fine-grained memory measured no better than coarse, system-scope accesses alike:
  // profiles/r04/mwgmem/)
  if (!T.pinned && mwg_block_realloc(m, 1, false)) return -1;
  return 0;
}

// ------------------------------------------------------------------ C-ABI
extern "C" {

const char *mgcm_last_error(void) { return g_err.c_str(); }

mgcm_model *mgcm_create(int sNx, int sNy, int OLx, int OLy, int Nr, int nSx, int nSy, int device) {
  if (sNx <= 0 || sNy <= 0 || Nr <= 0 || nSx <= 0 || nSy <= 0 || OLx < 2 || OLy < 2) {
    set_err("mgcm_create: invalid sizes (need OLx,OLy >= 2)");
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device) {
    set_err("mgcm_create: no HIP device %d (found %d)", device, ndev);
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) { set_err("mgcm_create: hipSetDevice failed"); return nullptr; }
  mgcm_model *m = new mgcm_model();
  m->device = device;
  Dims &d = m->d;
  d.sNx = sNx; d.sNy = sNy; d.OLx = OLx; d.OLy = OLy; d.Nr = Nr; d.nSx = nSx; d.nSy = nSy; d.nTiles = nSx * nSy;
  d.nx = sNx + 2 * OLx; d.ny = sNy + 2 * OLy; d.n2 = (long)d.nx * d.ny; d.n3 = d.n2 * Nr;
  d.t0 = 0; d.nT = d.nTiles;
  // defaults (model/src/set_defaults.F, resolved by ini_parms.F)
  Params &p = m->p;
  p.abEps = 0.01; p.alph_AB = 0.5; p.beta_AB = 5.0 / 12.0; p.useAB3 = 0; p.rhoConst = 999.8; p.gBaro = 9.81; p.sideDragFactor = 2.0; p.freeSurfFac = 1.0;
  p.implicSurfPress = 1.0; p.implicDiv2DFlow = 1.0; p.rkSign = -1.0;
  p.afFacMom = p.vfFacMom = p.pfFacMom = p.cfFacMom = p.foFacMom = p.mtFacMom = 1.0;
  p.momAdvection = p.momViscosity = p.momForcing = p.useCoriolis = 1;
  p.no_slip_sides = p.no_slip_bottom = 1; p.momDissip_In_AB = 1; p.momForcingOutAB = 0;
  p.cg2dMaxIters = 150; p.cg2dNormaliseRHS = 1;
  // CG2D in fused multiply-adds where the kernel supports it (k_cg2d_bxy): 2.14 -> 1.83 us per
  // iteration on global_ocean.90x40x15; the device-order oracle evaluates the same fma chains
  p.cg2dUseFMA = 1;
  p.gravity = 9.81; p.gravitySign = -1.0; p.rhoNil = 999.8; p.tAlpha = 2.0e-4; p.tempAdvection = 1;
  p.tempForcing = 1; p.tempAdvScheme = 2; p.implicitDiffusion = 0;
  p.saltAdvection = 1; p.saltForcing = 1; p.saltAdvScheme = 2; p.multiDimAdvection = 1; p.momStepping = 1;
  p.HeatCapacity_Cp = 3994.0; p.convertFW2Salt = 35.0; p.temp_EvPrRn = 123456.7; p.salt_EvPrRn = 0.0;
  p.nForcRec = 12; p.GM_Small_Number = 1.0e-20; p.GM_slopeSqCutoff = 1.0e48; p.GM_skewflx = 1.0;
  if (hipStreamCreateWithFlags(&m->ownStream, hipStreamNonBlocking) != hipSuccess) {
    set_err("mgcm_create: stream");
    delete m;
    return nullptr;
  }
  m->stream = m->ownStream;
  if (hipStreamCreateWithFlags(&m->stream2, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&m->evFork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&m->evHand, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&m->stream3, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&m->evEta0, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&m->evEta1, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&m->evJoin, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&m->evSnap, hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&m->ovlEv[0]) != hipSuccess || hipEventCreate(&m->ovlEv[1]) != hipSuccess) {
    set_err("mgcm_create: second stream / events");
    delete m;
    return nullptr;
  }
  // MGCM_OVERLAP=1 forces the second stream on, =0 off; otherwise the graph path picks by timing
  const char *ov = getenv("MGCM_OVERLAP");
  m->overlap = !(ov && atoi(ov) == 0);
  m->ovlAuto = !ov;
  // one arena per kind for the 2-D and 3-D fields (MG_F2D_LIST / MG_F3D_LIST order, common.h)
  d.N2all = d.n2 * d.nTiles;
  d.N3all = d.n3 * d.nTiles;
  double *arena[2] = {nullptr, nullptr};
  const long arenaN[2] = {(long)F2_COUNT * d.N2all, (long)F3_COUNT * d.N3all};
  for (int q = 0; q < 2; q++) {
    if (hipMalloc(&arena[q], arenaN[q] * sizeof(double)) != hipSuccess ||
        hipMemset(arena[q], 0, arenaN[q] * sizeof(double)) != hipSuccess) {
      set_err("mgcm_create: hipMalloc of the %s arena (%ld doubles)", q ? "3-D" : "2-D", arenaN[q]);
      mgcm_destroy(m);
      return nullptr;
    }
    m->allocs.push_back(arena[q]);
  }
  m->f.a2 = arena[0];
  m->f.a3 = arena[1];
  int n2i = 0, n3i = 0;
  for (auto &fd : FIELDS) {
    const long n = field_count(m, fd.kind);
    double *ptr = nullptr;
    if (fd.kind == F2D) ptr = arena[0] + (long)(n2i++) * d.N2all;
    else if (fd.kind == F3D) ptr = arena[1] + (long)(n3i++) * d.N3all;
    else if (hipMalloc(&ptr, n * sizeof(double)) != hipSuccess || hipMemset(ptr, 0, n * sizeof(double)) != hipSuccess) {
      set_err("mgcm_create: hipMalloc %s (%ld doubles)", fd.name, n);
      mgcm_destroy(m);
      return nullptr;
    } else {
      m->allocs.push_back(ptr);
    }
    field_ptr(m, &fd) = ptr;
  }
  if (hipMalloc(&m->d_ctr, 2 * sizeof(int)) != hipSuccess || hipMemset(m->d_ctr, 0, 2 * sizeof(int)) != hipSuccess ||
      hipMalloc(&m->d_rec, m->maxRec * sizeof(SolveRecord)) != hipSuccess) {
    set_err("mgcm_create: counters");
    mgcm_destroy(m);
    return nullptr;
  }
  build_latlon_halo(m);
  // the zero fills above run on the null stream, which the model's non-blocking streams do
  // not wait for: finish them before any stream-ordered upload (mgcm_put) can start
  if (hipDeviceSynchronize() != hipSuccess) {
    set_err("mgcm_create: zero fill");
    mgcm_destroy(m);
    return nullptr;
  }
  return m;
}

void mgcm_destroy(mgcm_model *m) {
  if (!m) return;
  hipSetDevice(m->device);
  if (m->stream) hipStreamSynchronize(m->stream);
  ev_collect(m);
  ev_free(m);
  drop_graphs(m);
  for (void *p : m->allocs) hipFree(p);
  if (m->monBuf) hipFree(m->monBuf);
  if (m->d_halo) hipFree(m->d_halo);
  if (m->d_srcOf) hipFree(m->d_srcOf);
  if (m->d_haloAll) hipFree(m->d_haloAll);
  for (int q = 0; q < 2; q++) {
    if (m->d_uv[q]) hipFree(m->d_uv[q]);
    if (m->d_uvAll[q]) hipFree(m->d_uvAll[q]);
  }
  if (m->d_tileInfo) hipFree(m->d_tileInfo);
  if (m->d_nbr) hipFree(m->d_nbr);
  if (m->d_gofs) hipFree(m->d_gofs);
  if (m->d_nb4) hipFree(m->d_nb4);
  if (m->d_blk) hipFree(m->d_blk);
  if (m->d_nbx) hipFree(m->d_nbx);
  if (m->d_blkx) hipFree(m->d_blkx);
  if (m->d_slot2) hipFree(m->d_slot2);
  if (m->d_ctr) hipFree(m->d_ctr);
  for (auto &q : m->exchBuf)
    if (q) hipFree(q);
  if (m->d_rec) hipFree(m->d_rec);
  if (m->mwgShared) (void)hipIpcCloseMemHandle(m->mwgShared);
  for (void *q : m->mwgAllocs) hipFree(q);
  for (int q = 0; q < 2; q++) {
    if (m->stHost[q]) hipHostFree(m->stHost[q]);
    if (m->stEv[q]) hipEventDestroy(m->stEv[q]);
    if (m->stCopied[q]) hipEventDestroy(m->stCopied[q]);
    if (m->stDev[q]) hipFree(m->stDev[q]);
  }
  if (m->stCopy) hipStreamDestroy(m->stCopy);
  if (m->ownStream) hipStreamDestroy(m->ownStream);
  if (m->stream2) hipStreamDestroy(m->stream2);
  if (m->evFork) hipEventDestroy(m->evFork);
  if (m->evSnap) hipEventDestroy(m->evSnap);
  if (m->evHand) hipEventDestroy(m->evHand);
  if (m->stream3) hipStreamDestroy(m->stream3);
  if (m->evEta0) hipEventDestroy(m->evEta0);
  if (m->evEta1) hipEventDestroy(m->evEta1);
  if (m->evJoin) hipEventDestroy(m->evJoin);
  for (auto &ev : m->ovlEv)
    if (ev) hipEventDestroy(ev);
  delete m;
}

int mgcm_set_param(mgcm_model *m, const char *name, double value) {
  drop_graphs(m);   // kernel arguments are captured by value
  if (!strcmp(name, "myIter")) {  // the device-side iteration counter (AB2 start, solve records)
    int it = (int)value;
    HIPCHK(hipSetDevice(m->device));
    HIPCHK(hipMemcpyAsync(m->d_ctr, &it, sizeof(int), hipMemcpyHostToDevice, m->stream));
    HIPCHK(hipStreamSynchronize(m->stream));
    return 0;
  }
  for (auto &pd : PARAMS)
    if (!strcmp(pd.name, name)) {
      char *ptr = reinterpret_cast<char *>(&m->p) + pd.off;
      if (pd.isint) *reinterpret_cast<int *>(ptr) = (int)value;
      else *reinterpret_cast<double *>(ptr) = value;
      return 0;
    }
  // options the kernels do not implement are accepted only at their default
  // (inert) value; anything else is an explicit error, never silently ignored.
  static const char *inert[] = {"implicitFreeSurface"};
  for (auto *n : inert)
    if (!strcmp(n, name)) {
      const bool isDefaultOff = (value == 0.0) || (!strcmp(n, "implicitFreeSurface") && value == 1.0);
      if (!isDefaultOff) return set_err("mgcm_set_param: option %s=%g is not supported by the device path yet", name, value);
      m->extra[name] = value;
      return 0;
    }
  m->extra[name] = value;
  return 0;
}

namespace mgcm {
__global__ void k_set_iter(int *ctr, int v) {
  if (threadIdx.x == 0) ctr[0] = v;
}
__global__ void k_add_iter(int *ctr, int inc) {
  if (threadIdx.x == 0) ctr[0] += inc;
}
}  // namespace mgcm

int mgcm_add_iter(mgcm_model *m, int inc) {
  HIPCHK(hipSetDevice(m->device));
  hipLaunchKernelGGL(mgcm::k_add_iter, dim3(1), dim3(64), 0, m->stream, m->d_ctr, inc);
  HIPCHK(hipGetLastError());
  return 0;
}

int mgcm_set_iter(mgcm_model *m, int myIter) {
  HIPCHK(hipSetDevice(m->device));
  hipLaunchKernelGGL(mgcm::k_set_iter, dim3(1), dim3(64), 0, m->stream, m->d_ctr, myIter);
  HIPCHK(hipGetLastError());
  return 0;
}

double mgcm_get_param(mgcm_model *m, const char *name) {
  if (!strcmp(name, "myIter")) {
    int it = 0;
    if (hipMemcpyAsync(&it, m->d_ctr, sizeof(int), hipMemcpyDeviceToHost, m->stream) != hipSuccess ||
        hipStreamSynchronize(m->stream) != hipSuccess)
      return NAN;
    return it;
  }
  // 5: k_cg2d_block in the reference order (cg2dRefOrder), 4: k_cg2d_mwg, 3: k_cg2d_bxy, 2: k_cg2d_blk2, 1: k_cg2d_block
  if (!strcmp(name, "cg2dKernel"))
    return m->p.cg2dRefOrder ? 5.0 : m->useMwg ? 4.0 : m->nBlkX > 0 ? 3.0 : (m->nBlk > 0 ? 2.0 : 1.0);
  if (!strcmp(name, "cg2dParts")) return m->useMwg ? (double)m->mwg.G : 1.0;
  // 1 when the multi-workgroup solve's parts are placed on one XCD (one L2: ~1 us hand-offs)
  if (!strcmp(name, "cg2dPinned")) return m->useMwg ? (double)m->mwg.pinned : 0.0;
  // THERMODYNAMICS on the second stream: 1 on, 0 off; -1 while the graph path is still timing
  // both (ovlMsOn / ovlMsOff: ovl_trial's event times of the two graphs, 8 steps each)
  if (!strcmp(name, "overlap")) return (m->ovlAuto && !m->ovlDecided) ? -1.0 : (m->overlap ? 1.0 : 0.0);
  if (!strcmp(name, "ovlMsOn")) return m->ovlMs[1];
  if (!strcmp(name, "ovlMsOff")) return m->ovlMs[0];
  if (!strcmp(name, "cg2dBxyVariant")) return (double)m->bxyVar;
  // the launch layout of the last FORWARD_STEP built (one_step): bit 0 THERMODYNAMICS folded
  // into DYNAMICS' grids (k_dt_l1/l2/l3), 1 DO_OCEANIC_PHYS + CALC_PHI_HYD in one pass,
  // 2 the tracers on the second stream, 3 joined only before the correction step
  if (!strcmp(name, "stepLayout")) return (double)m->stepLayout;
  // whether the selected kernel solves with fused multiply-adds (k_cg2d_bxy honours cg2dUseFMA)
  if (!strcmp(name, "cg2dFMA")) return (!m->p.cg2dRefOrder && !m->useMwg && m->nBlkX > 0 && m->p.cg2dUseFMA) ? 1.0 : 0.0;
  for (auto &pd : PARAMS)
    if (!strcmp(pd.name, name)) {
      const char *ptr = reinterpret_cast<const char *>(&m->p) + pd.off;
      return pd.isint ? (double)*reinterpret_cast<const int *>(ptr) : *reinterpret_cast<const double *>(ptr);
    }
  auto it = m->extra.find(name);
  return it == m->extra.end() ? NAN : it->second;
}

int mgcm_put(mgcm_model *m, const char *name, const double *host, long count) {
  const FieldDesc *fd = find_field(name);
  if (!fd) return set_err("mgcm_put: unknown field %s", name);
  const long n = field_count(m, fd->kind);
  if (count > n || count <= 0) return set_err("mgcm_put: %s count %ld > %ld", name, count, n);
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(mg_host_copy(field_ptr(m, fd), host, count * sizeof(double), hipMemcpyHostToDevice, m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  return 0;
}

namespace mgcm {
// The values of a staged batch to their fields: blockIdx.y = the field, its header entry
// (destination, start) read from the batch itself
__global__ void __launch_bounds__(256) k_put_scatter(const char *batch) {
  const long *hdr = reinterpret_cast<const long *>(batch);
  const long n = hdr[0];
  const int y = blockIdx.y;
  if (y >= n) return;
  double *dst = reinterpret_cast<double *>(hdr[1 + y]);
  const long o0 = hdr[1 + n + y], o1 = hdr[2 + n + y];
  const double *src = reinterpret_cast<const double *>(batch) + 2 + 2 * n;
  for (long i = o0 + blockIdx.x * 256L + threadIdx.x; i < o1; i += (long)gridDim.x * 256L) dst[i - o0] = src[i];
}
}  // namespace mgcm

// mgcm_put of n fields in stream order, without a host synchronisation: the host arrays are
// copied into a pinned slot as [n | destinations | starts | values], which goes up in one
// copy and is scattered to the fields by one launch.  A slot is reused only after its
// previous copy (two calls back) completed, so a step's upload never waits on the step before
// it; the host arrays may be reused as soon as the call returns.
int mgcm_put_batch_async(mgcm_model *m, int n, const char *const *names, const double *const *hosts,
                         const long *counts) {
  if (n <= 0) return 0;
  std::vector<double *> dst(n);
  long total = 0, maxc = 0;
  for (int i = 0; i < n; i++) {
    const FieldDesc *fd = find_field(names[i]);
    if (!fd) return set_err("mgcm_put_batch_async: unknown field %s", names[i]);
    const long lim = field_count(m, fd->kind);
    if (counts[i] > lim || counts[i] <= 0)
      return set_err("mgcm_put_batch_async: %s count %ld > %ld", names[i], counts[i], lim);
    dst[i] = field_ptr(m, fd);
    total += counts[i];
    maxc = std::max(maxc, counts[i]);
  }
  HIPCHK(hipSetDevice(m->device));
  const size_t bytes = (size_t)(2 + 2 * n + total) * sizeof(double);
  if (m->stCap < bytes) {
    HIPCHK(hipStreamSynchronize(m->stream));
    if (m->stCopy) HIPCHK(hipStreamSynchronize(m->stCopy));
    else HIPCHK(hipStreamCreateWithFlags(&m->stCopy, hipStreamNonBlocking));
    for (int q = 0; q < 2; q++) {
      if (m->stHost[q]) HIPCHK(hipHostFree(m->stHost[q]));
      if (m->stDev[q]) HIPCHK(hipFree(m->stDev[q]));
      m->stHost[q] = nullptr;
      m->stDev[q] = nullptr;
      HIPCHK(hipHostMalloc((void **)&m->stHost[q], bytes, hipHostMallocDefault));
      HIPCHK(hipMalloc((void **)&m->stDev[q], bytes));
      if (!m->stEv[q]) HIPCHK(hipEventCreateWithFlags(&m->stEv[q], hipEventDisableTiming));
      if (!m->stCopied[q]) HIPCHK(hipEventCreateWithFlags(&m->stCopied[q], hipEventDisableTiming));
    }
    m->stCap = bytes;
  }
  const int q = m->stNext;
  m->stNext ^= 1;
  HIPCHK(hipEventSynchronize(m->stEv[q]));   // slot q's previous scatter (two calls back) is done
  long *hdr = reinterpret_cast<long *>(m->stHost[q]);
  double *vals = reinterpret_cast<double *>(m->stHost[q]) + 2 + 2 * n;
  hdr[0] = n;
  long o = 0;
  for (int i = 0; i < n; i++) {
    hdr[1 + i] = reinterpret_cast<long>(dst[i]);
    hdr[1 + n + i] = o;
    memcpy(vals + o, hosts[i], counts[i] * sizeof(double));
    o += counts[i];
  }
  hdr[1 + 2 * n] = o;
  // the copy on the copy stream (beside whatever the model stream still runs), the scatter
  // in the model stream's order after it
  HIPCHK(hipMemcpyAsync(m->stDev[q], m->stHost[q], bytes, hipMemcpyHostToDevice, m->stCopy));
  HIPCHK(hipEventRecord(m->stCopied[q], m->stCopy));
  HIPCHK(hipStreamWaitEvent(m->stream, m->stCopied[q], 0));
  const unsigned gx = (unsigned)std::min<long>(64, (maxc + 255) / 256);
  hipLaunchKernelGGL(mgcm::k_put_scatter, dim3(gx, n), dim3(256), 0, m->stream, m->stDev[q]);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(m->stEv[q], m->stream));
  return 0;
}

int mgcm_put_async(mgcm_model *m, const char *name, const double *host, long count) {
  return mgcm_put_batch_async(m, 1, &name, &host, &count);
}

int mgcm_get(mgcm_model *m, const char *name, double *host, long count) {
  const FieldDesc *fd = find_field(name);
  if (!fd) return set_err("mgcm_get: unknown field %s", name);
  const long n = field_count(m, fd->kind);
  if (count > n || count <= 0) return set_err("mgcm_get: %s count %ld > %ld", name, count, n);
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(mg_host_copy(host, field_ptr(m, fd), count * sizeof(double), hipMemcpyDeviceToHost, m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  return 0;
}

double *mgcm_device_ptr(mgcm_model *m, const char *name) {
  const FieldDesc *fd = find_field(name);
  if (!fd) { set_err("mgcm_device_ptr: unknown field %s", name); return nullptr; }
  return field_ptr(m, fd);
}

int mgcm_set_halo_map(mgcm_model *m, const long *src_of_point, long count) {
  const long N2 = m->d.n2 * m->d.nTiles;
  if (count != N2) return set_err("mgcm_set_halo_map: count %ld != %ld", count, N2);
  m->h_halo.clear();
  // a map identical to the default lat-lon one keeps the global-index CG2D blocking
  build_latlon_halo(m);
  std::vector<long> ll = m->h_halo;
  m->h_halo.clear();
  for (long q = 0; q < N2; q++)
    if (src_of_point[q] >= 0 && src_of_point[q] != q) {
      m->h_halo.push_back(q);
      m->h_halo.push_back(src_of_point[q]);
    }
  m->latlonTopology = (ll == m->h_halo);
  m->ready = false;
  return 0;
}

int mgcm_set_uv_map(mgcm_model *m, const long *u1, const long *v1, const long *u0, const long *v0,
                    const int *tileFace, const int *tileEdge, long count) {
  const long N2 = m->d.n2 * m->d.nTiles;
  if (count != N2) return set_err("mgcm_set_uv_map: count %ld != %ld", count, N2);
  const long *src[2][2] = {{u0, v0}, {u1, v1}};
  for (int w = 0; w < 2; w++) {
    m->h_uv[w].assign((size_t)2 * N2, 0);
    for (int c = 0; c < 2; c++)
      for (long q = 0; q < N2; q++) {
        const long code = src[w][c][q];
        const long s = (code > 0 ? code : -code) - 1;
        if (code != 0 && (s < 0 || s >= 2 * N2)) return set_err("mgcm_set_uv_map: bad code %ld at %ld", code, q);
        m->h_uv[w][(size_t)c * N2 + q] = code;
      }
  }
  std::vector<int> info(2 * (size_t)m->d.nTiles);
  for (int t = 0; t < m->d.nTiles; t++) { info[t] = tileFace[t]; info[m->d.nTiles + t] = tileEdge[t]; }
  HIPCHK(hipSetDevice(m->device));
  if (m->d_tileInfo) (void)hipFree(m->d_tileInfo);
  HIPCHK(hipMalloc(&m->d_tileInfo, info.size() * sizeof(int)));
  HIPCHK(hipMemcpy(m->d_tileInfo, info.data(), info.size() * sizeof(int), hipMemcpyHostToDevice));
  m->f.tileFace = m->d_tileInfo;
  m->f.tileEdge = m->d_tileInfo + m->d.nTiles;
  m->p.cubeCorners = 1;
  m->uvMap = true;
  m->ready = false;
  drop_graphs(m);
  return 0;
}

// EXCH_UV_XYZ_RL / EXCH_UV_XY_RL of a C-grid vector pair: the EXCH2 vector map when one
// is installed, else the two components through the scalar (EXCH1) map.
static int exchange_uv(mgcm_model *m, double *u, double *v, int nz, bool withSigns) {
  if (!m->uvMap) {
    HIPCHK(launch_exchange(m->d, u, m->d_halo, m->nHalo, nz, m->stream));
    HIPCHK(launch_exchange(m->d, v, m->d_halo, m->nHalo, nz, m->stream));
    return 0;
  }
  const int w = withSigns ? 1 : 0;
  HIPCHK(launch_exchange_uv(m->d, u, v, m->d_uv[w], m->nUvU[w], m->nUvV[w], nz, m->stream));
  return 0;
}

// CALC_R_STAR (calc_r_star.F): on an EXCH2 topology k_calc_r_star evaluates the W/S
// factors in place and EXCH_UV_XY_RL(rStarFacW, rStarFacS, .FALSE.) (calc_r_star.F:256-257)
// refills their halos through the vector map; rStarDh*Dt and rStarExp* are pointwise
// functions of the new and old factors, so their halos are the same copies.
// In tile-sharded runs every process holds the whole 2-D state after the free-surface
// gathers, so the r* state (factors, hFac, CG2D operator) is recomputed on EVERY tile,
// redundantly and identically: no communication, and the replicated CG2D sees the global
// operator.
static Dims all_tiles(const Dims &d) { Dims a = d; a.t0 = 0; a.nT = d.nTiles; return a; }

// stagEx (cube/LLC maps, the whole domain): DO_STAGGER_FIELDS_EXCHANGES' u, v, w ride in
// CALC_R_STAR's grid (k_rstar_exmix, MG_FUSE_ENDS)
static hipError_t calc_r_star(mgcm_model *m, bool fuseEtaH = false, int fromX = 0, bool stagEx = false) {
  const Dims da = all_tiles(m->d);
  hipError_t e;
  if (stagEx) {
    XFields xw{};
    xw.p[0] = m->f.wVel; xw.nz[0] = m->d.Nr; xw.n = 1;
    e = launch_rstar_exmix(da, m->p, m->f, m->d_srcOf, fuseEtaH, fromX, m->f.uVel, m->f.vVel, m->d.Nr, m->d_uv[1],
                           m->nUvU[1], m->nUvV[1], xw, m->d_halo, m->nHalo, m->stream);
  } else
    e = launch_calc_r_star(da, m->p, m->f, m->d_srcOf, m->stream, fuseEtaH, fromX);
  if (e != hipSuccess || !m->uvMap) return e;
  double *us[3] = {m->f.rStarFacW, m->f.rStarDhWDt, m->f.rStarExpW}, *vs[3] = {m->f.rStarFacS, m->f.rStarDhSDt,
                                                                                 m->f.rStarExpS};
  return launch_exchange_uv_pairs(da, us, vs, 3, m->d_uvAll[0], m->nUvUAll[0], m->nUvVAll[0], m->stream);
}
// sfp: k_sfp_rhs fused into the r* column pass (FORWARD_STEP on the whole domain only: in a
// tile-sharded run the r* pass covers every tile and the right-hand side this process's own)
static hipError_t update_r_star_cg2d(mgcm_model *m, bool sfp = false, bool opEarly = false, bool pcHere = false) {
  return launch_update_r_star_cg2d(all_tiles(m->d), m->p, m->f, m->d_srcOf, m->stream, sfp, opEarly, pcHere);
}

int mgcm_init(mgcm_model *m) {
  auto ext = [&](const char *n, double dflt) { auto it = m->extra.find(n); return it == m->extra.end() ? dflt : it->second; };
  HIPCHK(hipSetDevice(m->device));
  // the hFac snapshot THERMODYNAMICS reads beside the pressure solve under r* (one_step)
  if (!m->snapH && m->p.nonlinFreeSurf > 0 && m->p.select_rStar > 0 && (m->p.tempStepping || m->p.saltStepping)) {
    HIPCHK(hipMalloc(&m->snapH, 6 * (size_t)m->d.N3all * sizeof(double)));
    m->allocs.push_back(m->snapH);
  }
  if (upload_halo(m)) return -1;
  if (build_nbr(m)) return -1;
  // CG2D kernel: the single-workgroup blocked solvers on lat-lon grids that tile into their
  // blocks; otherwise the multi-workgroup solver (the generic single-workgroup kernel measured
  // 12.7 against 4.2 us/iteration on the cube, round 3)
  m->useMwg = false;
  // cg2dRefOrder: the generic single-workgroup kernel with the reference's summation order
  // (parity runs on the reference's own tiling; refused where it does not fit one workgroup)
  if (m->p.cg2dRefOrder) {
    if (m->nPts > cg2d_ref_max_points())
      return set_err("mgcm_init: cg2dRefOrder needs <= %d interior points (one workgroup), have %d",
                     cg2d_ref_max_points(), m->nPts);
    if (m->p.useSRCGSolver) return set_err("mgcm_init: cg2dRefOrder with useSRCGSolver not implemented");
  } else if ((m->nBlkX == 0 && m->nBlk == 0) ||
             ext("cg2dForceMwg", 0.0) != 0.0) {
    // cg2dForceMwg: the multi-workgroup solver on a grid the single-workgroup kernels would
    // take (the tile-sharded device CG2D runs its parts in several processes)
    m->nBlkX = 0;
    m->nBlk = 0;
    if (build_mwg(m)) return -1;
  }
  if (m->p.useSRCGSolver && !m->useMwg && m->nBlkX == 0)
    return set_err("mgcm_init: useSRCGSolver (CG2D_SR) is implemented in the blocked single-workgroup and the "
                   "multi-workgroup CG2D only");
  if ((m->p.viscA4D != 0.0 || m->p.viscA4Z != 0.0) && (m->d.OLx < 3 || m->d.OLy < 3))
    return set_err("mgcm_init: biharmonic viscosity needs OLx, OLy >= 3 (del2u of the halo ring)");
  const bool rstar = m->p.nonlinFreeSurf > 0;
  if (rstar) {
    if (m->p.nonlinFreeSurf != 4 || m->p.select_rStar != 2)
      return set_err("mgcm_init: the non-linear free surface is implemented for nonlinFreeSurf=4, select_rStar=2 only");
    if (!m->p.exactConserv) return set_err("mgcm_init: nonlinFreeSurf needs exactConserv");
  }
  if (m->p.selectP_inEOS_Zc > 2) return set_err("mgcm_init: selectP_inEOS_Zc = 3 needs the non-hydrostatic pressure");
  if (m->p.selectP_inEOS_Zc == 2 && !m->p.storePhiHyd4Phys)
    return set_err("mgcm_init: selectP_inEOS_Zc = 2 needs storePhiHyd4Phys (set_parms.F:297)");
  // implicitViscosity: MOM_U/V_IMPLICIT_R (k_mom_impl); with the CD scheme also IMPLDIFF on
  // vVelD / uVelD (dynamics.F:614-634, k_impldiff_cd)
  if (m->p.implicitViscosity && (ext("momImplVertAdv", 0.0) != 0.0 || ext("selectImplicitDrag", 0.0) != 0.0))
    return set_err("mgcm_init: momImplVertAdv / selectImplicitDrag not implemented on the device");
  if (m->p.vectorInvariantMomentum) {
    // the MOM_VECINV subset k_mom_step implements (see kernels_dyn.hip)
    if (m->d.OLx < 2 || m->d.OLy < 2) return set_err("mgcm_init: vector-invariant momentum needs OLx, OLy >= 2");
    if (m->p.viscA4D != 0.0 || m->p.viscA4Z != 0.0)
      return set_err("mgcm_init: biharmonic viscosity with vectorInvariantMomentum not implemented on the device");
    if (m->p.useNHMTerms || m->p.select3dCoriScheme > 0 || m->p.useCDscheme)
      return set_err("mgcm_init: NH metric / 3-D Coriolis / CD scheme with vectorInvariantMomentum not implemented");
    if (m->p.selectVortScheme < 0 || m->p.selectVortScheme > 3 || m->p.selectKEscheme < 0 || m->p.selectKEscheme > 3 ||
        m->p.selectCoriScheme < 0 || m->p.selectCoriScheme > 3)
      return set_err("mgcm_init: selectVortScheme/selectKEscheme/selectCoriScheme outside 0..3");
    auto e = m->extra.find("useAbsVorticity");
    if (e != m->extra.end() && e->second != 0.0) return set_err("mgcm_init: useAbsVorticity not implemented");
  }
  if (m->uvMap && m->p.useCDscheme) return set_err("mgcm_init: CD scheme on an EXCH2 topology not implemented");
  if (m->p.implicSurfPress != 1.0 || m->p.implicDiv2DFlow != 1.0)
    return set_err("mgcm_init: implicSurfPress/implicDiv2DFlow != 1 not supported yet");
  const bool sph = ext("usingSphericalPolarGrid", 0.0) != 0.0;
  m->p.metricSphere = sph && ext("selectMetricTerms", 1.0) >= 1.0;
  m->p.recip_rSphere = sph ? 1.0 / ext("rSphere", 6370.0e3) : 0.0;   // ini_parms.F:1334
  if (ext("integr_GeoPot", 2.0) != 2.0) return set_err("mgcm_init: only integr_GeoPot = 2 is implemented");
  // tracer advection schemes implemented on the device: 2 (C2), 3 (U3) and 4 (C4) inside
  // GAD_CALC_RHS with Adams-Bashforth on the tendency, 30 (DST3) and 33 (DST3 flux-limited)
  // multi-dimensional; the vertical scheme must match the horizontal one
  auto okScheme = [&](int s, const char *vname) {
    return (s == 2 || s == 3 || s == 4 || ((s == 30 || s == 33) && m->p.multiDimAdvection)) &&
           ext(vname, (double)s) == (double)s;
  };
  auto wideScheme = [&](int s) { return s == 3 || s == 4; };
  if (((m->p.tempStepping && wideScheme(m->p.tempAdvScheme)) || (m->p.saltStepping && wideScheme(m->p.saltAdvScheme))) &&
      (m->uvMap || m->d.OLx < 2 || m->d.OLy < 2))
    return set_err("mgcm_init: advection schemes 3 / 4 need OLx, OLy >= 2 and a lat-lon topology on the device");
  // ADAMS_BASHFORTH3 (ALLOW_ADAMSBASHFORTH_3) is restated for the tracers' tendencies only
  if (m->p.useAB3 && (m->p.momStepping || (m->p.nonlinFreeSurf > 0 && m->p.select_rStar > 0) || m->p.staggerTimeStep))
    return set_err("mgcm_init: ADAMS_BASHFORTH3 only for the tracers (momStepping off, no r*, not staggered)");
  // (a restart would need both history slots, gtNm(:,:,:,1:2), which the pickup path does not carry)
  if (m->p.useAB3 && m->p.nIter0 != 0) return set_err("mgcm_init: ADAMS_BASHFORTH3 from a pickup (nIter0 != 0) not supported");
  // the cube's multi-dimensional split (3 face-dependent passes with corner fills,
  // gad_advection.F:339-367) runs the general pass kernels (kernels_thermo.hip k_advg_*),
  // which need the tile face / edge table of the EXCH2 topology and OLx = OLy (corner fills)
  auto mdScheme = [&](int s) { return s == 30 || s == 33; };
  if (m->uvMap && ((m->p.tempStepping && mdScheme(m->p.tempAdvScheme)) || (m->p.saltStepping && mdScheme(m->p.saltAdvScheme)))) {
    if (!m->f.tileFace) return set_err("mgcm_init: multi-dimensional advection on EXCH2 needs the tile face table");
    if (m->d.OLx != m->d.OLy) return set_err("mgcm_init: cube multi-dimensional advection needs OLx = OLy");
  }
  if (m->p.tempStepping && !okScheme(m->p.tempAdvScheme, "tempVertAdvScheme"))
    return set_err("mgcm_init: tempAdvScheme %d not implemented on the device", m->p.tempAdvScheme);
  if (m->p.saltStepping && !okScheme(m->p.saltAdvScheme, "saltVertAdvScheme"))
    return set_err("mgcm_init: saltAdvScheme %d not implemented on the device", m->p.saltAdvScheme);
  if (m->p.useGMRedi && m->p.GM_AdvForm && m->p.multiDimAdvection &&
      ((m->p.tempStepping && mdScheme(m->p.tempAdvScheme)) || (m->p.saltStepping && mdScheme(m->p.saltAdvScheme))))
    return set_err("mgcm_init: GM_AdvForm with multi-dimensional advection is not implemented on the device");
  if (m->p.useGMRedi && m->p.GM_AdvForm && m->p.GM_skewflx != 0.0)
    return set_err("mgcm_init: GM_AdvForm needs GM_skewflx = 0 (gmredi_readparms.F:243-244)");
  if (m->p.eosType != 0 && m->p.eosType != 1) return set_err("mgcm_init: eosType %d not implemented", m->p.eosType);
  if (m->d.Nr > 64) return set_err("mgcm_init: Nr = %d > 64 (column kernels hold a column in one workgroup)", m->d.Nr);
  if (m->p.periodicExternalForcing && (m->p.nForcRec < 1 || m->p.nForcRec > MG_MAXREC))
    return set_err("mgcm_init: nForcRec %d outside 1..%d", m->p.nForcRec, MG_MAXREC);
  drop_graphs(m);
  m->thetaA = m->f.theta;
  m->saltA = m->f.salt;
  m->useGraph = true;
  int it0 = m->p.nIter0;
  // every copy is ordered on the model's stream (a null-stream hipMemcpy does not wait for
  // the non-blocking streams)
  HIPCHK(hipMemcpyAsync(m->d_ctr, &it0, sizeof(int), hipMemcpyHostToDevice, m->stream));
  // INI_PSURF (ini_psurf.F:84) on a cold start: etaH = etaN (a pickup holds etaH)
  if (m->p.nIter0 == 0)
    HIPCHK(hipMemcpyAsync(m->f.etaH, m->f.etaN, m->d.n2 * m->d.nTiles * sizeof(double), hipMemcpyDeviceToDevice,
                          m->stream));
  if (rstar) {
    // INITIALISE_VARIA (initialise_varia.F:299-349): CALC_R_STAR(etaH) -> UPDATE_R_STAR ->
    // UPDATE_CG2D -> INTEGR_CONTINUITY(nIter0) (+ UPDATE_ETAH, EXCH w) -> CALC_R_STAR(etaH)
    HIPCHK(calc_r_star(m));
    HIPCHK(update_r_star_cg2d(m));
    HIPCHK(launch_corr_cont(m->d, m->p, m->f, 1, m->stream));
    HIPCHK(launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, true, 1, m->stream));
    HIPCHK(launch_exchange(m->d, m->f.wVel, m->d_halo, m->nHalo, m->d.Nr, m->stream));
    HIPCHK(calc_r_star(m));
    HIPCHK(hipStreamSynchronize(m->stream));
  }
  m->ready = true;
  return 0;
}

// EXCH_XY_RL(cg2d_x) + etaN (k_exch_eta) inside the CG2D launch: the single-workgroup
// blocked solver holds the whole solution, so its epilogue writes every point's value
static bool cg2d_fuses_eta(const mgcm_model *m) {
  return !m->p.cg2dRefOrder && !m->useMwg && m->nBlkX > 0 && m->d_slot2 && m->d.nT == m->d.nTiles;
}

static hipError_t launch_cg2d(mgcm_model *m, int maxIters, int nIterMin, bool fuseEta = false) {
  if (m->p.cg2dRefOrder)
    return launch_cg2d_block(m->d, m->p, m->f, m->d_nbr, m->d_gofs, m->nPts, maxIters, nIterMin, m->d_rec, m->d_ctr + 1,
                             m->stream);
  if (m->useMwg) {
    return launch_cg2d_mwg(m->d, m->p, m->f, m->mwg, maxIters, nIterMin, m->d_rec, m->d_ctr + 1, m->stream);
  }
  if (m->nBlkX > 0)
    return launch_cg2d_bxy(m->bxyVar, m->d, m->p, m->f, m->d_nbx, m->d_blkx, m->nBlkX, maxIters, nIterMin, m->d_rec,
                           m->d_ctr + 1, fuseEta ? m->d_slot2 : nullptr, m->d_srcOf, m->stream);
  if (m->nBlk > 0)
    return launch_cg2d_blk2(m->d, m->p, m->f, m->d_nb4, m->d_blk, m->nBlk, maxIters, nIterMin, m->d_rec, m->d_ctr + 1,
                            m->stream);
  return launch_cg2d_block(m->d, m->p, m->f, m->d_nbr, m->d_gofs, m->nPts, maxIters, nIterMin, m->d_rec, m->d_ctr + 1,
                           m->stream);
}

static int check_ready(mgcm_model *m) {
  if (!m->ready) return set_err("model not initialised: call mgcm_init() after loading the fields");
  return 0;
}

#define TIMED(K, CALL)                      \
  do {                                      \
    int ev_ = ev_begin(m, K);               \
    hipError_t e_ = (CALL);                 \
    ev_end(m, K, ev_);                      \
    if (e_ != hipSuccess) return set_err("%s: %s", KNAMES[K], hipGetErrorString(e_)); \
  } while (0)

static int dynamics_on(mgcm_model *m, bool ring) {
  TIMED(K_PHI, launch_phi_hyd(m->d, m->p, m->f, m->stream));   // CALC_PHI_HYD (dynamics.F:462)
  TIMED(K_MOM, launch_mom_step(m->d, m->p, m->f, m->d_ctr, m->stream, ring));
  return 0;
}
int mgcm_dynamics(mgcm_model *m) {
  if (check_ready(m)) return -1;
  return dynamics_on(m, true);
}

static TracerArgs tracer_args(mgcm_model *m, bool salt) {
  const Params &p = m->p;
  TracerArgs a{};
  const int scheme = salt ? p.saltAdvScheme : p.tempAdvScheme;
  a.tr = salt ? m->f.salt : m->f.theta;
  a.trNext = salt ? m->f.saltNext : m->f.thetaNext;
  a.gNm1 = salt ? m->f.gsNm1 : m->f.gtNm1;
  a.scr = salt ? m->f.cpScr : m->f.gTscr;   // own scratch each: the two may run concurrently
  a.cp = salt ? m->f.advScr2 : m->f.advScr1;
  a.sfc = salt ? m->f.surfaceForcingS : m->f.surfaceForcingT;
  a.diffKh = salt ? p.diffKhS : p.diffKhT;
  a.diffKr = salt ? p.diffKrS : p.diffKrT;
  a.dT = p.deltaTtracer;
  a.advection = salt ? p.saltAdvection : p.tempAdvection;
  a.forcing = salt ? p.saltForcing : p.tempForcing;
  // gad_init_fixed.F:126-162: multi-dim advection for the schemes that are not
  // Adams-Bashforth ones; AB (2 or 3) on the tendency for C2, U3 and C4
  const bool abScheme = scheme == 2 || scheme == 3 || scheme == 4;
  a.multiDim = p.multiDimAdvection && a.advection && !abScheme;
  a.useAB = abScheme;
  a.limiter = scheme == 33;   // DST3 (30) without, DST3FL (33) with the flux limiter
  a.scheme = scheme;
  a.gNm2 = salt ? m->f.gsNm2 : m->f.gtNm2;
  return a;
}

// TEMP_INTEGRATE / SALT_INTEGRATE on stream `st` (the theta/salt ping-pong swap is host-side)
static int tracers_on(mgcm_model *m, hipStream_t st, const Fields *fo = nullptr) {
  const TracerArgs aT = tracer_args(m, false), aS = tracer_args(m, true);
  const Fields &F = fo ? *fo : m->f;   // the fields the kernels read (fo: the hFac snapshot)
  if (tracer_hpair_ok(m->d, m->p, aT, aS)) {   // small grids: both tracers per launch
    TIMED(K_TEMP, launch_tracer_hpair(m->d, m->p, F, aT, aS, m->d_ctr, st));
    std::swap(m->f.theta, m->f.thetaNext);
    std::swap(m->f.salt, m->f.saltNext);
    return 0;
  }
  if (m->p.tempStepping) {
    TIMED(K_TEMP, launch_tracer_step(m->d, m->p, F, tracer_args(m, false), m->d_ctr, st));
    std::swap(m->f.theta, m->f.thetaNext);   // CYCLE_TRACER: the new theta is the other buffer
  }
  if (m->p.saltStepping) {
    TIMED(K_TEMP, launch_tracer_step(m->d, m->p, F, tracer_args(m, true), m->d_ctr, st));
    std::swap(m->f.salt, m->f.saltNext);
  }
  return 0;
}

int mgcm_thermodynamics(mgcm_model *m) {
  if (check_ready(m)) return -1;
  // forward_step.F:656 DO_OCEANIC_PHYS (every step: forcing records, EOS, GM tensor),
  // :732 THERMODYNAMICS (staggerTimeStep = F; the tracers only when stepped)
  TIMED(K_PHYS, launch_oceanic_phys(m->d, m->p, m->f, m->d_ctr, m->stream));
  return tracers_on(m, m->stream);
}

// The routine-level ops run the same kernels as one_step, split at the reference's
// routine boundaries (forward_step.F:925-976), so a host that calls them in FORWARD_STEP
// order reproduces mgcm_forward_step bit for bit.
static int solve_impl(mgcm_model *m) {
  TIMED(K_RHS, launch_sfp_rhs(m->d, m->p, m->f, m->stream));
  const int nIterMin = m->p.cg2dUseMinResSol - 1;
  TIMED(K_CG2D, launch_cg2d(m, m->p.cg2dMaxIters, nIterMin));
  // EXCH_XY_RL(cg2d_x) + etaN = recip_Bo*cg2d_x (solve_for_pressure.F:309-330)
  TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, false, 0, m->stream));
  return 0;
}

int mgcm_solve_for_pressure(mgcm_model *m) {
  if (check_ready(m)) return -1;
  return solve_impl(m);
}

int mgcm_momentum_correction_step(mgcm_model *m) {
  if (check_ready(m)) return -1;
  TIMED(K_CORR, launch_correction(m->d, m->p, m->f, m->stream));
  return 0;
}

int mgcm_integr_continuity(mgcm_model *m) {
  if (check_ready(m)) return -1;
  // integr_continuity.F:66-310 (exactConserv eta, INTEGRATE_FOR_W incl. r*) from the corrected
  // uVel, vVel; :324-350 EXCH etaN + UPDATE_ETAH (PmEpR under real fresh water)
  TIMED(K_CONT, launch_corr_cont(m->d, m->p, m->f, 2, m->stream));
  if (m->p.exactConserv) TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, true, 0, m->stream));
  return 0;
}

int mgcm_update_r_star(mgcm_model *m) {
  if (check_ready(m)) return -1;
  // UPDATE_R_STAR(.TRUE.) + UPDATE_CG2D (forward_step.F:829-877)
  if (m->p.nonlinFreeSurf > 0) TIMED(K_RSTAR, update_r_star_cg2d(m));
  return 0;
}

int mgcm_calc_r_star(mgcm_model *m) {
  if (check_ready(m)) return -1;
  // CALC_R_STAR(etaH) (forward_step.F:965-977)
  if (m->p.nonlinFreeSurf > 0) TIMED(K_RSTAR, calc_r_star(m));
  return 0;
}

static XFields blocking_fields(const mgcm_model *m, int tracers = 1);

int mgcm_blocking_exchanges(mgcm_model *m) {
  if (check_ready(m)) return -1;
  // DO_FIELDS_BLOCKING_EXCHANGES (do_fields_blocking_exchanges.F:54-97): the set FORWARD_STEP
  // exchanges (one_step), without advancing the step counter
  if (m->uvMap) TIMED(K_EXCH, exchange_uv(m, m->f.uVel, m->f.vVel, m->d.Nr, true) ? hipErrorUnknown : hipSuccess);
  TIMED(K_EXCH, launch_exchange_multi(m->d, blocking_fields(m), m->d_halo, m->nHalo, nullptr, m->stream));
  return 0;
}

int mgcm_stagger_exchanges(mgcm_model *m) {
  if (check_ready(m)) return -1;
  // DO_STAGGER_FIELDS_EXCHANGES (do_stagger_fields_exchanges.F:37-43): EXCH_UV_3D_RL(uVel,
  // vVel, .TRUE.) and EXCH_3D_RL(wVel) before the staggered THERMODYNAMICS -- the exchange
  // one_step makes there
  if (m->uvMap) {
    XFields xw{};
    xw.p[0] = m->f.wVel; xw.nz[0] = m->d.Nr; xw.n = 1;
    TIMED(K_EXCH, launch_exchange_mixed(m->d, m->f.uVel, m->f.vVel, m->d.Nr, m->d_uv[1], m->nUvU[1], m->nUvV[1], xw,
                                        m->d_halo, m->nHalo, nullptr, m->stream));
  } else {
    TIMED(K_EXCH, exchange_uv(m, m->f.uVel, m->f.vVel, m->d.Nr, true) ? hipErrorUnknown : hipSuccess);
    TIMED(K_EXCH, launch_exchange(m->d, m->f.wVel, m->d_halo, m->nHalo, m->d.Nr, m->stream));
  }
  return 0;
}

int mgcm_oceanic_phys(mgcm_model *m) {
  if (check_ready(m)) return -1;
  TIMED(K_PHYS, launch_oceanic_phys(m->d, m->p, m->f, m->d_ctr, m->stream));
  return 0;
}

int mgcm_tracer_step(mgcm_model *m) {
  if (check_ready(m)) return -1;
  return tracers_on(m, m->stream);
}

// EXCH_XY_RL / EXCH_XYZ_RL / EXCH_UV_*_RL on a caller's (host) array: staged through a
// device scratch pair, exchanged with the model's maps, copied back.
static int exch_scratch(mgcm_model *m, int nz) {
  const long need = (long)nz * m->d.n2 * m->d.nTiles;
  if (need <= m->exchCap) return 0;
  for (auto &q : m->exchBuf)
    if (q) { hipFree(q); q = nullptr; }
  HIPCHK(hipMalloc(&m->exchBuf[0], need * sizeof(double)));
  HIPCHK(hipMalloc(&m->exchBuf[1], need * sizeof(double)));
  m->exchCap = need;
  return 0;
}

int mgcm_exchange_host(mgcm_model *m, double *u, double *v, int nz, int vector, int withSigns) {
  // needs only the halo maps (usable before mgcm_init: the reference exchanges while
  // initialising, e.g. INI_FIELDS)
  if (!m->d_srcOf && upload_halo(m)) return -1;
  if (nz < 1 || nz > m->d.Nr) return set_err("mgcm_exchange_host: nz = %d outside 1..%d", nz, m->d.Nr);
  if (vector && !v) return set_err("mgcm_exchange_host: a vector exchange needs both components");
  if (exch_scratch(m, nz)) return -1;
  HIPCHK(hipSetDevice(m->device));
  const size_t bytes = (size_t)nz * m->d.n2 * m->d.nTiles * sizeof(double);
  double *host[2] = {u, v};
  for (int c = 0; c < 2; c++)
    if (host[c]) HIPCHK(mg_host_copy(m->exchBuf[c], host[c], bytes, hipMemcpyHostToDevice, m->stream));
  // every tile's halo, also when this model steps a tile subset (the host array is the domain)
  const long *hmap = m->d_haloAll ? m->d_haloAll : m->d_halo;
  const int nh = m->d_haloAll ? m->nHaloAll : m->nHalo;
  if (vector && m->uvMap) {
    const int w = withSigns ? 1 : 0;
    HIPCHK(launch_exchange_uv(m->d, m->exchBuf[0], m->exchBuf[1], m->d_uvAll[w], m->nUvUAll[w], m->nUvVAll[w], nz,
                              m->stream));
  } else {
    for (int c = 0; c < 2; c++)
      if (host[c]) HIPCHK(launch_exchange(m->d, m->exchBuf[c], hmap, nh, nz, m->stream));
  }
  for (int c = 0; c < 2; c++)
    if (host[c]) HIPCHK(mg_host_copy(host[c], m->exchBuf[c], bytes, hipMemcpyDeviceToHost, m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  return 0;
}

const char *mgcm_param_name(int i) {
  const int n = (int)(sizeof(PARAMS) / sizeof(PARAMS[0]));
  return (i >= 0 && i < n) ? PARAMS[i].name : nullptr;
}

long mgcm_field_count(mgcm_model *m, const char *name) {
  const FieldDesc *fd = find_field(name);
  if (!fd) { set_err("mgcm_field_count: unknown field %s", name); return -1; }
  return field_count(m, fd->kind);
}

// tracers: 1 every field (the reference's set), 0 without theta/salt (exchanged beside the
// pressure solve, one_step), 2 theta/salt only
static XFields blocking_fields(const mgcm_model *m, int tracers) {
  XFields x{};
  // do_fields_blocking_exchanges.F:54-97 (+ EXCH_UV_DGRID of uVelD/vVelD with the CD scheme,
  // totPhiHyd when the EOS reads it)
  // (on an EXCH2 topology u, v go through the vector map instead: exchange_uv)
  double *fl[] = {m->f.uVel, m->f.vVel, m->f.wVel, m->f.theta, m->f.salt, m->f.uVelD, m->f.vVelD, m->f.totPhiHyd};
  const bool use[] = {!m->uvMap, !m->uvMap, true, m->p.tempStepping != 0, m->p.saltStepping != 0, m->p.useCDscheme != 0,
                      m->p.useCDscheme != 0, m->p.storePhiHyd4Phys != 0};
  for (int q = 0; q < 8; q++) {
    const bool tr = q == 3 || q == 4;
    if (use[q] && (tracers == 1 || (tracers == 2) == tr)) { x.p[x.n] = fl[q]; x.nz[x.n] = m->d.Nr; x.n++; }
  }
  return x;
}

// One FORWARD_STEP with the fused end-of-step kernels: EXCH(cg2d_x)+etaN,
// correction+continuity, EXCH(eta)+UPDATE_ETAH, and every blocking exchange plus
// the counter bump in one launch.  Same arithmetic as the separate C-ABI ops.
static int one_step(mgcm_model *m) {
  // THERMODYNAMICS reads u, v, w, hFac and DO_OCEANIC_PHYS's outputs and writes only the
  // tracers' other buffers and AB histories; DYNAMICS reads none of those.  So once
  // DO_OCEANIC_PHYS is done the two run concurrently (second stream), joined before
  // UPDATE_R_STAR / SOLVE_FOR_PRESSURE (which rewrite hFac, then u, v, w).
  // staggerTimeStep (forward_step.F:1003-1036): THERMODYNAMICS after the pressure solve and
  // continuity, with the new velocities; DO_OCEANIC_PHYS still opens the step
  const bool stagger = m->p.staggerTimeStep != 0 && m->p.momStepping;
  const bool tracers = m->p.tempStepping || m->p.saltStepping;
  const bool fork = !stagger && m->overlap && !m->timing && m->p.momStepping && tracers;
  bool endFused = false;   // CALC_R_STAR + blocking exchanges in one launch (below)
  bool stagEx = false;     // CALC_R_STAR + the staggered exchanges in one launch (below)
  // Under the linear free surface nothing between DYNAMICS and the correction step touches
  // what THERMODYNAMICS reads or writes (no r* rewrite of hFac; SOLVE_FOR_PRESSURE and CG2D
  // read gU, gV, hFac and eta, write the solver's vectors and etaN), so the tracers may run
  // beside the pressure solve too and join before MOMENTUM_CORRECTION_STEP rewrites u, v, w.
  // The fork comes after CALC_DIV_GHAT (beside the CG2D: the pressure solve leaves most CUs
  // idle while DYNAMICS and CALC_DIV_GHAT, alone, have the chip), under the linear free
  // surface only.  LLC-90 round 3 (profiles/r03/thermo_at/): 1.98 ms forked after
  // DO_OCEANIC_PHYS, 1.86 after DYNAMICS, 1.88 after CALC_DIV_GHAT; round 5, with the faster
  // solve, after CALC_DIV_GHAT wins (below)
  const bool lateJoin = fork && m->p.nonlinFreeSurf <= 0;
  const bool thermoLate = lateJoin;
  // With the late join (THERMODYNAMICS beside the pressure solve) the new tracers' halos are
  // filled on the tracers' stream right after them -- DO_FIELDS_BLOCKING_EXCHANGES' theta and
  // salt, which nothing before it reads -- so the end-of-step exchange carries only the
  // velocities (MG_FUSE_TREX)
  const bool trEx = lateJoin && mg_fuse_on(MG_FUSE_TREX);
  // the VI path's halo-ring AB2 (launch_mom_ring) on the tracers' stream with them, when they
  // fork right after DYNAMICS (MG_FUSE_RING; joined with them before the correction step)
  const bool ringAside = thermoLate && mom_ring_separable(m->d, m->p) && mg_fuse_on(MG_FUSE_RING);
  auto fork_thermo = [&]() -> int {
    HIPCHK(hipEventRecord(m->evFork, m->stream));
    HIPCHK(hipStreamWaitEvent(m->stream2, m->evFork, 0));
    if (ringAside) HIPCHK(launch_mom_ring(m->d, m->p, m->f, m->d_ctr, m->stream2));
    if (tracers_on(m, m->stream2)) return -1;
    if (trEx) {
      const XFields xt = blocking_fields(m, 2);
      if (xt.n > 0) HIPCHK(launch_exchange_multi(m->d, xt, m->d_halo, m->nHalo, nullptr, m->stream2));
    }
    HIPCHK(hipEventRecord(m->evJoin, m->stream2));
    return 0;
  };
  // Early fork on a small grid: THERMODYNAMICS' tracer kernels share DYNAMICS' launches
  // (kernels_step.hip, MG_FUSE_DT) instead of running on the second stream -- no fork, no join
  const TracerArgs aT = tracer_args(m, false), aS = tracer_args(m, true);
  // (decided without the timing switch: one stream, so the eager timed pass runs the layout
  // the graph replays -- bench.py's per-kernel times and PMC attribution then describe it)
  const bool forkable = !stagger && m->overlap && m->p.momStepping && tracers;
  // THERMODYNAMICS beside the pressure solve under r* too (MG_FUSE_TCG): UPDATE_R_STAR(.TRUE.)
  // rewrites the hFac it reads before the solve, so it reads a copy taken on its own stream
  // right after the fork -- the hFac of the step's start, the values FORWARD_STEP's order
  // gives it.  DYNAMICS runs alone (no fold), UPDATE_R_STAR waits only for the copy, the
  // correction step for the tracers.  Opt-in (MGCM_STEP_FUSE |= 512): bit-identical, but on
  // config 2 the fold into DYNAMICS' launches stays faster, 0.2885 against 0.307 ms/step
  // (profiles/r04/tcg/): the tracers' launches beside DYNAMICS cost more than the 190 us
  // single-CU solve they could hide behind
  const bool tcg = forkable && m->p.nonlinFreeSurf > 0 && m->p.select_rStar > 0 && m->snapH &&
                   mg_fuse_on(MG_FUSE_TCG);
  const bool tcgFork = tcg && fork;
  const bool dtFused = forkable && !tcg && m->p.nonlinFreeSurf > 0 &&
                       dyn_thermo_fusable(m->d, m->p, aT, aS);
  auto fork_tcg = [&]() -> int {
    HIPCHK(hipEventRecord(m->evFork, m->stream));
    HIPCHK(hipStreamWaitEvent(m->stream2, m->evFork, 0));
    HIPCHK(launch_hfac_snapshot(m->d, m->f, m->snapH, m->stream2));
    HIPCHK(hipEventRecord(m->evSnap, m->stream2));
    HIPCHK(launch_gm_tensor(m->d, m->p, m->f, m->stream2));
    const Fields fT = hfac_snapshot_fields(m->d, m->f, m->snapH);
    if (tracers_on(m, m->stream2, &fT)) return -1;
    HIPCHK(hipEventRecord(m->evJoin, m->stream2));
    return 0;
  };
  // the multi-workgroup CG2D keeps its CUs to itself while the tracers run beside it
  m->mwg.exclusive = thermoLate ? 1 : 0;
  // DO_OCEANIC_PHYS + DYNAMICS' CALC_PHI_HYD in one column pass where exact (phys_phi_fusable:
  // THERMODYNAMICS, between them in FORWARD_STEP, reads DO_OCEANIC_PHYS's output and writes
  // nothing CALC_PHI_HYD reads)
  const bool physPhi = !stagger && m->p.momStepping && phys_phi_fusable(m->d, m->p);
  // (the graph's layout: the eager timed pass, one stream, serialises a fork it reports here)
  m->stepLayout = (dtFused ? 1 : 0) | (physPhi ? 2 : 0) | (forkable && !dtFused ? 4 : 0) |
                  ((forkable && m->p.nonlinFreeSurf <= 0) || tcg ? 8 : 0);
  // GMREDI_CALC_TENSOR beside CALC_PHI_HYD (launch_gm_phi) where THERMODYNAMICS, its reader,
  // runs after DYNAMICS (staggered, or forked after CALC_DIV_GHAT) and the fold does not apply
  const bool gmPhi = (stagger || thermoLate) && !dtFused && !physPhi && !m->timing && gm_phi_fusable(m->d, m->p);
  // the VI path's halo-ring AB2 in DO_OCEANIC_PHYS's grid where it is not beside the solve
  // (k_phys_ring, MG_FUSE_RINGP: the staggered cube)
  bool ringPhys = false;
  const bool ringPhysOk = !ringAside && !physPhi && mom_ring_separable(m->d, m->p) && mg_fuse_on(MG_FUSE_RINGP);
  auto phys = [&]() -> int {
    if (physPhi) TIMED(K_PHYS, launch_phys_phi(m->d, m->p, m->f, m->d_ctr, m->stream));
    // (GMREDI_CALC_TENSOR in launch_dyn_thermo's first grid when it takes it)
    else TIMED(K_PHYS, launch_oceanic_phys(m->d, m->p, m->f, m->d_ctr, m->stream,
                                           !(dtFused && dyn_thermo_takes_gm(m->p)) && !gmPhi && !tcgFork,
                                           ringPhysOk ? &ringPhys : nullptr));
    return 0;
  };
  if (stagger || fork || dtFused) {
    if (phys()) return -1;
    if (tcgFork) {
      if (fork_tcg()) return -1;
    } else if (fork && !thermoLate && !dtFused && fork_thermo()) return -1;
  } else {
    if (phys() || tracers_on(m, m->stream)) return -1;
  }
  // UPDATE_CG2D beside DYNAMICS (ucg2d.h, MG_FUSE_OPE): the operator from h0Fac*rStarFac in
  // the fold's first grid, the preconditioner in its second; UPDATE_R_STAR then rewrites hFac only
  const bool opEarly = dtFused && m->p.nonlinFreeSurf > 2 && dyn_thermo_takes_gm(m->p) && m->d.nT == m->d.nTiles &&
                       mg_fuse_on(MG_FUSE_OPE);
  // (round 4 measured the operator also in GMREDI_CALC_TENSOR + CALC_PHI_HYD's grid on the
  // staggered cube: slower, 0.4235-0.4257 against 0.4165-0.4234 ms/step, profiles/r04/ope_cs/;
  // removed in round 5)
  if (m->p.momStepping) {
    if (dtFused) {
      TIMED(K_MOM, launch_dyn_thermo(m->d, m->p, m->f, aT, aS, m->d_ctr, m->stream, opEarly ? m->d_srcOf : nullptr));
      std::swap(m->f.theta, m->f.thetaNext);   // CYCLE_TRACER: the new tracers are the other buffers
      std::swap(m->f.salt, m->f.saltNext);
    } else if (physPhi) TIMED(K_MOM, launch_mom_step(m->d, m->p, m->f, m->d_ctr, m->stream, !ringAside && !ringPhys));
    else if (gmPhi) {
      TIMED(K_PHI, launch_gm_phi(m->d, m->p, m->f, m->stream));
      TIMED(K_MOM, launch_mom_step(m->d, m->p, m->f, m->d_ctr, m->stream, !ringAside && !ringPhys));
    } else if (dynamics_on(m, !ringAside && !ringPhys)) return -1;
    // (the late fork comes after CALC_DIV_GHAT, below)
    if (tcgFork) HIPCHK(hipStreamWaitEvent(m->stream, m->evSnap, 0));   // the copy before hFac is rewritten
    else if (fork && !lateJoin && !dtFused) HIPCHK(hipStreamWaitEvent(m->stream, m->evJoin, 0));
    // forward_step.F:829-877: UPDATE_R_STAR(.TRUE.) + UPDATE_CG2D
    // (launch fusions, common.h MGCM_STEP_FUSE: CALC_DIV_GHAT in the r* column pass;
    // EXCH(cg2d_x) + etaN in the single-workgroup CG2D's epilogue -- off by default: one CU
    // walking every 2-D point costs more than the launch it saves)
    const bool sfpFused = mg_fuse_on(MG_FUSE_SFP) && m->p.nonlinFreeSurf > 0 && m->d.nT == m->d.nTiles;
    if (m->p.nonlinFreeSurf > 0)
      TIMED(K_RSTAR, update_r_star_cg2d(m, sfpFused, opEarly, false));
    if (!sfpFused) TIMED(K_RHS, launch_sfp_rhs(m->d, m->p, m->f, m->stream));
    // the late fork: THERMODYNAMICS beside the CG2D only, CALC_DIV_GHAT (an HBM stream, on the
    // critical path) alone before it -- LLC-90 1.528-1.532 -> 1.474-1.476 ms/step, alternating
    // on one box (profiles/r05/thermo_at/); the tracers still finish inside the solve
    if (thermoLate && fork_thermo()) return -1;
    const bool etaFused = mg_fuse_on(MG_FUSE_ETA) && cg2d_fuses_eta(m);
    TIMED(K_CG2D, launch_cg2d(m, m->p.cg2dMaxIters, m->p.cg2dUseMinResSol - 1, etaFused));
    // Under exactConserv the etaN of EXCH_XY_RL(cg2d_x) + etaN = recip_Bo*cg2d_x
    // (solve_for_pressure.F:309-330) is read only by MOMENTUM_CORRECTION_STEP's gradient before
    // INTEGR_CONTINUITY's EXCH(eta) + UPDATE_ETAH replaces it; k_corr_cont derives that eta from
    // cg2d_x at the exchange sources itself, so k_exch_eta runs on a third stream beside it
    // (MG_FUSE_ETAA), joined before the etaN rewrite
    // Under exactConserv nothing else reads that etaN either: INTEGR_CONTINUITY's EXCH(eta) +
    // UPDATE_ETAH overwrites it everywhere but at points neither interior nor mapped, where it
    // keeps recip_Bo*cg2d_x -- so with MG_FUSE_ETAX k_exch_eta is not launched at all: k_corr_cont
    // reads eta from cg2d_x as above and the UPDATE_ETAH pass forms those points' etaN itself
    // (fromX; cg2d_x's halo is left unexchanged: the next SOLVE_FOR_PRESSURE rewrites cg2d_x
    // everywhere before anything reads it)
    const bool etaX = !etaFused && m->p.exactConserv && mg_fuse_on(MG_FUSE_ETAX) && m->d.nT == m->d.nTiles;
    const bool etaAside = !etaX && !etaFused && m->p.exactConserv && !m->timing && mg_fuse_on(MG_FUSE_ETAA) &&
                          m->d.nT == m->d.nTiles;
    if (etaX) {
    } else if (etaAside) {
      HIPCHK(hipEventRecord(m->evEta0, m->stream));
      HIPCHK(hipStreamWaitEvent(m->stream3, m->evEta0, 0));
      HIPCHK(launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, false, 0, m->stream3));
      HIPCHK(hipEventRecord(m->evEta1, m->stream3));
    } else if (!etaFused) {
      TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, false, 0, m->stream));
    }
    if (lateJoin || tcgFork) HIPCHK(hipStreamWaitEvent(m->stream, m->evJoin, 0));
    TIMED(K_CONT, launch_corr_cont(m->d, m->p, m->f, 0, m->stream, (etaAside || etaX) ? m->d_srcOf : nullptr));
    if (etaAside) HIPCHK(hipStreamWaitEvent(m->stream, m->evEta1, 0));
    // forward_step.F:965-977: CALC_R_STAR(etaH(n+1)); the next step's RESET_NLFS_VARS +
    // UPDATE_R_STAR(.FALSE.) restore the hFac in place, so they are not repeated here.
    // Under r* the exactConserv EXCH(eta) + UPDATE_ETAH runs inside CALC_R_STAR's pass
    // (k_calc_r_star<FUSE>)
    const bool fuseEtaH = m->p.exactConserv && m->p.nonlinFreeSurf > 0;
    if (m->p.exactConserv && !fuseEtaH)
      TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, true, 0, m->stream, etaX ? 1 : 0));
    // CALC_R_STAR and the blocking exchanges in one grid on the small lat-lon grids
    // (k_rstar_exch; independent, and nothing between them in the non-staggered step)
    endFused = m->p.nonlinFreeSurf > 0 && !stagger && !m->uvMap && m->d.nT == m->d.nTiles &&
               mg_hfuse(MG_FUSE_END, m->d.nx, m->d.ny, m->d.nT, m->d.Nr);
    if (endFused)
      TIMED(K_RSTAR, launch_rstar_exch(m->d, m->p, m->f, m->d_srcOf, fuseEtaH, blocking_fields(m), m->d_halo, m->nHalo,
                                       m->d_ctr, m->stream, etaX ? 1 : 0));
    else if (m->p.nonlinFreeSurf > 0) {
      stagEx = stagger && tracers && m->uvMap && m->d.nT == m->d.nTiles &&
               mg_hfuse(MG_FUSE_ENDS, m->d.nx, m->d.ny, m->d.nT, m->d.Nr);
      TIMED(K_RSTAR, calc_r_star(m, fuseEtaH, etaX ? 1 : 0, stagEx));
    }
  } else {
    if (mgcm_integr_continuity(m)) return -1;
  }
  if (stagger && tracers) {
    // DO_STAGGER_FIELDS_EXCHANGES (do_stagger_fields_exchanges.F:37-43) + THERMODYNAMICS
    if (stagEx) {     // (in CALC_R_STAR's grid, above)
    } else if (m->uvMap) {   // u, v through the vector map and w through the scalar map, one launch
      XFields xw{};
      xw.p[0] = m->f.wVel; xw.nz[0] = m->d.Nr; xw.n = 1;
      TIMED(K_EXCH, launch_exchange_mixed(m->d, m->f.uVel, m->f.vVel, m->d.Nr, m->d_uv[1], m->nUvU[1], m->nUvV[1], xw,
                                          m->d_halo, m->nHalo, nullptr, m->stream));
    } else {
      TIMED(K_EXCH, exchange_uv(m, m->f.uVel, m->f.vVel, m->d.Nr, true) ? hipErrorUnknown : hipSuccess);
      TIMED(K_EXCH, launch_exchange(m->d, m->f.wVel, m->d_halo, m->nHalo, m->d.Nr, m->stream));
    }
    if (tracers_on(m, m->stream)) return -1;
  }
  if (endFused) return 0;
  const XFields xEnd = blocking_fields(m, trEx ? 0 : 1);
  if (m->uvMap)   // the vector pair and the scalar fields in one launch
    TIMED(K_EXCH, launch_exchange_mixed(m->d, m->f.uVel, m->f.vVel, m->d.Nr, m->d_uv[1], m->nUvU[1], m->nUvV[1], xEnd,
                                        m->d_halo, m->nHalo, m->d_ctr, m->stream));
  else
    TIMED(K_EXCH, launch_exchange_multi(m->d, xEnd, m->d_halo, m->nHalo, m->d_ctr, m->stream));
  return 0;
}

static void drop_graphs(mgcm_model *m) {
  for (auto &row : m->graphExec)
    for (auto &ge : row)
      if (ge) { (void)hipGraphExecDestroy(ge); ge = nullptr; }
  for (auto &row : m->graph1Exec)
    for (auto &ge : row)
      if (ge) { (void)hipGraphExecDestroy(ge); ge = nullptr; }
}

// Which theta/salt ping-pong buffers are current (the kernels' arguments differ).
static int buffer_parity(const mgcm_model *m) {
  return (m->f.theta == m->thetaA ? 0 : 1) + (m->f.salt == m->saltA ? 0 : 2);
}

// Two FORWARD_STEPs captured once into a hipGraph per buffer parity (the tracer
// ping-pong swaps twice, so the pointers are back where they started), then
// replayed: no per-kernel host launch cost inside a batch.
static int two_step_graph(mgcm_model *m, hipGraphExec_t *out) {
  const int q = buffer_parity(m), o = m->overlap ? 1 : 0;
  if (!m->graphExec[o][q]) {
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamBeginCapture(m->stream, hipStreamCaptureModeThreadLocal));
    int rc = one_step(m);
    if (!rc) rc = one_step(m);
    hipError_t e = hipStreamEndCapture(m->stream, &g);
    if (rc) { if (g) (void)hipGraphDestroy(g); return -1; }
    HIPCHK(e);
    e = hipGraphInstantiate(&m->graphExec[o][q], g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIPCHK(e);
  }
  *out = m->graphExec[o][q];
  return 0;
}

// One FORWARD_STEP captured per buffer parity (the tracer ping-pong flips it, so consecutive
// single steps alternate between two of these graphs): a caller that steps one at a time --
// the Fortran drop-ins, with host work between steps -- still replays instead of launching.
static int one_step_graph(mgcm_model *m, hipGraphExec_t *out) {
  const int q = buffer_parity(m), o = m->overlap ? 1 : 0;
  if (!m->graph1Exec[o][q]) {
    double *pre[4] = {m->f.theta, m->f.thetaNext, m->f.salt, m->f.saltNext};
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamBeginCapture(m->stream, hipStreamCaptureModeThreadLocal));
    const int rc = one_step(m);
    hipError_t e = hipStreamEndCapture(m->stream, &g);
    if (rc) { if (g) (void)hipGraphDestroy(g); return -1; }
    HIPCHK(e);
    e = hipGraphInstantiate(&m->graph1Exec[o][q], g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIPCHK(e);
    // the capture ran one_step's host side (CYCLE_TRACER's pointer swaps) without launching:
    // keep the pointers it leaves for every replay, and undo them until the replay
    double **tr[4] = {&m->f.theta, &m->f.thetaNext, &m->f.salt, &m->f.saltNext};
    for (int k = 0; k < 4; k++) m->graph1Tr[o][q][k] = *tr[k];
    m->f.theta = pre[0]; m->f.thetaNext = pre[1]; m->f.salt = pre[2]; m->f.saltNext = pre[3];
  }
  *out = m->graph1Exec[o][q];
  return 0;
}
int mgcm_tracer_parity(mgcm_model *m, int set) {
  if (set < 0) return buffer_parity(m);
  if (set > 3) return set_err("mgcm_tracer_parity: parity %d outside 0..3", set);
  double *tB = m->f.theta == m->thetaA ? m->f.thetaNext : m->f.theta;
  double *sB = m->f.salt == m->saltA ? m->f.saltNext : m->f.salt;
  m->f.theta = (set & 1) ? tB : m->thetaA;
  m->f.thetaNext = (set & 1) ? m->thetaA : tB;
  m->f.salt = (set & 2) ? sB : m->saltA;
  m->f.saltNext = (set & 2) ? m->saltA : sB;
  return set;
}

// after a one-step replay: the tracer pointers one_step would have left
static void one_step_graph_done(mgcm_model *m, int o, int q) {
  m->f.theta = m->graph1Tr[o][q][0]; m->f.thetaNext = m->graph1Tr[o][q][1];
  m->f.salt = m->graph1Tr[o][q][2]; m->f.saltNext = m->graph1Tr[o][q][3];
}

static int ovl_trial(mgcm_model *m);

// Builds the graphs of the next batch and, when the THERMODYNAMICS overlap is still
// undecided, runs its trial now (on a copy of the state) so that no later timed batch
// contains the trial's 20 steps.
int mgcm_prepare(mgcm_model *m) {
  if (check_ready(m)) return -1;
  if (!m->useGraph) return 0;
  HIPCHK(hipSetDevice(m->device));
  if (m->ovlAuto && !m->ovlDecided && ovl_trial(m)) return -1;
  hipGraphExec_t ge;
  return two_step_graph(m, &ge);
}

// THERMODYNAMICS overlap auto-selection: the device state (both field arenas, the other
// fields, counters, solve records) is copied aside, 20 steps run through the two graphs --
// on, off (one two-step graph each: builds and warms them), then on, off, on, off of two
// graphs each, bracketed by events -- and the state is copied back, so the caller's steps
// are untouched; the faster graph is kept.  Both graphs compute identical results.
static int ovl_trial(mgcm_model *m) {
  const bool forkable = !m->p.staggerTimeStep && m->p.momStepping && (m->p.tempStepping || m->p.saltStepping);
  if (!forkable) { m->ovlDecided = true; return 0; }   // one_step never forks: nothing to choose
  std::vector<std::pair<void *, size_t>> parts = {
      {m->f.a2, (size_t)F2_COUNT * m->d.N2all * sizeof(double)},
      {m->f.a3, (size_t)F3_COUNT * m->d.N3all * sizeof(double)},
      {m->d_ctr, 2 * sizeof(int)},
      {m->d_rec, (size_t)m->maxRec * sizeof(SolveRecord)}};
  for (auto &fd : FIELDS)
    if (fd.kind != F2D && fd.kind != F3D && field_ptr(m, &fd))
      parts.push_back({field_ptr(m, &fd), (size_t)field_count(m, fd.kind) * sizeof(double)});
  size_t total = 0;
  for (auto &pr : parts) total += (pr.second + 255) & ~(size_t)255;
  char *save = nullptr;
  if (hipMalloc(&save, total) != hipSuccess) {   // no room for the copy: keep the overlap on, untimed
    (void)hipGetLastError();
    m->ovlDecided = true;
    return 0;
  }
  // one exit path: the copy is always restored and freed, the overlap mode always reset
  // when the trial fails
  const bool ovl0 = m->overlap;
  int rc = 0;
  size_t off = 0;
  for (auto &pr : parts) {
    if (!rc && hipMemcpyAsync(save + off, pr.first, pr.second, hipMemcpyDeviceToDevice, m->stream) != hipSuccess) rc = -1;
    off += (pr.second + 255) & ~(size_t)255;
  }
  for (int ph = 0; ph < 6 && !rc; ph++) {
    const int pairs = ph < 2 ? 1 : 2, mode = (ph & 1) ? 0 : 1;
    m->overlap = mode != 0;
    hipGraphExec_t ge;
    if (two_step_graph(m, &ge)) { rc = -1; break; }   // built before the events (same parity after a pair)
    if (hipEventRecord(m->ovlEv[0], m->stream) != hipSuccess) { rc = -1; break; }
    for (int r = 0; r < pairs && !rc; r++)
      if (two_step_graph(m, &ge) || hipGraphLaunch(ge, m->stream) != hipSuccess) rc = -1;
    float ms = 0.f;
    if (rc || hipEventRecord(m->ovlEv[1], m->stream) != hipSuccess || hipEventSynchronize(m->ovlEv[1]) != hipSuccess ||
        hipEventElapsedTime(&ms, m->ovlEv[0], m->ovlEv[1]) != hipSuccess) { rc = -1; break; }
    if (ph >= 2) m->ovlMs[mode] += ms;
  }
  int rs = 0;
  off = 0;
  for (auto &pr : parts) {
    if (hipMemcpyAsync(pr.first, save + off, pr.second, hipMemcpyDeviceToDevice, m->stream) != hipSuccess) rs = -1;
    off += (pr.second + 255) & ~(size_t)255;
  }
  if (hipStreamSynchronize(m->stream) != hipSuccess) rs = -1;
  (void)hipFree(save);
  if (rc || rs) {
    m->overlap = ovl0;
    return set_err(rs ? "ovl_trial: restoring the saved state failed" : "ovl_trial: graph replay failed");
  }
  m->ovlDecided = true;
  m->overlap = m->ovlMs[1] <= m->ovlMs[0];
  return 0;
}

int mgcm_forward_step(mgcm_model *m, int nsteps) {
  if (check_ready(m)) return -1;
  if (nsteps <= 0 || nsteps > m->maxRec) return set_err("mgcm_forward_step: nsteps %d out of range", nsteps);
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(hipMemsetAsync(m->d_ctr + 1, 0, sizeof(int), m->stream));
  int s = 0;
  if (m->useGraph && !m->timing) {
    if (m->ovlAuto && !m->ovlDecided && nsteps >= 2 && ovl_trial(m)) return -1;
    for (; s + 2 <= nsteps; s += 2) {
      hipGraphExec_t ge;
      if (two_step_graph(m, &ge)) return -1;
      HIPCHK(hipGraphLaunch(ge, m->stream));
    }
  }
  // an odd step (a caller stepping one at a time): the one-step graph of this parity
  if (s < nsteps && m->useGraph && !m->timing) {
    const int q = buffer_parity(m), o = m->overlap ? 1 : 0;
    hipGraphExec_t ge;
    if (one_step_graph(m, &ge)) return -1;
    HIPCHK(hipGraphLaunch(ge, m->stream));
    one_step_graph_done(m, o, q);
    s++;
  }
  for (; s < nsteps; s++)
    if (one_step(m)) return -1;
  m->lastBatch = nsteps;
  return 0;
}

// ---- tile-sharded runs (mitgcm_amd/parallel.py drives the collectives) ----------
int mgcm_set_tile_range(mgcm_model *m, int t0, int nT) {
  if (t0 < 0 || nT < 1 || t0 + nT > m->d.nTiles)
    return set_err("mgcm_set_tile_range: tiles [%d, %d) outside [0, %d)", t0, t0 + nT, m->d.nTiles);
  m->d.t0 = t0;
  m->d.nT = nT;
  drop_graphs(m);
  if (m->ready) {
    HIPCHK(hipSetDevice(m->device));
    HIPCHK(hipStreamSynchronize(m->stream));
    if (upload_halo(m)) return -1;
  }
  return 0;
}

int mgcm_set_stream(mgcm_model *m, void *stream) {
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(hipStreamSynchronize(m->stream));
  drop_graphs(m);
  m->stream = stream ? (hipStream_t)stream : m->ownStream;
  return 0;
}

// The 3-D fields whose halo sources travel between processes: the blocking-exchange set
// with u and v always included (on an EXCH2 topology the vector map may read either
// component of a source point, exch2_uv_3d_rx.template).
// group 0: all of them; 1: the tracers (final once THERMODYNAMICS has run, so their
// exchange can travel while DYNAMICS and the solve compute); 2: the rest.
static XFields transfer_fields(const mgcm_model *m, int group = 0) {
  XFields x{};
  double *fl[] = {m->f.uVel, m->f.vVel, m->f.wVel, m->f.theta, m->f.salt, m->f.uVelD, m->f.vVelD, m->f.totPhiHyd};
  const bool use[] = {true, true, true, m->p.tempStepping != 0, m->p.saltStepping != 0, m->p.useCDscheme != 0,
                      m->p.useCDscheme != 0, m->p.storePhiHyd4Phys != 0};
  const bool tracer[] = {false, false, false, true, true, false, false, false};
  for (int q = 0; q < 8; q++)
    if (use[q] && (group == 0 || (group == 1) == tracer[q])) { x.p[x.n] = fl[q]; x.nz[x.n] = m->d.Nr; x.n++; }
  return x;
}

int mgcm_exchange_nfields(mgcm_model *m) { return transfer_fields(m).n; }
int mgcm_exchange_nfields_group(mgcm_model *m, int group) {
  if (group < 0 || group > 2) return -1;
  return transfer_fields(m, group).n;
}

int mgcm_halo_pack(mgcm_model *m, const long *idx, long n, double *buf, int unpack) {
  return mgcm_halo_pack_group(m, 0, idx, n, buf, unpack);
}

int mgcm_halo_pack_group(mgcm_model *m, int group, const long *idx, long n, double *buf, int unpack) {
  if (check_ready(m)) return -1;
  if (group < 0 || group > 2) return set_err("mgcm_halo_pack_group: no group %d", group);
  HIPCHK(launch_halo_pack(m->d, transfer_fields(m, group), idx, n, buf, unpack, m->stream));
  return 0;
}

// Cross-stream ordering for callers whose collectives run on another stream: direction 0
// makes `other` wait for the work issued on the model's stream so far (the model's outputs,
// e.g. a packed halo buffer or tile partials, are then safe to read there); 1 makes the
// model's stream wait for the work issued on `other` so far (e.g. a received buffer).
int mgcm_stream_handoff(mgcm_model *m, void *other, int direction) {
  hipStream_t o = (hipStream_t)other;
  if (o == m->stream) return 0;
  HIPCHK(hipSetDevice(m->device));
  if (direction == 0) {
    HIPCHK(hipEventRecord(m->evHand, m->stream));
    HIPCHK(hipStreamWaitEvent(o, m->evHand, 0));
  } else {
    HIPCHK(hipEventRecord(m->evHand, o));
    HIPCHK(hipStreamWaitEvent(m->stream, m->evHand, 0));
  }
  return 0;
}

int mgcm_tile_copy(mgcm_model *m, const char *name, int t0, int nT, void *buf, int toField) {
  const FieldDesc *fd = find_field(name);
  if (!fd || fd->kind == F1D) return set_err("mgcm_tile_copy: no 2-D/3-D field '%s'", name);
  if (t0 < 0 || nT < 0 || t0 + nT > m->d.nTiles) return set_err("mgcm_tile_copy: bad tile range");
  const long per = fd->kind == F2D ? m->d.n2 : m->d.n3;
  double *f = field_ptr(m, fd) + t0 * per;
  const size_t bytes = (size_t)nT * per * sizeof(double);
  HIPCHK(hipMemcpyAsync(toField ? f : buf, toField ? buf : f, bytes, hipMemcpyDeviceToDevice, m->stream));
  return 0;
}

static int mwg_block_uncached(mgcm_model *m);

// Everyone sharing a hand-off block must tag with the same launch epoch: the epoch words
// (each process's / model's own, T.epoch) restart at 0 wherever a block is shared, and the
// block itself is zeroed by its owner then, so granules an earlier solve of one sharer left
// (tagged with that sharer's epochs) match no tag of the shared solves.  A hand-off that
// times out in a shared solve is fatal for the run (the epochs may then diverge: each sharer's
// first part reads the shared timeout word at its own time): ShardedModel.check_solves raises,
// the Fortran drop-ins die (fortran_abi.hip); re-sharing restarts both words.
static int mwg_restart_epoch(mgcm_model *m, bool zeroBlock) {
  if (zeroBlock) HIPCHK(hipMemset(m->mwg.ctr, 0, m->mwg.hsBytes));
  HIPCHK(hipMemset(m->mwg.epoch, 0, 64));
  HIPCHK(hipDeviceSynchronize());
  return 0;
}

// The tile-sharded device CG2D: every process launches the multi-workgroup solver's parts
// of its own tiles, all on ONE hand-off block (granules, epoch, timeout word), which the
// first process exports by IPC and the others map; every granule access is then at system
// scope.  The sums keep the single-launch order, so the solve is the 1-process solve.
int mgcm_cg2d_shared_export(mgcm_model *m, void *handle) {
  if (!m->useMwg || m->mwg.partsPerTile <= 0)
    return set_err("mgcm_cg2d_shared_export: needs the multi-workgroup CG2D on whole-domain tables (cg2dForceMwg)");
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(hipStreamSynchronize(m->stream));
  // the importers' launches may run on other GPUs: an uncached block (mwg_block_uncached)
  if (mwg_block_uncached(m) || mwg_restart_epoch(m, true)) return -1;
  hipIpcMemHandle_t h;
  HIPCHK(hipIpcGetMemHandle(&h, (void *)m->mwg.ctr));
  memcpy(handle, &h, sizeof h);
  return 0;
}

int mgcm_cg2d_shared_import(mgcm_model *m, const void *handle) {
  if (!m->useMwg || m->mwg.partsPerTile <= 0)
    return set_err("mgcm_cg2d_shared_import: needs the multi-workgroup CG2D on whole-domain tables (cg2dForceMwg)");
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(hipStreamSynchronize(m->stream));
  if (m->mwgShared) { (void)hipIpcCloseMemHandle(m->mwgShared); m->mwgShared = nullptr; }
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof h);
  void *p = nullptr;
  HIPCHK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  m->mwgShared = p;
  const size_t partGr = (size_t)2 * 3 * m->mwg.G * 2;
  m->mwg.ctr = (unsigned *)p;
  m->mwg.part = (unsigned long long *)((char *)p + 64);
  m->mwg.xs = m->mwg.part + partGr;
  m->mwg.sys = 1;
  if (mwg_restart_epoch(m, false)) return -1;
  drop_graphs(m);
  return 0;
}

int mgcm_cg2d_shared_bytes(mgcm_model *m) { return m->useMwg ? (int)sizeof(hipIpcMemHandle_t) : -1; }

// After a caller replays its own captured steps (ShardedModel.replay): the number of steps
// the batch recorded, so mgcm_solve_stats finds them.
int mgcm_end_steps(mgcm_model *m, int nsteps) {
  if (nsteps < 0 || nsteps > m->maxRec) return set_err("mgcm_end_steps: nsteps %d out of range", nsteps);
  m->lastBatch = nsteps;
  return 0;
}

int mgcm_begin_steps(mgcm_model *m) {
  if (check_ready(m)) return -1;
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(hipMemsetAsync(m->d_ctr + 1, 0, sizeof(int), m->stream));
  m->lastBatch = 0;
  return 0;
}

// FORWARD_STEP split at its exchange points (tile-sharded runs, mitgcm_amd/parallel.py
// drives the collectives in between):
//   1: DO_OCEANIC_PHYS, THERMODYNAMICS (staggerTimeStep = F), DYNAMICS, UPDATE_R_STAR +
//      UPDATE_CG2D (r*, every tile), the SOLVE_FOR_PRESSURE right-hand side;
//      [all-gather cg2d_b, cg2d_x]
//   2: CG2D on the whole domain (replicated), EXCH + etaN everywhere, correction +
//      continuity on this process's tiles;  [all-gather the new eta (exactConserv)]
//   3: EXCH eta + UPDATE_ETAH everywhere, CALC_R_STAR (r*, every tile);
//      [send/recv the 3-D halo sources]
//   5: staggerTimeStep only: DO_STAGGER_FIELDS_EXCHANGES on this process's tiles, then
//      THERMODYNAMICS with the new velocities;  [send/recv the 3-D halo sources again]
//   4: DO_FIELDS_BLOCKING_EXCHANGES of this process's tiles, step counters.
// THERMODYNAMICS onto the second stream (after the model stream's work so far) and its join
static int shard_fork_thermo(mgcm_model *m, bool ring = false) {
  HIPCHK(hipEventRecord(m->evFork, m->stream));
  HIPCHK(hipStreamWaitEvent(m->stream2, m->evFork, 0));
  if (ring) HIPCHK(launch_mom_ring(m->d, m->p, m->f, m->d_ctr, m->stream2));   // as one_step (MG_FUSE_RING)
  if (tracers_on(m, m->stream2)) return -1;
  HIPCHK(hipEventRecord(m->evJoin, m->stream2));
  return 0;
}
static int shard_join_thermo(mgcm_model *m) {
  if (m->shardFork == 1 || m->shardFork == 3) HIPCHK(hipStreamWaitEvent(m->stream, m->evJoin, 0));
  m->shardFork = 0;
  m->mwg.exclusive = 0;
  return 0;
}

int mgcm_step_phase(mgcm_model *m, int phase) {
  if (check_ready(m)) return -1;
  if (!m->p.momStepping) return set_err("mgcm_step_phase: requires momStepping");
  const bool stagger = m->p.staggerTimeStep != 0;
  const bool tracers = m->p.tempStepping || m->p.saltStepping;
  switch (phase) {
    case 16:  // DO_OCEANIC_PHYS, THERMODYNAMICS on the second stream as the resident step forks it
              // (one_step): beside DYNAMICS under r* (joined before UPDATE_R_STAR, which rewrites
              // hFac), beside the pressure solve under the linear free surface (forked after
              // DYNAMICS, joined before MOMENTUM_CORRECTION_STEP rewrites u, v, w)
      if (stagger || !tracers || m->timing) {   // nothing to fork (the timed pass: one stream)
        phase = 8;
      } else {
        if (m->shardFork) return set_err("mgcm_step_phase(16): the previous step's THERMODYNAMICS not joined");
        TIMED(K_PHYS, launch_oceanic_phys(m->d, m->p, m->f, m->d_ctr, m->stream));
        if (m->p.nonlinFreeSurf > 0) {
          if (shard_fork_thermo(m)) return -1;
          m->shardFork = 1;
        } else {
          m->shardFork = 2;
        }
        return 0;
      }
      [[fallthrough]];
    case 1:   // = 8 then 9
    case 8:   // DO_OCEANIC_PHYS + THERMODYNAMICS (non-staggered): the tracers are final
      TIMED(K_PHYS, launch_oceanic_phys(m->d, m->p, m->f, m->d_ctr, m->stream));
      if (!stagger && tracers_on(m, m->stream)) return -1;
      if (phase == 8) return 0;
      [[fallthrough]];
    case 9: {   // DYNAMICS, UPDATE_R_STAR + UPDATE_CG2D, CALC_DIV_GHAT
      const bool ringAside = m->shardFork == 2 && mom_ring_separable(m->d, m->p) && mg_fuse_on(MG_FUSE_RING);
      if (dynamics_on(m, !ringAside)) return -1;
      if (m->shardFork == 1 && shard_join_thermo(m)) return -1;
      if (m->p.nonlinFreeSurf > 0) TIMED(K_RSTAR, update_r_star_cg2d(m));
      TIMED(K_RHS, launch_sfp_rhs(m->d, m->p, m->f, m->stream));
      if (m->shardFork == 2) {   // after CALC_DIV_GHAT, as one_step forks it
        if (shard_fork_thermo(m, ringAside)) return -1;
        m->shardFork = 3;
        m->mwg.exclusive = 1;   // the multi-workgroup CG2D keeps its CUs while the tracers run
      }
      return 0;
    }
    case 2:
      TIMED(K_CG2D, launch_cg2d(m, m->p.cg2dMaxIters, m->p.cg2dUseMinResSol - 1));
      TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, false, 0, m->stream));
      if (shard_join_thermo(m)) return -1;
      TIMED(K_CONT, launch_corr_cont(m->d, m->p, m->f, 0, m->stream));
      return 0;
    case 10:  // the device CG2D over this process's parts (hand-off block shared by IPC)
      if (!m->useMwg || m->mwg.partsPerTile <= 0)
        return set_err("mgcm_step_phase(10): needs the multi-workgroup CG2D on whole-domain tables (cg2dForceMwg)");
      if (m->d.nT < m->d.nTiles && !m->mwg.sys)
        return set_err("mgcm_step_phase(10): a tile subset needs the shared hand-off block (mgcm_cg2d_shared_*)");
      TIMED(K_CG2D, launch_cg2d_mwg(m->d, m->p, m->f, m->mwg, m->p.cg2dMaxIters, m->p.cg2dUseMinResSol - 1, m->d_rec, m->d_ctr + 1, m->stream,
                                    m->d.t0 * m->mwg.partsPerTile, m->d.nT * m->mwg.partsPerTile));
      return 0;
    case 6:   // phase 2 after a CG2D driven by the caller (mgcm_cg2d_op: distributed CG2D)
      TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, false, 0, m->stream));
      if (shard_join_thermo(m)) return -1;
      TIMED(K_CONT, launch_corr_cont(m->d, m->p, m->f, 0, m->stream));
      return 0;
    // phase 2 / 6 split at the THERMODYNAMICS join, so the caller can send the new tracers'
    // halo sources while the correction step runs: 19 the replicated CG2D alone, 17 EXCH(x) +
    // etaN and the join, 18 the correction + continuity pass
    case 19:
      TIMED(K_CG2D, launch_cg2d(m, m->p.cg2dMaxIters, m->p.cg2dUseMinResSol - 1));
      return 0;
    case 17:
      TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, false, 0, m->stream));
      return shard_join_thermo(m);
    case 18:
      TIMED(K_CONT, launch_corr_cont(m->d, m->p, m->f, 0, m->stream));
      return 0;
    case 3:
      if (shard_join_thermo(m)) return -1;
      if (m->p.exactConserv) TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, true, 0, m->stream));
      if (m->p.nonlinFreeSurf > 0) TIMED(K_RSTAR, calc_r_star(m));
      return 0;
    case 5:
      if (!stagger) return 0;
      TIMED(K_EXCH, exchange_uv(m, m->f.uVel, m->f.vVel, m->d.Nr, true) ? hipErrorUnknown : hipSuccess);
      TIMED(K_EXCH, launch_exchange(m->d, m->f.wVel, m->d_halo, m->nHalo, m->d.Nr, m->stream));
      return tracers_on(m, m->stream);
    case 4:
      if (m->uvMap) TIMED(K_EXCH, exchange_uv(m, m->f.uVel, m->f.vVel, m->d.Nr, true) ? hipErrorUnknown : hipSuccess);
      TIMED(K_EXCH, launch_exchange_multi(m->d, blocking_fields(m), m->d_halo, m->nHalo, m->d_ctr, m->stream));
      m->lastBatch++;
      return 0;
    // the routine-level split of a sharded step (one Fortran host stepping several models,
    // fortran_abi.hip: the reference's routine boundaries with the cross-model copies between)
    case 11:  // SOLVE_FOR_PRESSURE's right-hand side (CALC_DIV_GHAT) on this model's tiles
      TIMED(K_RHS, launch_sfp_rhs(m->d, m->p, m->f, m->stream));
      return 0;
    case 12:  // CG2D on the whole (gathered) domain + EXCH_XY_RL(cg2d_x) + etaN everywhere
      TIMED(K_CG2D, launch_cg2d(m, m->p.cg2dMaxIters, m->p.cg2dUseMinResSol - 1));
      [[fallthrough]];
    case 13:  // EXCH_XY_RL(cg2d_x) + etaN everywhere, after a CG2D done by phase 10 / mgcm_cg2d_tiles
      TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, false, 0, m->stream));
      return 0;
    case 14:  // INTEGR_CONTINUITY's column pass (after MOMENTUM_CORRECTION_STEP) on this model's tiles
      TIMED(K_CONT, launch_corr_cont(m->d, m->p, m->f, 2, m->stream));
      return 0;
    case 15:  // INTEGR_CONTINUITY's EXCH(eta) + UPDATE_ETAH everywhere (exactConserv; gathered eta)
      if (m->p.exactConserv) TIMED(K_ETA, launch_exch_eta(m->d, m->p, m->f, m->d_srcOf, true, 0, m->stream));
      return 0;
  }
  return set_err("mgcm_step_phase: no phase %d", phase);
}

// ---- the box's HBM reference rate (bench.py: SURVEY.md 8(d)'s roofline denominator) ---------
namespace mgcm {
__global__ void __launch_bounds__(256) k_triad(double2 *__restrict__ a, const double2 *__restrict__ b,
                                               const double2 *__restrict__ c, double s, long n2) {
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < n2; q += (long)gridDim.x * 256) {
    const double2 x = b[q], y = c[q];
    a[q] = make_double2(x.x + s * y.x, x.y + s * y.y);
  }
}
}  // namespace mgcm
// STREAM triad a = b + s*c over three fp64 arrays of n doubles on `device`, 16 B per lane,
// best of `reps` (event-timed): GB/s at 24 bytes per element.
int mgcm_stream_triad(int device, long n, int reps, double *gbs) {
  if (n <= 0 || (n & 1) || reps <= 0 || !gbs) return set_err("mgcm_stream_triad: bad arguments");
  HIPCHK(hipSetDevice(device));
  double *a = nullptr, *b = nullptr, *c = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = 0;
  float best = 1e30f;
  if (hipMalloc(&a, n * sizeof(double)) != hipSuccess || hipMalloc(&b, n * sizeof(double)) != hipSuccess ||
      hipMalloc(&c, n * sizeof(double)) != hipSuccess || hipStreamCreate(&st) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess ||
      hipMemsetAsync(b, 0, n * sizeof(double), st) != hipSuccess || hipMemsetAsync(c, 0, n * sizeof(double), st) != hipSuccess)
    rc = set_err("mgcm_stream_triad: allocation");
  const unsigned grid = 256 * 16;   // 16 workgroups per CU, grid-stride
  for (int r = -1; rc == 0 && r < reps; r++) {   // r = -1: warm-up
    hipEventRecord(e0, st);
    hipLaunchKernelGGL(mgcm::k_triad, dim3(grid), dim3(256), 0, st, (double2 *)a, (const double2 *)b, (const double2 *)c, 3.0,
                       n / 2);
    hipEventRecord(e1, st);
    if (hipEventSynchronize(e1) != hipSuccess) { rc = set_err("mgcm_stream_triad: kernel"); break; }
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (r >= 0 && ms < best) best = ms;
  }
  if (rc == 0) *gbs = 24.0 * (double)n / (best * 1e-3) / 1e9;
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  if (st) hipStreamDestroy(st);
  if (a) hipFree(a);
  if (b) hipFree(b);
  if (c) hipFree(c);
  return rc;
}

// ---- several models stepped by one host (fortran_abi.hip's tile-sharded drop-ins) ---------
void *mgcm_get_stream(mgcm_model *m) { return (void *)m->stream; }

// The interior points whose values the halos of tiles [t0, t0+nT) copy (the scalar EXCH map
// and, on EXCH2 topologies, both vector maps), outside those tiles: what another model that
// steps them must deliver before this one's local halo fill (the in-process HaloPlan).
long mgcm_halo_sources(mgcm_model *m, int t0, int nT, long *out, long cap) {
  if (t0 < 0 || nT < 1 || t0 + nT > m->d.nTiles) return set_err("mgcm_halo_sources: bad tile range");
  const long n2 = m->d.n2, N2 = n2 * m->d.nTiles, lo = (long)t0 * n2, hi = (long)(t0 + nT) * n2;
  std::vector<long> src;
  for (size_t h = 0; h + 1 < m->h_halo.size(); h += 2)
    if (m->h_halo[h] >= lo && m->h_halo[h] < hi) src.push_back(m->h_halo[h + 1]);
  if (m->uvMap)
    for (int w = 0; w < 2; w++)
      for (int c = 0; c < 2; c++)
        for (long q = lo; q < hi; q++) {
          const long code = m->h_uv[w][(size_t)c * N2 + q];
          if (code != 0) src.push_back(((code < 0 ? -code : code) - 1) % N2);
        }
  std::sort(src.begin(), src.end());
  src.erase(std::unique(src.begin(), src.end()), src.end());
  long n = 0;
  for (long v : src)
    if (v < lo || v >= hi) {
      if (out && n < cap) out[n] = v;
      n++;
    }
  return n;
}

// The device CG2D's parts of tiles [t0, t0+nT) on this model's stream and arrays (its
// cg2d_b, cg2d_x and operator must hold those tiles' values): a host stepping several models
// on one GPU launches one model's arrays for all of them (the gathered right-hand side), on
// several GPUs one launch per GPU on one shared hand-off block (mgcm_cg2d_share).
int mgcm_cg2d_tiles(mgcm_model *m, int t0, int nT) {
  if (check_ready(m)) return -1;
  if (!m->useMwg || m->mwg.partsPerTile <= 0)
    return set_err("mgcm_cg2d_tiles: needs the multi-workgroup CG2D on whole-domain tables (cg2dForceMwg)");
  if (t0 < 0 || nT < 1 || t0 + nT > m->d.nTiles) return set_err("mgcm_cg2d_tiles: bad tile range");
  if (nT < m->d.nTiles && !m->mwg.sys)
    return set_err("mgcm_cg2d_tiles: a tile subset needs the shared hand-off block (mgcm_cg2d_share)");
  HIPCHK(hipSetDevice(m->device));
  TIMED(K_CG2D, launch_cg2d_mwg(m->d, m->p, m->f, m->mwg, m->p.cg2dMaxIters, m->p.cg2dUseMinResSol - 1, m->d_rec, m->d_ctr + 1, m->stream,
                                t0 * m->mwg.partsPerTile, nT * m->mwg.partsPerTile));
  return 0;
}

// The hand-off block re-allocated as uncached (mem 1) or fine-grained (mem 2) device memory,
// its granules accessed at system scope (sys) or agent scope.
static int mwg_block_realloc(mgcm_model *m, int mem, bool sys) {
  const size_t partGr = (size_t)2 * 3 * m->mwg.G * 2;
  char *blk = nullptr;
  if (mem != 2 && hipExtMallocWithFlags((void **)&blk, m->mwg.hsBytes, hipDeviceMallocUncached) != hipSuccess) blk = nullptr;
  if (!blk) HIPCHK(hipExtMallocWithFlags((void **)&blk, m->mwg.hsBytes, hipDeviceMallocFinegrained));
  HIPCHK(hipMemset(blk, 0, m->mwg.hsBytes));
  HIPCHK(hipDeviceSynchronize());
  for (auto &q : m->mwgAllocs)
    if (q == m->mwgBlock) { (void)hipFree(q); q = blk; }
  m->mwgBlock = blk;
  m->mwg.ctr = (unsigned *)blk;
  m->mwg.part = (unsigned long long *)(blk + 64);
  m->mwg.xs = m->mwg.part + partGr;
  m->mwg.sys = sys ? 1 : 0;
  drop_graphs(m);
  return 0;
}

// A hand-off block that other launches poll from another GPU: uncached device memory, so no
// GPU's L2 holds a stale copy of a granule (coarse-grained hipMalloc memory is coherent only at
// kernel boundaries); every granule access is then at system scope (T.sys).
static int mwg_block_uncached(mgcm_model *m) {
  if (m->mwg.sys) return 0;
  return mwg_block_realloc(m, 1, true);
}

// In-process sharing of `owner`'s hand-off block by m (another model of the same host, on
// another GPU): the block becomes uncached device memory of the owner's GPU, m's launches map
// it by peer access, and both poll at system scope.  m == owner prepares the owner only.
int mgcm_cg2d_share(mgcm_model *m, mgcm_model *owner) {
  if (!m->useMwg || !owner->useMwg || m->mwg.partsPerTile <= 0 || m->mwg.G != owner->mwg.G)
    return set_err("mgcm_cg2d_share: both models need the same whole-domain multi-workgroup CG2D (cg2dForceMwg)");
  HIPCHK(hipSetDevice(owner->device));
  HIPCHK(hipStreamSynchronize(owner->stream));
  if (mwg_block_uncached(owner)) return -1;
  if (m == owner) return mwg_restart_epoch(owner, true);
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(hipStreamSynchronize(m->stream));
  if (m->device != owner->device) {
    hipError_t e = hipDeviceEnablePeerAccess(owner->device, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return set_err("mgcm_cg2d_share: peer access %d -> %d: %s",
                                                                                  m->device, owner->device, hipGetErrorString(e));
    (void)hipGetLastError();
  }
  m->mwg.ctr = owner->mwg.ctr;
  m->mwg.part = owner->mwg.part;
  m->mwg.xs = owner->mwg.xs;
  m->mwg.sys = 1;
  if (mwg_restart_epoch(m, false)) return -1;
  drop_graphs(m);
  return 0;
}

// Distributed CG2D building blocks (kernels_cg2d_dist.hip): one op of cg2d.F over this
// process's tiles, per-tile partial sums into the device buffer part[2*nTiles].
int mgcm_cg2d_op(mgcm_model *m, int op, double a0, double *part) {
  if (check_ready(m)) return -1;
  if (op < 0 || op > 15) return set_err("mgcm_cg2d_op: no op %d", op);
  const bool sums = op == 0 || op == 2 || op == 3 || op == 5 || op == 6 || op == 10 || op == 13 || op == 14;
  if (!part && sums) return set_err("mgcm_cg2d_op: op %d needs the partials buffer", op);
  HIPCHK(launch_cgd(m->d, m->p, m->f, op, a0, part, m->stream));
  return 0;
}

int mgcm_cg2d_record(mgcm_model *m, double firstResidual, double lastResidual, double rhsMax, double sumRHS,
                     int numIters, double minResidualSq, int nIterMin) {
  if (check_ready(m)) return -1;
  HIPCHK(launch_cgd_record(m->d_rec, m->d_ctr + 1, firstResidual, lastResidual, rhsMax, sumRHS, numIters, minResidualSq,
                           nIterMin, m->stream));
  return 0;
}

int mgcm_field_pack(mgcm_model *m, const char *name, const long *idx, long n, double *buf, int unpack) {
  const FieldDesc *fd = find_field(name);
  if (!fd || fd->kind != F2D) return set_err("mgcm_field_pack: no 2-D field '%s'", name);
  HIPCHK(launch_field_pack(field_ptr(m, fd), idx, n, buf, unpack, m->stream));
  return 0;
}

int mgcm_exchange_field(mgcm_model *m, const char *name) {
  const FieldDesc *fd = find_field(name);
  if (!fd || fd->kind == F1D) return set_err("mgcm_exchange_field: no 2-D/3-D field '%s'", name);
  HIPCHK(launch_exchange(m->d, field_ptr(m, fd), m->d_halo, m->nHalo, fd->kind == F2D ? 1 : m->d.Nr, m->stream));
  return 0;
}

int mgcm_sync(mgcm_model *m) {
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(hipStreamSynchronize(m->stream));
  ev_collect(m);
  return 0;
}

int mgcm_solve_stats(mgcm_model *m, int back, double *firstResidual, double *lastResidual, int *numIters,
                     double *rhsMax) {
  HIPCHK(hipStreamSynchronize(m->stream));
  int slot = m->lastBatch - 1 - back;
  if (m->lastBatch == 0) slot = 0;
  if (slot < 0) return set_err("mgcm_solve_stats: no such step");
  SolveRecord r;
  HIPCHK(hipMemcpy(&r, m->d_rec + slot, sizeof r, hipMemcpyDeviceToHost));
  if (firstResidual) *firstResidual = r.firstResidual;
  if (lastResidual) *lastResidual = r.lastResidual;
  if (numIters) *numIters = r.numIters;
  if (rhsMax) *rhsMax = r.rhsMax;
  return 0;
}

// The min-residual bookkeeping of a step's solve (cg2dUseMinResSol): the lowest squared
// residual reached and its iteration (cg2d.F minResidualSq, nIterMin; -1 / -1 when off).
int mgcm_solve_minres(mgcm_model *m, int back, double *minResidualSq, int *nIterMin) {
  HIPCHK(hipStreamSynchronize(m->stream));
  int slot = m->lastBatch - 1 - back;
  if (m->lastBatch == 0) slot = 0;
  if (slot < 0) return set_err("mgcm_solve_minres: no such step");
  SolveRecord r;
  HIPCHK(hipMemcpy(&r, m->d_rec + slot, sizeof r, hipMemcpyDeviceToHost));
  if (minResidualSq) *minResidualSq = r.minResidualSq;
  if (nIterMin) *nIterMin = r.nIterMin;
  return 0;
}

// The last n steps' solve records in one copy (oldest first): what a caller checks after a
// batch without a device-to-host transfer per step.
int mgcm_solve_history(mgcm_model *m, int n, int *numIters, double *firstResidual, double *lastResidual) {
  HIPCHK(hipStreamSynchronize(m->stream));
  if (n < 0 || n > m->lastBatch) return set_err("mgcm_solve_history: %d steps asked, %d in the last batch", n, m->lastBatch);
  if (n == 0) return 0;
  std::vector<SolveRecord> r((size_t)n);
  HIPCHK(hipMemcpy(r.data(), m->d_rec + (m->lastBatch - n), (size_t)n * sizeof(SolveRecord), hipMemcpyDeviceToHost));
  for (int q = 0; q < n; q++) {
    if (numIters) numIters[q] = r[q].numIters;
    if (firstResidual) firstResidual[q] = r[q].firstResidual;
    if (lastResidual) lastResidual[q] = r[q].lastResidual;
  }
  return 0;
}

// MONITOR's dynstat block (pkg/monitor/monitor.F:103-129, MON_CALC_STATS_RL) on the device:
// plane partials by k_mon_stats, added here in (tile, level) order; out[6][5] = (max, min,
// mean, sd, del2) of eta, uvel, vvel, wvel, theta, salt over this process's tiles.
int mgcm_monitor(mgcm_model *m, double *out) {
  if (check_ready(m)) return -1;
  HIPCHK(hipSetDevice(m->device));
  const Dims &d = m->d;
  const Fields &f = m->f;
  const int nzmax = d.Nr;
  const size_t nval = (size_t)MON_NF * d.nT * nzmax * MON_NV;
  if (m->monCap < nval) {
    if (m->monBuf) (void)hipFree(m->monBuf);
    m->monBuf = nullptr;
    HIPCHK(hipMalloc(&m->monBuf, nval * sizeof(double)));
    m->monCap = nval;
  }
  MonSpecs S{};
  S.s[0] = MonSpec{f.etaN, f.maskInC, f.maskInC, f.rA, f.drF, 1, 0, 0};
  S.s[1] = MonSpec{f.uVel, f.hFacW, f.maskInW, f.rAw, f.drF, d.Nr, 1, 1};
  S.s[2] = MonSpec{f.vVel, f.hFacS, f.maskInS, f.rAs, f.drF, d.Nr, 1, 1};
  S.s[3] = MonSpec{f.wVel, f.maskC, f.maskInC, f.rA, f.drC, d.Nr, 1, 1};
  S.s[4] = MonSpec{f.theta, f.hFacC, f.maskInC, f.rA, f.drF, d.Nr, 1, 1};
  S.s[5] = MonSpec{f.salt, f.hFacC, f.maskInC, f.rA, f.drF, d.Nr, 1, 1};
  std::vector<double> h(nval);
  double nb[MON_NF], d2[MON_NF], vol[MON_NF], sum[MON_NF], mn[MON_NF], mx[MON_NF], sd[MON_NF];
  for (int pass = 0; pass < 2; pass++) {
    HIPCHK(launch_mon_stats(d, S, nzmax, m->monBuf, pass, m->stream));
    HIPCHK(hipMemcpyAsync(h.data(), m->monBuf, nval * sizeof(double), hipMemcpyDeviceToHost, m->stream));
    HIPCHK(hipStreamSynchronize(m->stream));
    for (int fi = 0; fi < MON_NF; fi++) {
      double a[MON_NV] = {0.0, 0.0, 0.0, 0.0, INFINITY, -INFINITY};
      for (int t = 0; t < d.nT; t++)
        for (int k = 0; k < S.s[fi].nz; k++) {
          const double *v = &h[(((size_t)fi * d.nT + t) * nzmax + k) * MON_NV];
          for (int q = 0; q < 4; q++) a[q] = a[q] + v[q];
          a[4] = fmin(a[4], v[4]);
          a[5] = fmax(a[5], v[5]);
        }
      if (pass == 0) {
        nb[fi] = a[0]; d2[fi] = a[1]; vol[fi] = a[2]; sum[fi] = a[3]; mn[fi] = a[4]; mx[fi] = a[5];
        S.mean[fi] = vol[fi] > 0.0 ? sum[fi] / vol[fi] : 0.0;
      } else {
        sd[fi] = vol[fi] > 0.0 ? sqrt(a[3] / vol[fi]) : 0.0;
      }
    }
  }
  for (int fi = 0; fi < MON_NF; fi++) {
    const bool any = nb[fi] > 0.0;   // mon_calc_stats_rl.F: min = max = 0 with no wet point
    out[fi * 5 + 0] = any ? mx[fi] : 0.0;
    out[fi * 5 + 1] = any ? mn[fi] : 0.0;
    out[fi * 5 + 2] = S.mean[fi];
    out[fi * 5 + 3] = sd[fi];
    out[fi * 5 + 4] = any ? sqrt(d2[fi]) / nb[fi] : 0.0;
  }
  return 0;
}

void mgcm_kernel_timing(mgcm_model *m, int enable) {
  hipStreamSynchronize(m->stream);
  ev_collect(m);
  for (int k = 0; k < K_N; k++) { m->kms[k] = 0; m->kcnt[k] = 0; }
  m->timing = enable != 0;
}

double mgcm_kernel_ms(mgcm_model *m, const char *name, int *launches) {
  hipStreamSynchronize(m->stream);
  ev_collect(m);
  for (int k = 0; k < K_N; k++)
    if (!strcmp(KNAMES[k], name)) {
      if (launches) *launches = m->kcnt[k];
      return m->kcnt[k] ? m->kms[k] / m->kcnt[k] : 0.0;
    }
  if (launches) *launches = 0;
  return -1.0;
}

// The order in which the selected CG2D kernel forms its global sums (GLOBAL_SUM_TILE_RL's
// replacement), for the oracle to restate it: thread tid accumulates the per-point terms of
// plan[p*NT + tid] (2-D flat offsets; -1 = padding) for p = 0..PPT-1 in order, starting from
// 0.0; the NT thread partials are then combined by the pairwise tree the DPP row sums,
// row broadcasts and the cross-wave row sum implement (block_sum / block_sum_nw: lanes
// (2i, 2i+1), then pairs of pairs, ..., in thread order, zero-padded to a power of two).
int mgcm_cg2d_sum_plan(mgcm_model *m, int *plan, long capacity, int *NT, int *PPT, int *NG) {
  if (!m->ready) return set_err("mgcm_cg2d_sum_plan: model not initialised");
  int nt, ppt, ng = 1;
  std::vector<int> tab;
  if (m->useMwg) {
    int rpt;
    cg2d_mwg_geometry(&nt, &ppt, &rpt);
    ng = m->mwg.G;
    tab = m->mwgPlan;
  } else if (m->nBlkX > 0) {
    int BX, BY;
    cg2d_bxy_geometry(m->bxyVar, &BX, &BY, &nt);
    ppt = BX * BY;
    std::vector<int> blkx((size_t)ppt * nt);
    HIPCHK(hipMemcpy(blkx.data(), m->d_blkx, blkx.size() * sizeof(int), hipMemcpyDeviceToHost));
    tab.assign((size_t)ppt * nt, -1);
    for (int t = 0; t < m->nBlkX; t++)
      for (int q = 0; q < ppt; q++) tab[(size_t)q * nt + t] = blkx[(size_t)ppt * t + q];
  } else if (m->nBlk > 0) {
    nt = 1024; ppt = 4;
    std::vector<int> blk((size_t)4 * nt);
    HIPCHK(hipMemcpy(blk.data(), m->d_blk, blk.size() * sizeof(int), hipMemcpyDeviceToHost));
    tab.assign((size_t)4 * nt, -1);
    for (int t = 0; t < m->nBlk; t++)
      for (int q = 0; q < 4; q++) tab[(size_t)q * nt + t] = blk[(size_t)4 * t + q];
  } else {
    nt = 1024; ppt = cg2d_block_ppt(m->nPts);
    std::vector<int> gofs((size_t)ppt * nt);
    HIPCHK(hipMemcpy(gofs.data(), m->d_gofs, gofs.size() * sizeof(int), hipMemcpyDeviceToHost));
    tab.assign((size_t)ppt * nt, -1);
    for (int q = 0; q < ppt; q++)
      for (int t = 0; t < nt; t++)
        if (t + q * nt < m->nPts) tab[(size_t)q * nt + t] = gofs[(size_t)t + (size_t)q * nt];
  }
  *NT = nt;
  *PPT = ppt;
  *NG = ng;
  if ((long)tab.size() > capacity) return set_err("mgcm_cg2d_sum_plan: capacity %ld < %zu", capacity, tab.size());
  memcpy(plan, tab.data(), tab.size() * sizeof(int));
  return 0;
}

int mgcm_cg2d(mgcm_model *m, double *cg2d_b, double *cg2d_x, double *firstResidual, double *minResidualSq,
              double *lastResidual, int *numIters, int *nIterMin) {
  if (check_ready(m)) return -1;
  const long n = m->d.n2 * m->d.nTiles;
  HIPCHK(hipSetDevice(m->device));
  HIPCHK(mg_host_copy(m->f.cg2d_b, cg2d_b, n * sizeof(double), hipMemcpyHostToDevice, m->stream));
  HIPCHK(mg_host_copy(m->f.cg2d_x, cg2d_x, n * sizeof(double), hipMemcpyHostToDevice, m->stream));
  HIPCHK(hipMemsetAsync(m->d_ctr + 1, 0, sizeof(int), m->stream));
  // CG2D itself (cg2d.F): useSRCGSolver selects CG2D_SR only in SOLVE_FOR_PRESSURE
  const int sr = m->p.useSRCGSolver;
  m->p.useSRCGSolver = 0;
  const int ev = ev_begin(m, K_CG2D);
  const hipError_t le = launch_cg2d(m, *numIters, *nIterMin);
  ev_end(m, K_CG2D, ev);
  m->p.useSRCGSolver = sr;
  HIPCHK(le);
  HIPCHK(mg_host_copy(cg2d_b, m->f.cg2d_b, n * sizeof(double), hipMemcpyDeviceToHost, m->stream));
  HIPCHK(mg_host_copy(cg2d_x, m->f.cg2d_x, n * sizeof(double), hipMemcpyDeviceToHost, m->stream));
  SolveRecord r;
  HIPCHK(hipMemcpyAsync(&r, m->d_rec, sizeof r, hipMemcpyDeviceToHost, m->stream));
  HIPCHK(hipStreamSynchronize(m->stream));
  *firstResidual = r.firstResidual;
  *minResidualSq = r.minResidualSq;
  *lastResidual = r.lastResidual;
  *numIters = r.numIters;
  *nIterMin = r.nIterMin;
  return 0;
}

}  // extern "C"
