// fortran_abi.hip -- the Fortran side of the drop-in boundary.
//
// MITgcm's plugin mechanism is source shadowing: a file in a genmake2 `-mods` directory
// replaces the same-named routine of model/src or eesupp/src (tools/genmake2:2231-2241).
// The shims in mitgcm_amd/fortran/mods/ keep the reference's SUBROUTINE names and argument
// lists and call the entry points below (lower case + '_', every argument by reference,
// CHARACTER lengths appended as size_t -- amdflang's external convention).
//
// Coherence model (the "device mirror" keyed by COMMON-block address):
//   * MGCM_AMD_BIND(name, array, count, kind) registers a host array -- a COMMON-block member
//     of DYNVARS.h / GRID.h / SURFACE.h / FFIELDS.h / CG2D.h / GMREDI.h -- under the device
//     field of the same name, in one of three kinds: 1 static (grid metrics, masks: uploaded
//     once, by MGCM_AMD_INIT), 0 state, 2 host input (what the host's LOAD_FIELDS_DRIVER
//     writes every step: the forcing fields);
//   * while the model initialises (INITIALISE_VARIA runs UPDATE_CG2D, CALC_R_STAR,
//     UPDATE_R_STAR, INTEGR_CONTINUITY through the drop-ins, interleaved with host INI_*
//     routines) the host copy is authoritative: each drop-in uploads the state before and
//     downloads it after;
//   * from the first DO_OCEANIC_PHYS / THERMODYNAMICS / DYNAMICS -- routines only
//     FORWARD_STEP calls -- the device copy is authoritative: the state is uploaded once,
//     each step uploads only the host input (before DO_OCEANIC_PHYS), and the state comes
//     back only after the DO_FIELDS_BLOCKING_EXCHANGES of a step whose end a host routine
//     reads (MONITOR, DO_THE_MODEL_IO, DO_WRITE_PICKUP: monitorFreq, dumpFreq, chkPtFreq,
//     pChkPtFreq by the reference's DIFFERENT_MULTIPLE test, and the last iteration
//     nEndIter), or when the host asks (MGCM_AMD_HOST_SYNC; MGCM_AMD_DEVICE_SYNC pushes a
//     host-modified state back).  A step in between moves the forcing fields (6 2-D arrays)
//     and nothing else across PCIe.
// mgcm_amd_transfer_stats_ counts the copies, so a host can check the schedule.
//
// Errors: no return channel exists in the reference (it prints and STOPs), so every
// failure prints "ABNORMAL END: <routine>: <reason>" and aborts.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mitgcm_amd.h"

namespace {

struct Bound {
  std::string name;   // device field
  double *host;
  long count;         // doubles moved
  int kind;           // 0 state, 1 static, 2 host input (MGCM_AMD_BIND)
  int stride = 1, off = 0;   // host element q*stride + off <-> device element q
};

// When a host routine reads the state at the end of a step (the device-authoritative
// mirror downloads it then): the frequencies of PARAMS.h, in seconds, and nEndIter.
struct Readers {
  double monitorFreq = 0.0, dumpFreq = 0.0, chkPtFreq = 0.0, pChkPtFreq = 0.0, deltaTClock = 0.0;
  int nEndIter = -1;
};

struct FortranSide {
  mgcm_model *m = nullptr;
  int dims[7] = {0, 0, 0, 0, 0, 0, 0};   // sNx sNy OLx OLy Nr nSx nSy
  std::vector<Bound> bound;
  bool ready = false;
  bool deviceAuth = false;   // the device copy of the state is authoritative (time loop)
  long devIter = -1;         // the iteration counter last written to the device (-1: unknown)
  double lastTime = 0.0;     // myTime / myIter of the latest routine drop-in
  int lastIter = 0;
  Readers rd;
  long nUp = 0, nDown = 0;   // copies of whole bound arrays, for mgcm_amd_transfer_stats_
  double bytesUp = 0.0, bytesDown = 0.0;
};
FortranSide g;

[[noreturn]] void die(const char *where, const char *why = nullptr) {
  fprintf(stderr, "ABNORMAL END: %s: %s\n", where, why ? why : mgcm_last_error());
  fflush(stderr);
  abort();
}

std::string fstr(const char *s, size_t len) {   // Fortran CHARACTER: blank padded, no NUL
  while (len > 0 && (s[len - 1] == ' ' || s[len - 1] == '\0')) len--;
  return std::string(s, len);
}

mgcm_model *model(const char *where) {
  if (!g.m) die(where, "called before MGCM_AMD_SETUP");
  return g.m;
}

// The device's iteration counter (AB2's first step, the CD scheme's start), written only
// when it changes (FORWARD_STEP advances myIter after DYNAMICS, forward_step.F:806), in
// stream order: no host synchronisation.
void set_iter(const char *where, int myIter) {
  if (g.devIter == myIter) return;
  if (mgcm_set_iter(g.m, myIter)) die(where);
  g.devIter = myIter;
}

// kinds: bit k set = move the arrays of kind k
void upload(const char *where, unsigned kinds) {
  std::vector<double> tmp;
  for (auto &b : g.bound) {
    if (!((kinds >> b.kind) & 1u)) continue;
    const double *src = b.host;
    if (b.stride != 1) {
      tmp.resize(b.count);
      for (long q = 0; q < b.count; q++) tmp[q] = b.host[q * b.stride + b.off];
      src = tmp.data();
    }
    if (mgcm_put(g.m, b.name.c_str(), src, b.count)) die(where);
    g.nUp++;
    g.bytesUp += 8.0 * b.count;
  }
}

void download(const char *where) {
  if (mgcm_sync(g.m)) die(where);
  std::vector<double> tmp;
  for (auto &b : g.bound) {
    if (b.kind != 0) continue;   // static and host-input arrays are never written on the device
    g.nDown++;
    g.bytesDown += 8.0 * b.count;
    if (b.stride == 1) {
      if (mgcm_get(g.m, b.name.c_str(), b.host, b.count)) die(where);
      continue;
    }
    tmp.resize(b.count);
    if (mgcm_get(g.m, b.name.c_str(), tmp.data(), b.count)) die(where);
    for (long q = 0; q < b.count; q++) b.host[q * b.stride + b.off] = tmp[q];
  }
}

constexpr unsigned K_STATE = 1u << 0, K_STATIC = 1u << 1, K_INPUT = 1u << 2;

// The time loop has begun (a routine only FORWARD_STEP calls): the host's state goes up
// once and the device copy becomes the authoritative one.
void enter_time_loop(const char *where) {
  if (g.deviceAuth) return;
  upload(where, K_STATE | K_INPUT);
  g.deviceAuth = true;
}

// One routine drop-in.  Host-authoritative (initialisation): state in, the device
// routine, state out.  Device-authoritative: the host input first when `input`.
void routine(const char *where, int (*fn)(mgcm_model *), int myIter, double myTime, bool input = false) {
  model(where);
  if (!g.ready) die(where, "called before MGCM_AMD_INIT");
  g.lastIter = myIter;
  g.lastTime = myTime;
  if (!g.deviceAuth) {
    upload(where, K_STATE | K_INPUT);
    set_iter(where, myIter);
    if (fn(g.m)) die(where);
    download(where);
    return;
  }
  if (input) upload(where, K_INPUT);
  set_iter(where, myIter);
  if (fn(g.m)) die(where);
}

// eesupp/src/different_multiple.F: is val1 the step nearest to a multiple of freq?
bool different_multiple(double freq, double val1, double step) {
  if (freq == 0.0) return false;
  if (fabs(step) > freq) return true;
  const double v1 = val1, v2 = val1 - step, v3 = val1 + step;
  const double v4 = nearbyint(v1 / freq) * freq;
  const double d1 = v1 - v4, d2 = v2 - v4, d3 = v3 - v4;
  return fabs(d1) < fabs(d2) && fabs(d1) <= fabs(d3);
}

// Does a host routine read the state at the end of this step?  MONITOR
// (monitor.F:48), DO_THE_MODEL_IO (do_the_model_io.F:106), DO_WRITE_PICKUP
// (do_write_pickup.F:61-63, modelEnd) -- a superset is harmless, a miss is not.
bool host_reads_state(double myTime, int myIter) {
  const Readers &r = g.rd;
  return myIter == r.nEndIter || different_multiple(r.monitorFreq, myTime, r.deltaTClock) ||
         different_multiple(r.dumpFreq, myTime, r.deltaTClock) ||
         different_multiple(r.chkPtFreq, myTime, r.deltaTClock) ||
         different_multiple(r.pChkPtFreq, myTime, r.deltaTClock);
}

const Bound *bound_at(const double *p) {
  for (auto &b : g.bound)
    if (b.host == p) return &b;
  return nullptr;
}

}  // namespace

extern "C" {

// --------------------------------------------------------------------- set-up
/* The tile set of SIZE.h; nProcs = nPx*nPy and nThreads = nTx*nTy must be 1 (one host
 * process and thread per model, SURVEY.md 8(b) "Threading").  Re-creates the model when
 * the sizes change. */
void mgcm_amd_setup_(const int *sNx, const int *sNy, const int *OLx, const int *OLy, const int *Nr, const int *nSx,
                     const int *nSy, const int *nProcs, const int *nThreads) {
  if (*nProcs != 1 || *nThreads != 1) die("MGCM_AMD_SETUP", "the drop-ins need nPx*nPy = nTx*nTy = 1");
  const int d[7] = {*sNx, *sNy, *OLx, *OLy, *Nr, *nSx, *nSy};
  if (g.m && memcmp(d, g.dims, sizeof d) == 0) return;
  if (g.m) mgcm_destroy(g.m);
  g = FortranSide{};
  g.m = mgcm_create(d[0], d[1], d[2], d[3], d[4], d[5], d[6], 0);
  if (!g.m) die("MGCM_AMD_SETUP");
  memcpy(g.dims, d, sizeof d);
}

/* The halo maps of a pkg/exch2 topology (MGCM_AMD_EXCH2_MAPS, mods/mgcm_amd_exch2.F): the
 * reference's own EXCH2_3D_RL / EXCH2_UV_CGRID_3D_RL run on index arrays.  ids: per point
 * the flat index of the point it copies (its own when untouched); u1/v1 (withSigns) and
 * u0/v0: 0 or +-(source+1) into [u | v]; per tile its face and facet-edge bits. */
void mgcm_amd_set_maps_(const double *ids, const double *u1, const double *v1, const double *u0, const double *v0,
                        const int *tFace, const int *tEdge, const int *nPts) {
  model("MGCM_AMD_SET_MAPS");
  const long n = *nPts;
  std::vector<long> src(n), cu1(n), cv1(n), cu0(n), cv0(n);
  for (long q = 0; q < n; q++) {
    src[q] = (long)ids[q];
    cu1[q] = (long)u1[q]; cv1[q] = (long)v1[q]; cu0[q] = (long)u0[q]; cv0[q] = (long)v0[q];
  }
  if (mgcm_set_halo_map(g.m, src.data(), n)) die("MGCM_AMD_SET_MAPS");
  if (mgcm_set_uv_map(g.m, cu1.data(), cv1.data(), cu0.data(), cv0.data(), tFace, tEdge, n)) die("MGCM_AMD_SET_MAPS");
  g.ready = false;
}

/* One run-time parameter under its PARAMS.h name (LOGICALs as 0/1, INTEGERs as reals). */
void mgcm_amd_param_(const char *name, const double *value, size_t len) {
  model("MGCM_AMD_PARAM");
  const std::string n = fstr(name, len);
  // the host-side schedule of state readers stays here (no device meaning)
  Readers &r = g.rd;
  if (n == "monitorFreq") { r.monitorFreq = *value; return; }
  if (n == "dumpFreq") { r.dumpFreq = *value; return; }
  if (n == "chkPtFreq") { r.chkPtFreq = *value; return; }
  if (n == "pChkPtFreq") { r.pChkPtFreq = *value; return; }
  if (n == "nEndIter") { r.nEndIter = (int)*value; return; }
  if (n == "deltaTClock") r.deltaTClock = *value;
  if (mgcm_set_param(g.m, n.c_str(), *value)) die("MGCM_AMD_PARAM");
  g.ready = false;
}

/* Register a host array (a COMMON-block member) of `count` doubles as the device field
 * `name` (same name), of kind 0 (state), 1 (static) or 2 (host input), see above.  1-D profiles may be shorter than the device's Nr+1 (drF(Nr)).
 * phiRef(2*Nr+1) of set_ref_state.F is bound as the device's phiRefC = phiRef(2k). */
void mgcm_amd_bind_(const char *name, double *array, const int *count, const int *kind, size_t len) {
  model("MGCM_AMD_BIND");
  std::string n = fstr(name, len);
  if (*kind < 0 || *kind > 2) die("MGCM_AMD_BIND", "kind must be 0 (state), 1 (static) or 2 (host input)");
  Bound nb{n, array, *count, *kind};
  if (n == "phiRef") {
    const int Nr = g.dims[4];
    if (*count != 2 * Nr + 1) die("MGCM_AMD_BIND", "phiRef must have 2*Nr+1 entries");
    nb.name = "phiRefC";
    nb.count = Nr;
    nb.stride = 2;
    nb.off = 1;
  }
  const long have = mgcm_field_count(g.m, nb.name.c_str());
  if (have < 0) die("MGCM_AMD_BIND");
  if (nb.count < 1 || nb.count > have) {
    fprintf(stderr, "ABNORMAL END: MGCM_AMD_BIND: %s has %ld doubles, the device field %ld\n", n.c_str(), nb.count,
            have);
    abort();
  }
  for (auto &b : g.bound)
    if (b.name == nb.name) {
      b = nb;
      return;
    }
  g.bound.push_back(nb);
  g.ready = false;
}

/* Upload every bound array and finish the device set-up (mgcm_init); the host state
 * stays authoritative until the time loop: anything mgcm_init derives on the device is
 * overwritten by the host's state again. */
void mgcm_amd_init_(const int *myIter) {
  model("MGCM_AMD_INIT");
  // device options with no PARAMS.h counterpart, from the environment:
  // MGCM_CG2D_REFORDER=1 sums CG2D in the reference's order (cg2dRefOrder, parity runs)
  if (const char *e = getenv("MGCM_CG2D_REFORDER"))
    if (mgcm_set_param(g.m, "cg2dRefOrder", atof(e))) die("MGCM_AMD_INIT");
  upload("MGCM_AMD_INIT", K_STATIC | K_STATE | K_INPUT);
  if (mgcm_set_param(g.m, "myIter", (double)*myIter)) die("MGCM_AMD_INIT");
  if (mgcm_init(g.m)) die("MGCM_AMD_INIT");
  upload("MGCM_AMD_INIT", K_STATE | K_INPUT);
  if (mgcm_set_param(g.m, "myIter", (double)*myIter)) die("MGCM_AMD_INIT");
  g.devIter = *myIter;
  g.deviceAuth = false;
  g.ready = true;
}

/* The host reads the state now (a host routine outside the shadowed set): the device
 * copy comes down if it is the authoritative one. */
void mgcm_amd_host_sync_(const int *myThid) {
  (void)myThid;
  model("MGCM_AMD_HOST_SYNC");
  if (g.ready && g.deviceAuth) download("MGCM_AMD_HOST_SYNC");
}

/* The host has changed the state (e.g. re-read a pickup): it goes up to the device. */
void mgcm_amd_device_sync_(const int *myThid) {
  (void)myThid;
  model("MGCM_AMD_DEVICE_SYNC");
  if (g.ready && g.deviceAuth) upload("MGCM_AMD_DEVICE_SYNC", K_STATE | K_INPUT);
}

/* Waits for the device work issued so far (a timing aid for hosts that clock steps). */
void mgcm_amd_step_fence_(const int *myThid) {
  (void)myThid;
  if (mgcm_sync(model("MGCM_AMD_STEP_FENCE"))) die("MGCM_AMD_STEP_FENCE");
}

/* Whole-array copies so far (uploads, downloads) and their bytes. */
void mgcm_amd_transfer_stats_(int *nUploads, int *nDownloads, double *bytesUp, double *bytesDown) {
  *nUploads = (int)g.nUp;
  *nDownloads = (int)g.nDown;
  *bytesUp = g.bytesUp;
  *bytesDown = g.bytesDown;
}

// ------------------------------------------------------------ routine drop-ins
/* SUBROUTINE DO_OCEANIC_PHYS(myTime, myIter, myThid)     model/src/do_oceanic_phys.F:43 */
void do_oceanic_phys_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  enter_time_loop("DO_OCEANIC_PHYS_AMD");
  routine("DO_OCEANIC_PHYS_AMD", mgcm_oceanic_phys, *myIter, *myTime, true);
}
/* SUBROUTINE THERMODYNAMICS(myTime, myIter, myThid)      model/src/thermodynamics.F:25 */
void thermodynamics_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  enter_time_loop("THERMODYNAMICS_AMD");
  routine("THERMODYNAMICS_AMD", mgcm_tracer_step, *myIter, *myTime);
}
/* SUBROUTINE DYNAMICS(myTime, myIter, myThid)            model/src/dynamics.F:21 */
void dynamics_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  enter_time_loop("DYNAMICS_AMD");
  routine("DYNAMICS_AMD", mgcm_dynamics, *myIter, *myTime);
}
/* SUBROUTINE UPDATE_R_STAR(useLatest, myTime, myIter, myThid)   model/src/update_r_star.F:6
 * useLatest = .TRUE. (forward_step.F:838): the new r* factors and hFac, and UPDATE_CG2D's
 * operator (update_cg2d.F:7, forward_step.F:868) with them -- one device pass.
 * useLatest = .FALSE. (RESET_NLFS_VARS + UPDATE_R_STAR at the start of the step,
 * forward_step.F:469-477) restores the hFac of the previous step's end, which the mirror
 * already holds: nothing to do. */
void update_r_star_amd_(const int *useLatest, const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  if (*useLatest) routine("UPDATE_R_STAR_AMD", mgcm_update_r_star, *myIter, *myTime);
}
/* SUBROUTINE UPDATE_CG2D(myTime, myIter, myThid)         model/src/update_cg2d.F:7
 * Folded into UPDATE_R_STAR_AMD(.TRUE.), which FORWARD_STEP calls just before it. */
void update_cg2d_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myTime; (void)myIter; (void)myThid;
  model("UPDATE_CG2D_AMD");
}
/* SUBROUTINE CALC_R_STAR(etaFld, myTime, myIter, myThid)  model/src/calc_r_star.F:10
 * FORWARD_STEP passes etaH (forward_step.F:976): the bound array. */
void calc_r_star_amd_(const double *etaFld, const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  const Bound *b = bound_at(etaFld);
  if (!b || b->name != "etaH") die("CALC_R_STAR_AMD", "etaFld must be the bound etaH");
  routine("CALC_R_STAR_AMD", mgcm_calc_r_star, *myIter, *myTime);
}
/* SUBROUTINE SOLVE_FOR_PRESSURE(myTime, myIter, myThid)  model/src/solve_for_pressure.F:7 */
void solve_for_pressure_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  routine("SOLVE_FOR_PRESSURE_AMD", mgcm_solve_for_pressure, *myIter, *myTime);
}
/* SUBROUTINE MOMENTUM_CORRECTION_STEP(myTime, myIter, myThid)
 *                                                   model/src/momentum_correction_step.F:7 */
void momentum_correction_step_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  routine("MOMENTUM_CORRECTION_STEP_AMD", mgcm_momentum_correction_step, *myIter, *myTime);
}
/* SUBROUTINE INTEGR_CONTINUITY(uFld, vFld, myTime, myIter, myThid)
 *                                                   model/src/integr_continuity.F:13
 * FORWARD_STEP passes uVel, vVel (forward_step.F:955): the bound arrays. */
void integr_continuity_amd_(const double *uFld, const double *vFld, const double *myTime, const int *myIter,
                            const int *myThid) {
  (void)myThid;
  const Bound *bu = bound_at(uFld), *bv = bound_at(vFld);
  if (!bu || !bv || bu->name != "uVel" || bv->name != "vVel")
    die("INTEGR_CONTINUITY_AMD", "uFld, vFld must be the bound uVel, vVel");
  routine("INTEGR_CONTINUITY_AMD", mgcm_integr_continuity, *myIter, *myTime);
}
/* SUBROUTINE DO_FIELDS_BLOCKING_EXCHANGES(myThid)   model/src/do_fields_blocking_exchanges.F:7 */
/* The last device routine of a step: the state comes down when a host routine reads it
 * next (MONITOR / DO_THE_MODEL_IO / DO_WRITE_PICKUP at this step's end time, known from
 * the step's earlier drop-ins, which FORWARD_STEP calls with the advanced myTime). */
void do_fields_blocking_exchanges_amd_(const int *myThid) {
  (void)myThid;
  const int it = g.lastIter;
  const double t = g.lastTime;
  routine("DO_FIELDS_BLOCKING_EXCHANGES_AMD", mgcm_blocking_exchanges, it, t);
  if (g.deviceAuth && host_reads_state(t, it)) download("DO_FIELDS_BLOCKING_EXCHANGES_AMD");
}

// -------------------------------------------------- exchanges and global sums
/* SUBROUTINE EXCH_XY_RL(phi, myThid)             eesupp/src/exch_xy_rx.template:9 */
void exch_xy_rl_amd_(double *phi, const int *myThid) {
  (void)myThid;
  if (mgcm_exchange_host(model("EXCH_XY_RL_AMD"), phi, nullptr, 1, 0, 0)) die("EXCH_XY_RL_AMD");
}
/* SUBROUTINE EXCH_XYZ_RL(phi, myThid)            eesupp/src/exch_xyz_rx.template:8 */
void exch_xyz_rl_amd_(double *phi, const int *myThid) {
  (void)myThid;
  if (mgcm_exchange_host(model("EXCH_XYZ_RL_AMD"), phi, nullptr, g.dims[4], 0, 0)) die("EXCH_XYZ_RL_AMD");
}
/* SUBROUTINE EXCH_UV_XY_RL(uPhi, vPhi, withSigns, myThid)   eesupp/src/exch_uv_xy_rx.template:11 */
void exch_uv_xy_rl_amd_(double *u, double *v, const int *withSigns, const int *myThid) {
  (void)myThid;
  if (mgcm_exchange_host(model("EXCH_UV_XY_RL_AMD"), u, v, 1, 1, *withSigns != 0)) die("EXCH_UV_XY_RL_AMD");
}
/* SUBROUTINE EXCH_UV_XYZ_RL(uPhi, vPhi, withSigns, myThid)  eesupp/src/exch_uv_xyz_rx.template:12 */
void exch_uv_xyz_rl_amd_(double *u, double *v, const int *withSigns, const int *myThid) {
  (void)myThid;
  if (mgcm_exchange_host(model("EXCH_UV_XYZ_RL_AMD"), u, v, g.dims[4], 1, *withSigns != 0))
    die("EXCH_UV_XYZ_RL_AMD");
}
/* SUBROUTINE GLOBAL_SUM_TILE_RL(phiTile, sumPhi, myThid)    eesupp/src/global_sum_tile.F:14
 * One process: the tile partials summed in global tile order, bi fastest, from zero
 * (global_sum_tile.F:150-156) -- the order every device reduction of the path keeps at
 * the tile level. */
void global_sum_tile_rl_amd_(const double *phiTile, double *sumPhi, const int *myThid) {
  (void)myThid;
  model("GLOBAL_SUM_TILE_RL_AMD");
  const int n = g.dims[5] * g.dims[6];
  double s = 0.0;
  for (int t = 0; t < n; t++) s = s + phiTile[t];
  *sumPhi = s;
}

// ------------------------------------------------------------------- CG2D
/* Registers the CG2D operator of CG2D.h (ini_cg2d.F:61-237 outputs) for CG2D_AMD; a model
 * made by MGCM_AMD_SETUP is reused when the sizes agree (Nr taken from it). */
void ini_cg2d_amd_(const int *sNx, const int *sNy, const int *OLx, const int *OLy, const int *nSx, const int *nSy,
                   const double *aW2d, const double *aS2d, const double *aC2d, const double *pW, const double *pS,
                   const double *pC, const double *cg2dNorm, const double *cg2dTolerance_sq,
                   const int *cg2dNormaliseRHS) {
  const int one = 1, Nr = g.m ? g.dims[4] : 1;
  if (!(g.m && g.dims[0] == *sNx && g.dims[1] == *sNy && g.dims[2] == *OLx && g.dims[3] == *OLy &&
        g.dims[5] == *nSx && g.dims[6] == *nSy))
    mgcm_amd_setup_(sNx, sNy, OLx, OLy, &Nr, nSx, nSy, &one, &one);
  const long n = mgcm_field_count(g.m, "aW2d");
  if (mgcm_put(g.m, "aW2d", aW2d, n) || mgcm_put(g.m, "aS2d", aS2d, n) || mgcm_put(g.m, "aC2d", aC2d, n) ||
      mgcm_put(g.m, "pW", pW, n) || mgcm_put(g.m, "pS", pS, n) || mgcm_put(g.m, "pC", pC, n) ||
      mgcm_set_param(g.m, "cg2dNorm", *cg2dNorm) || mgcm_set_param(g.m, "cg2dTolerance_sq", *cg2dTolerance_sq) ||
      mgcm_set_param(g.m, "cg2dNormaliseRHS", (double)*cg2dNormaliseRHS))
    die("INI_CG2D_AMD");
  if (!g.ready) {
    if (mgcm_init(g.m)) die("INI_CG2D_AMD");
    g.ready = true;
  }
}

/* SUBROUTINE CG2D(cg2d_b, cg2d_x, firstResidual, minResidualSq, lastResidual, numIters,
 *                 nIterMin, myThid)                        model/src/cg2d.F:13-17 */
void cg2d_amd_(double *cg2d_b, double *cg2d_x, double *firstResidual, double *minResidualSq, double *lastResidual,
               int *numIters, int *nIterMin, const int *myThid) {
  (void)myThid;
  if (!g.m || !g.ready) die("CG2D_AMD", "called before INI_CG2D_AMD");
  if (mgcm_cg2d(g.m, cg2d_b, cg2d_x, firstResidual, minResidualSq, lastResidual, numIters, nIterMin)) die("CG2D_AMD");
}

}  // extern "C"
