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
// Tiles over GPUs (the reference's tile set of one process spread over device models, SURVEY
// 8(e) "tiles shard one-per-GPU" with the host staying one Fortran process): MGCM_AMD_MODELS =
// N (or "auto" = min(tiles, GPUs); default 1) device models, model i owning the contiguous,
// balanced tile range i of the global tile order (bi fastest) on GPU MGCM_AMD_DEVICES[i]
// (default: contiguous blocks of models per GPU, one model per GPU when N <= GPUs).  Every
// model holds the whole domain's arrays; its 3-D kernels step its own tiles.  A routine
// drop-in runs the routine on every model, with the exchange points of the MPI reference in
// between -- where an MPI rank would EXCH or GLOBAL_SUM, the models copy device to device:
//   * DO_FIELDS_BLOCKING_EXCHANGES: the 3-D halo sources a model's halos read from another
//     model's tiles (exch1_rx.template:170-198 / exch2_rx1_cube.template:118-247's send/recv),
//     packed, copied GPU to GPU, unpacked, then each model's local halo fill;
//   * SOLVE_FOR_PRESSURE: the right-hand side's tile blocks to every model, then CG2D --
//     the multi-workgroup device CG2D, launched once per GPU over the tiles of that GPU's
//     models on ONE hand-off block shared by the GPUs (uncached, system scope), the
//     solution's blocks back to every model; or, where the solver is a single-CU kernel,
//     the whole (gathered) solve on every model -- same sums as one model, bit for bit;
//   * INTEGR_CONTINUITY (exactConserv): the new free surface's blocks to every model before
//     EXCH(eta) + UPDATE_ETAH; the r* passes (UPDATE_R_STAR, CALC_R_STAR) run on every tile
//     of every model (2-D, identical inputs).
// Copies move only tile blocks and halo-source points; the host state comes down from each
// tile's owner.  Results are bit-identical to one model at any N (tests/test_gpu_refhost.py).
// The device ordering between models is by events (every exchange point is a cross-stream
// barrier), so no host synchronisation enters a step.
//
// Errors: no return channel exists in the reference (it prints and STOPs), so every
// failure prints "ABNORMAL END: <routine>: <reason>" and aborts.
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mitgcm_amd.h"

namespace mgcm {   // model.hip: the registered host ranges host<->device copies split at
void mg_host_ranges_set(const uintptr_t *lo, const uintptr_t *hi, size_t n);
hipError_t mg_host_copy(void *dst, const void *src, size_t bytes, hipMemcpyKind kind, hipStream_t s);
}

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
  bool everyStep = false;   // a host routine reads the state after every step (useSBO, state diagnostics)
};

// One device model of the host's tile set: tiles [t0, t0+nT) on GPU dev.
struct Shard {
  mgcm_model *m = nullptr;
  int dev = 0, t0 = 0, nT = 0;
  int gpu = 0;   // the GPU the model stands for (== dev, except under MGCM_AMD_DEVICES=virtual)
  hipEvent_t ev = nullptr;   // cross-model barriers
};
// The halo sources model s's tiles deliver to model d (sorted 2-D offsets, the same on both
// sides: every model holds the domain at the same offsets), with a send buffer on s's GPU and
// a receive buffer on d's.
struct Link {
  int s = 0, d = 0;
  long n = 0;
  long *idxS = nullptr, *idxD = nullptr;
  double *sbuf = nullptr, *rbuf = nullptr;
  hipEvent_t ev = nullptr;   // on s: the copy into rbuf is done
};
// Per GPU: the model that launches the device CG2D over the tiles of all that GPU's models.
struct CgLead {
  int shard = 0, t0 = 0, nT = 0;
};

struct FortranSide {
  mgcm_model *m = nullptr;               // model 0: the tile set's single-model entries (EXCH_*, CG2D)
  std::vector<Shard> sh;                 // every device model (sh[0].m == m)
  std::vector<Link> links;
  std::vector<CgLead> cgLeads;
  bool cgDevice = false;                 // CG2D: device multi-workgroup solve (else replicated)
  bool exactConserv = false;
  std::vector<void *> devAllocs;         // (device, pointer) pairs of the links' buffers
  int dims[7] = {0, 0, 0, 0, 0, 0, 0};   // sNx sNy OLx OLy Nr nSx nSy
  std::vector<Bound> bound;
  bool ready = false;
  bool deviceAuth = false;   // the device copy of the state is authoritative (time loop)
  long devIter = -1;         // the iteration counter last written to the device (-1: unknown)
  double lastTime = 0.0;     // myTime / myIter of the latest routine drop-in
  int lastIter = 0;
  // myTime / myIter after FORWARD_STEP advances them (forward_step.F:806-807), from a drop-in
  // FORWARD_STEP calls after that line in the current step (SOLVE_FOR_PRESSURE, ...); unset
  // (advValid false) until one runs
  bool advValid = false;
  double advTime = 0.0;
  int advIter = 0;
  Readers rd;
  // Graph-replayed steps (one model): the drop-in sequence of a device-authoritative step is
  // recorded; once one has run eagerly in FORWARD_STEP's order, every later step runs as ONE
  // replay of the captured step at its DO_OCEANIC_PHYS (after the forcing upload), and the
  // step's other drop-ins only check that they come in the recorded order (fusedPos)
  std::vector<std::string> seq, fusedSeq;
  bool recording = false, canFuse = false, fused = false;
  size_t fusedPos = 0;
  // N > 1 models: the recorded step captured across every model's stream (the cross-model
  // copies as memcpy nodes, the barriers as event edges) into one graph per tracer-buffer
  // parity, and the parity each model is left at by the captured step's host-side swaps
  struct MultiGraph {
    hipGraphExec_t exec = nullptr;
    std::vector<int> pre, post;   // every model's tracer parity before / after the captured step
  } mg[4];
  bool capturing = false;     // set_iter inside a capture: device increments, not values
  bool capMulti = false;      // ... with every model on its own stream (MGCM_AMD_CAPTURE=multi)
  // Events recorded inside a multi-model capture: with the pool on (the default), every
  // record of a captured step takes an event of its own from evPool (filled before the
  // capture, kept for the graphs' life), so no hipEvent_t is recorded twice in one graph
  struct EvPool {
    int dev = 0;
    std::vector<hipEvent_t> ev;
    size_t next = 0;
  };
  std::vector<EvPool> evPools;
  bool multiGraphOff = false; // a capture failed: the multi-model steps stay eager
  // Models over several GPUs: the recorded step as per-GPU graphs cut at every cross-GPU
  // exchange point (segments): segment k of GPU group j is captured on that group's lead
  // stream (the group's other models issue there too), and a replay launches segment k of
  // every group, then the cross-GPU barrier as plain events, then segment k+1 (seg_replay)
  struct SegGraphs {
    std::vector<std::vector<hipGraphExec_t>> seg;   // [segment][group]
    std::vector<int> pre, post;
  } sgr[4];
  bool segMode = false, segFail = false;            // inside a segmented capture / it failed
  std::vector<hipGraphExec_t> segCur;               // the open segment's graphs (one per group)
  std::vector<std::vector<hipGraphExec_t>> segAll;
  long nUp = 0, nDown = 0;   // copies of whole bound arrays, for mgcm_amd_transfer_stats_
  // the state arrays' host pages, registered with HIP once the time loop begins (downloads
  // then go straight to the COMMON blocks by DMA); false when registration was refused
  bool hostRegistered = false, regTried = false;
  std::vector<std::vector<double>> strided;   // downloads of the strided bound arrays
  double bytesUp = 0.0, bytesDown = 0.0;
};
FortranSide g;

[[noreturn]] void die(const char *where, const char *why = nullptr) {
  fprintf(stderr, "ABNORMAL END: %s: %s\n", where, why ? why : mgcm_last_error());
  fflush(stderr);
  abort();
}

// A fault in the host process (SIGSEGV, SIGBUS) prints the host stack, then hands the signal
// to whatever handled it before (the Fortran runtime's, the HIP runtime's, or the default
// action): the reference's hosts have no other channel for it.  Installed by MGCM_AMD_INIT,
// after the HIP runtime has set up its own.
struct sigaction g_oldSegv, g_oldBus;
void fatal_signal(int sig) {
  static const char msg[] = "ABNORMAL END: MGCM_AMD: fatal signal in the host process; stack:\n";
  (void)!write(2, msg, sizeof msg - 1);
  void *fr[64];
  const int n = backtrace(fr, 64);
  backtrace_symbols_fd(fr, n, 2);
  sigaction(sig, sig == SIGSEGV ? &g_oldSegv : &g_oldBus, nullptr);
  raise(sig);
}
void install_fault_report() {
  static bool done = false;
  if (done) return;
  done = true;
  struct sigaction sa {};
  sa.sa_handler = fatal_signal;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_oldSegv);
  sigaction(SIGBUS, &sa, &g_oldBus);
}

std::string fstr(const char *s, size_t len) {   // Fortran CHARACTER: blank padded, no NUL
  while (len > 0 && (s[len - 1] == ' ' || s[len - 1] == '\0')) len--;
  return std::string(s, len);
}

mgcm_model *model(const char *where) {
  if (!g.m) die(where, "called before MGCM_AMD_SETUP");
  return g.m;
}

void hipchk(hipError_t e, const char *where) {
  if (e != hipSuccess) die(where, hipGetErrorString(e));
}
hipStream_t stream_of(const Shard &s) { return (hipStream_t)mgcm_get_stream(s.m); }

// MGCM_AMD_CAPTURE=debug: each stage of a multi-model capture and replay printed (and the
// replay waited for), down to the device operations of the captured drop-ins, to place a
// fault inside the runtime
bool cap_opt(const char *tok);
bool cap_dbg_on() {
  static const bool on = cap_opt("debug");
  return on;
}
void cap_dbg(const char *what, int q) {
  if (cap_dbg_on()) { fprintf(stderr, "MGCM_AMD capture[%d]: %s\n", q, what); fflush(stderr); }
}
void cap_op(const char *what, int model) {
  if (cap_dbg_on() && g.capturing) { fprintf(stderr, "MGCM_AMD   op %s model %d\n", what, model); fflush(stderr); }
}

// MGCM_AMD_CAPTURE: comma-separated options of the multi-model step capture -- "multi" / "one"
// (each model keeps its own stream in the capture / all on model 0's; default: multi from 4
// models on), "relaxed" (capture
// mode), "nopool" (events re-recorded instead of one per record), "debug" (stage prints)
bool cap_opt(const char *tok) {
  const char *e = getenv("MGCM_AMD_CAPTURE");
  if (!e) return false;
  const size_t n = strlen(tok);
  for (const char *p = e; *p;) {
    const char *c = strchr(p, ',');
    const size_t len = c ? (size_t)(c - p) : strlen(p);
    if (len == n && !strncmp(p, tok, n)) return true;
    if (!c) break;
    p = c + 1;
  }
  return false;
}
bool cap_pool_on() {
  static const bool off = cap_opt("nopool");
  return !off;
}
// the event a record on device `dev` uses: outside a capture (or with the pool off) the
// caller's own; inside one, a fresh event of that device's pool
hipEvent_t rec_event(int dev, hipEvent_t own, const char *where) {
  if (!g.capturing || !cap_pool_on()) return own;
  for (auto &p : g.evPools)
    if (p.dev == dev) {
      if (p.next >= p.ev.size()) die(where, "capture event pool exhausted");
      return p.ev[p.next++];
    }
  die(where, "no capture event pool for the device");
}
// before a capture: every device's pool holds at least `per` events not yet handed out
void fill_pools(int per, const char *where) {
  for (auto &s : g.sh) {
    bool have = false;
    for (auto &p : g.evPools) have = have || p.dev == s.dev;
    if (!have) g.evPools.push_back(FortranSide::EvPool{s.dev, {}, 0});
  }
  for (auto &p : g.evPools) {
    hipchk(hipSetDevice(p.dev), where);
    while (p.ev.size() < p.next + (size_t)per) {
      hipEvent_t e;
      hipchk(hipEventCreateWithFlags(&e, hipEventDisableTiming), where);
      p.ev.push_back(e);
    }
  }
}
bool multi() { return g.sh.size() > 1; }
long n2() { return (long)(g.dims[0] + 2 * g.dims[2]) * (g.dims[1] + 2 * g.dims[3]); }
long nTiles() { return (long)g.dims[5] * g.dims[6]; }

// every model runs fn (its own tiles; the r* passes every tile)
void run_all(const char *where, int (*fn)(mgcm_model *)) {
  for (size_t i = 0; i < g.sh.size(); i++) {
    auto &s = g.sh[i];
    cap_op(where, (int)i);
    hipchk(hipSetDevice(s.dev), where);
    if (fn(s.m)) die(where);
  }
  cap_op("(issued)", -1);
}
void phase_all(const char *where, int phase) {
  for (size_t i = 0; i < g.sh.size(); i++) {
    auto &s = g.sh[i];
    if (cap_dbg_on() && g.capturing) { fprintf(stderr, "MGCM_AMD   op %s phase %d model %zu\n", where, phase, i); fflush(stderr); }
    hipchk(hipSetDevice(s.dev), where);
    if (mgcm_step_phase(s.m, phase)) die(where);
  }
}

// Cross-model barrier on the device: every model's stream waits for the work every other
// model has issued so far (no host synchronisation).
void seg_boundary(const char *where);
__global__ void k_capture_join() {}
void barrier_all(const char *where) {
  if (!multi()) return;
  if (g.segMode) return seg_boundary(where);   // segmented capture: the barrier is a cut
  cap_op("barrier", -1);
  if (g.capturing && g.capMulti) {
    // captured across the models' streams: through model 0 -- it waits for every other model,
    // runs an empty kernel, and every other model waits for that.  The all-to-all form below,
    // captured over 4 or more streams, makes hipStreamEndCapture fault (SIGSEGV inside the HIP
    // runtime, ROCm 7.2) -- reproduced by tools/capture_repro.hip alone, with kernels only and
    // one barrier; fan-in, fan-out and this gather form capture and replay at 4 and 6 streams
    // (profiles/r06/cap_repro/)
    const Shard &s0 = g.sh[0];
    for (size_t i = 1; i < g.sh.size(); i++) {
      const Shard &s = g.sh[i];
      hipchk(hipSetDevice(s.dev), where);
      const hipEvent_t e = rec_event(s.dev, s.ev, where);
      hipchk(hipEventRecord(e, stream_of(s)), where);
      hipchk(hipSetDevice(s0.dev), where);
      hipchk(hipStreamWaitEvent(stream_of(s0), e, 0), where);
    }
    hipchk(hipSetDevice(s0.dev), where);
    hipLaunchKernelGGL(k_capture_join, dim3(1), dim3(64), 0, stream_of(s0));
    hipchk(hipGetLastError(), where);
    const hipEvent_t e0 = rec_event(s0.dev, s0.ev, where);
    hipchk(hipEventRecord(e0, stream_of(s0)), where);
    for (size_t i = 1; i < g.sh.size(); i++) {
      hipchk(hipSetDevice(g.sh[i].dev), where);
      hipchk(hipStreamWaitEvent(stream_of(g.sh[i]), e0, 0), where);
    }
    return;
  }
  std::vector<hipEvent_t> ev(g.sh.size());
  for (size_t i = 0; i < g.sh.size(); i++) {
    const Shard &s = g.sh[i];
    hipchk(hipSetDevice(s.dev), where);
    ev[i] = rec_event(s.dev, s.ev, where);
    hipchk(hipEventRecord(ev[i], stream_of(s)), where);
  }
  for (size_t i = 0; i < g.sh.size(); i++) {
    hipchk(hipSetDevice(g.sh[i].dev), where);
    for (size_t j = 0; j < g.sh.size(); j++)
      if (i != j) hipchk(hipStreamWaitEvent(stream_of(g.sh[i]), ev[j], 0), where);
  }
}

// The tile blocks [t0, t0+nT) of a 2-D field from model `from` to every other model.
void copy_blocks(const char *where, const char *name, int from, int t0, int nT) {
  cap_op(name, from);
  const Shard &a = g.sh[from];
  const long per = n2();
  const double *src = mgcm_device_ptr(a.m, name);
  if (!src) die(where);
  hipchk(hipSetDevice(a.dev), where);
  for (size_t j = 0; j < g.sh.size(); j++) {
    if ((int)j == from) continue;
    double *dst = mgcm_device_ptr(g.sh[j].m, name);
    if (!dst) die(where);
    hipchk(hipMemcpyAsync(dst + t0 * per, src + t0 * per, (size_t)nT * per * sizeof(double), hipMemcpyDeviceToDevice,
                          stream_of(a)),
           where);
  }
}
// GLOBAL all-gather of a 2-D field's tile blocks: every model's own tiles to every other model
void gather2d(const char *where, const char *name) {
  barrier_all(where);
  for (size_t i = 0; i < g.sh.size(); i++) copy_blocks(where, name, (int)i, g.sh[i].t0, g.sh[i].nT);
  barrier_all(where);
}

// The 3-D halo sources of a field group (mgcm_halo_pack_group: 0 all of
// DO_FIELDS_BLOCKING_EXCHANGES' fields) along every link: pack on the owner, copy GPU to GPU,
// unpack on the reader -- then each model's local halo fill reads them.  The barrier before
// keeps a link's receive buffer from being refilled while its reader still unpacks the
// previous transfer; after it, each reader's stream has waited for its own links' copies
// (per-link events) and needs nothing from the others.
void xfer3d(const char *where, int group) {
  barrier_all(where);
  cap_op("xfer3d", group);
  const int Nr = g.dims[4];
  if (g.segMode || (g.capturing && g.capMulti)) {
    // the senders' packs and copies, a cut (segmented capture) or a barrier through model 0
    // (multi-stream capture: per-link events over 6 streams -- each model waiting for its 4
    // cube neighbours -- fault the runtime's capture as the all-to-all barrier does), then the
    // receivers' unpacks
    for (auto &L : g.links) {
      const Shard &a = g.sh[L.s];
      const int nf = mgcm_exchange_nfields_group(a.m, group);
      if (nf <= 0) continue;
      hipchk(hipSetDevice(a.dev), where);
      if (mgcm_halo_pack_group(a.m, group, L.idxS, L.n, L.sbuf, 0)) die(where);
      hipchk(hipMemcpyAsync(L.rbuf, L.sbuf, (size_t)nf * Nr * L.n * sizeof(double), hipMemcpyDeviceToDevice,
                            stream_of(a)),
             where);
    }
    barrier_all(where);   // (a segment cut under segMode)
    for (auto &L : g.links) {
      const Shard &b = g.sh[L.d];
      const int nf = mgcm_exchange_nfields_group(b.m, group);
      if (nf <= 0) continue;
      hipchk(hipSetDevice(b.dev), where);
      if (mgcm_halo_pack_group(b.m, group, L.idxD, L.n, L.rbuf, 1)) die(where);
    }
    return;
  }
  for (auto &L : g.links) {
    const Shard &a = g.sh[L.s], &b = g.sh[L.d];
    const int nf = mgcm_exchange_nfields_group(a.m, group);
    if (nf <= 0) continue;
    hipchk(hipSetDevice(a.dev), where);
    if (mgcm_halo_pack_group(a.m, group, L.idxS, L.n, L.sbuf, 0)) die(where);
    hipchk(hipMemcpyAsync(L.rbuf, L.sbuf, (size_t)nf * Nr * L.n * sizeof(double), hipMemcpyDeviceToDevice,
                          stream_of(a)),
           where);
    const hipEvent_t le = rec_event(a.dev, L.ev, where);
    hipchk(hipEventRecord(le, stream_of(a)), where);
    hipchk(hipSetDevice(b.dev), where);
    hipchk(hipStreamWaitEvent(stream_of(b), le, 0), where);
    if (mgcm_halo_pack_group(b.m, group, L.idxD, L.n, L.rbuf, 1)) die(where);
  }
}

// ---- the device routines a drop-in runs (on every model, with the exchange points) ------
void op_oceanic_phys(const char *w) { run_all(w, mgcm_oceanic_phys); }
void op_tracer_step(const char *w) { run_all(w, mgcm_tracer_step); }
void op_dynamics(const char *w) { run_all(w, mgcm_dynamics); }
void op_update_r_star(const char *w) { run_all(w, mgcm_update_r_star); }
void op_calc_r_star(const char *w) { run_all(w, mgcm_calc_r_star); }
void op_correction(const char *w) { run_all(w, mgcm_momentum_correction_step); }
// SOLVE_FOR_PRESSURE: CALC_DIV_GHAT on the own tiles, the right-hand side and the first
// guess (cg2d_x = Bo_surf*etaN, set with it: solve_for_pressure.F:129,176-177) to every model,
// CG2D, EXCH(cg2d_x) + etaN everywhere
void op_solve(const char *w) {
  if (!multi()) return run_all(w, mgcm_solve_for_pressure);
  phase_all(w, 11);
  gather2d(w, "cg2d_b");
  gather2d(w, "cg2d_x");
  if (!g.cgDevice) {
    // the single-CU solve of the gathered domain + EXCH(cg2d_x) + etaN, once per GPU (its lead
    // model: every model of a GPU would solve the same problem to the same bits), the result
    // copied to that GPU's other models
    const size_t bytes = (size_t)n2() * nTiles() * sizeof(double);
    for (auto &c : g.cgLeads) {
      const Shard &L = g.sh[c.shard];
      hipchk(hipSetDevice(L.dev), w);
      if (mgcm_step_phase(L.m, 12)) die(w);
      for (size_t j = 0; j < g.sh.size(); j++) {
        if ((int)j == c.shard || g.sh[j].gpu != L.gpu) continue;
        for (const char *nm : {"cg2d_x", "etaN"}) {
          const double *src = mgcm_device_ptr(L.m, nm);
          double *dst = mgcm_device_ptr(g.sh[j].m, nm);
          if (!src || !dst) die(w);
          hipchk(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream_of(L)), w);
        }
      }
    }
    return barrier_all(w);
  }
  // the device CG2D: one launch per GPU over its models' tiles (its lead's arrays hold the
  // gathered right-hand side), all launches on one hand-off block; then each GPU's solution
  // blocks to every other model
  for (auto &c : g.cgLeads) {
    hipchk(hipSetDevice(g.sh[c.shard].dev), w);
    if (mgcm_cg2d_tiles(g.sh[c.shard].m, c.t0, c.nT)) die(w);
  }
  barrier_all(w);
  for (auto &c : g.cgLeads) copy_blocks(w, "cg2d_x", c.shard, c.t0, c.nT);
  barrier_all(w);
  phase_all(w, 13);
}
// INTEGR_CONTINUITY: the column pass on the own tiles, then (exactConserv) the new free
// surface's blocks to every model and EXCH(eta) + UPDATE_ETAH everywhere
void op_continuity(const char *w) {
  if (!multi()) return run_all(w, mgcm_integr_continuity);
  phase_all(w, 14);
  if (!g.exactConserv) return;
  gather2d(w, "cg2d_b");
  phase_all(w, 15);
}
// DO_FIELDS_BLOCKING_EXCHANGES: the halo sources between models, then every local fill
void op_blocking(const char *w) {
  if (multi()) xfer3d(w, 0);
  run_all(w, mgcm_blocking_exchanges);
}
// DO_STAGGER_FIELDS_EXCHANGES: the velocities' halo sources between models (group 2: the
// non-tracer fields), then every local uVel, vVel, wVel fill
void op_stagger(const char *w) {
  if (multi()) xfer3d(w, 2);
  run_all(w, mgcm_stagger_exchanges);
}

// The device's iteration counter (AB2's first step, the CD scheme's start), written only
// when it changes (FORWARD_STEP advances myIter after DYNAMICS, forward_step.F:806), in
// stream order: no host synchronisation.
void set_iter(const char *where, int myIter) {
  if (g.devIter == myIter) return;
  for (auto &s : g.sh) {
    hipchk(hipSetDevice(s.dev), where);
    // inside a capture the step's advance is an increment (the graph replays at any myIter)
    if (g.capturing ? mgcm_add_iter(s.m, myIter - (int)g.devIter) : mgcm_set_iter(s.m, myIter)) die(where);
  }
  g.devIter = myIter;
}

// kinds: bit k set = move the arrays of kind k (to every model: each holds the domain), as
// one staged batch per model in stream order (mgcm_put_batch_async: no host wait)
void upload(const char *where, unsigned kinds) {
  std::vector<std::vector<double>> tmp;
  std::vector<const char *> names;
  std::vector<const double *> src;
  std::vector<long> cnt;
  tmp.reserve(g.bound.size());
  for (auto &b : g.bound) {
    if (!((kinds >> b.kind) & 1u)) continue;
    const double *p = b.host;
    if (b.stride != 1) {
      tmp.emplace_back(b.count);
      for (long q = 0; q < b.count; q++) tmp.back()[q] = b.host[q * b.stride + b.off];
      p = tmp.back().data();
    }
    names.push_back(b.name.c_str());
    src.push_back(p);
    cnt.push_back(b.count);
    g.nUp++;
    g.bytesUp += 8.0 * b.count;
  }
  if (names.empty()) return;
  for (auto &s : g.sh) {
    hipchk(hipSetDevice(s.dev), where);
    if (mgcm_put_batch_async(s.m, (int)names.size(), names.data(), src.data(), cnt.data())) die(where);
  }
}

void sync_all(const char *where) {
  for (auto &s : g.sh)
    if (mgcm_sync(s.m)) die(where);
}

// The state arrays' pages registered for DMA (page-rounded, overlapping ranges merged): a
// download is then one copy engine transfer straight into the COMMON block instead of a
// staged copy.  A refusal leaves them unregistered (the copies still work, staged by HIP).
void register_host() {
  if (g.regTried) return;
  g.regTried = true;
  if (getenv("MGCM_AMD_REGISTER") && atoi(getenv("MGCM_AMD_REGISTER")) == 0) return;
  const uintptr_t pg = 4096;
  std::vector<std::pair<uintptr_t, uintptr_t>> iv;
  for (auto &b : g.bound)
    if (b.kind == 0) {
      const uintptr_t a = (uintptr_t)b.host, e = a + (uintptr_t)(b.count * b.stride) * sizeof(double);
      iv.push_back({a & ~(pg - 1), (e + pg - 1) & ~(pg - 1)});
    }
  std::sort(iv.begin(), iv.end());
  std::vector<std::pair<uintptr_t, uintptr_t>> merged;
  for (auto &r : iv)
    if (!merged.empty() && r.first <= merged.back().second) merged.back().second = std::max(merged.back().second, r.second);
    else merged.push_back(r);
  size_t done = 0;
  for (auto &r : merged) {
    if (hipHostRegister((void *)r.first, r.second - r.first, hipHostRegisterPortable) != hipSuccess) {
      (void)hipGetLastError();
      break;
    }
    done++;
  }
  size_t bytes = 0;
  for (auto &r : merged) bytes += r.second - r.first;
  if (done != merged.size()) {   // all or nothing
    for (size_t i = 0; i < done; i++) (void)hipHostUnregister((void *)merged[i].first);
    fprintf(stderr, "MGCM_AMD: state pages not registered (range %zu of %zu refused); downloads staged\n", done + 1,
            merged.size());
    return;
  }
  g.hostRegistered = true;
  std::vector<uintptr_t> lo, hi;
  for (auto &r : merged) { lo.push_back(r.first); hi.push_back(r.second); }
  mgcm::mg_host_ranges_set(lo.data(), hi.data(), merged.size());
  fprintf(stderr, "MGCM_AMD: state pages registered for DMA: %zu ranges, %.1f MB\n", merged.size(), bytes / 1e6);
}

// A solve that gave up -- a grid hand-off of the multi-workgroup CG2D timed out: numIters =
// -1, cg2d_x unconverged, and on a shared hand-off block the sharers' launch epochs may
// disagree from then on (model.hip, mwg_restart_epoch) -- stops the run, read where the host
// waits for the device anyway (a download, the step fence).  Each device-CG2D lead records
// its own launch.
void check_solve(const char *where) {
  auto chk = [&](mgcm_model *m) {
    int it = 0;
    if (mgcm_solve_stats(m, 0, nullptr, nullptr, &it, nullptr)) die(where);
    if (it < 0) die(where, "CG2D gave up: a grid hand-off of the multi-workgroup solve timed out (numIters = -1)");
  };
  if (multi() && g.cgDevice)
    for (auto &c : g.cgLeads) chk(g.sh[c.shard].m);
  else
    chk(g.m);
}

// The state down: a tiled array (2-D or 3-D, tile-major) block by block from each tile's
// owner, anything else (1-D profiles) from model 0.  Every copy is queued first (each
// model's stream, behind the step), then one wait.
void download(const char *where) {
  const long per2 = n2(), per3 = per2 * g.dims[4], nt = nTiles();
  if (g.strided.size() != g.bound.size()) g.strided.resize(g.bound.size());
  for (size_t i = 0; i < g.bound.size(); i++) {
    Bound &b = g.bound[i];
    if (b.kind != 0) continue;   // static and host-input arrays are never written on the device
    g.nDown++;
    g.bytesDown += 8.0 * b.count;
    const long per = b.count == per2 * nt ? per2 : b.count == per3 * nt ? per3 : 0;
    double *dst = b.host;
    if (b.stride != 1) {
      g.strided[i].resize(b.count);
      dst = g.strided[i].data();
    }
    if (multi() && per) {
      for (auto &s : g.sh) {
        const double *dp = mgcm_device_ptr(s.m, b.name.c_str());
        if (!dp) die(where);
        hipchk(hipSetDevice(s.dev), where);
        hipchk(mgcm::mg_host_copy(dst + s.t0 * per, dp + s.t0 * per, (size_t)s.nT * per * sizeof(double),
                                  hipMemcpyDeviceToHost, stream_of(s)),
               where);
      }
      continue;
    }
    const double *dp = mgcm_device_ptr(g.m, b.name.c_str());
    if (!dp) die(where);
    hipchk(hipSetDevice(g.sh[0].dev), where);
    hipchk(mgcm::mg_host_copy(dst, dp, (size_t)b.count * sizeof(double), hipMemcpyDeviceToHost, stream_of(g.sh[0])),
           where);
  }
  sync_all(where);
  check_solve(where);
  for (size_t i = 0; i < g.bound.size(); i++) {
    Bound &b = g.bound[i];
    if (b.kind != 0 || b.stride == 1) continue;
    for (long q = 0; q < b.count; q++) b.host[q * b.stride + b.off] = g.strided[i][q];
  }
}

constexpr unsigned K_STATE = 1u << 0, K_STATIC = 1u << 1, K_INPUT = 1u << 2;

// The time loop has begun (a routine only FORWARD_STEP calls): the host's state goes up
// once and the device copy becomes the authoritative one.
void enter_time_loop(const char *where) {
  if (g.deviceAuth) return;
  upload(where, K_STATE | K_INPUT);
  g.deviceAuth = true;
  register_host();
}

// One routine drop-in.  Host-authoritative (initialisation): state in, the device
// routine, state out.  Device-authoritative: the host input first when `input`.  myIter /
// myTime are the values the reference passes the routine; the device's counter (AB2's
// first-step rule, the CD scheme's start) is set to devIter when given (staggered
// THERMODYNAMICS lags only that index, temp_integrate.F:154-155).
constexpr int kNoIter = -2147483647 - 1;
void routine(const char *where, void (*op)(const char *), int myIter, double myTime, bool input = false,
             int devIter = kNoIter) {
  model(where);
  if (!g.ready) die(where, "called before MGCM_AMD_INIT");
  g.lastIter = myIter;
  g.lastTime = myTime;
  const int it = devIter == kNoIter ? myIter : devIter;
  if (!g.deviceAuth) {
    upload(where, K_STATE | K_INPUT);
    set_iter(where, it);
    op(where);
    download(where);
    return;
  }
  if (input) upload(where, K_INPUT);
  set_iter(where, it);
  op(where);
}

// Partition and wiring of N device models (MGCM_AMD_MODELS), after mgcm_init of each: tile
// ranges, the CG2D mode and its per-GPU leads, the halo-source links, the barrier events.
void setup_shards(const char *where) {
  const int N = (int)g.sh.size(), nt = (int)nTiles();
  const int base = nt / N, rem = nt % N;
  for (int i = 0, t = 0; i < N; i++) {
    Shard &s = g.sh[i];
    s.t0 = t;
    s.nT = base + (i < rem ? 1 : 0);
    t += s.nT;
    hipchk(hipSetDevice(s.dev), where);
    if (!s.ev) hipchk(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming), where);
    if (mgcm_set_tile_range(s.m, s.t0, s.nT)) die(where);
  }
  g.exactConserv = mgcm_get_param(g.m, "exactConserv") != 0.0;
  // CG2D: the multi-workgroup solver runs tile-sharded (one launch per GPU); a single-CU
  // kernel solves the gathered domain on every model
  g.cgDevice = mgcm_get_param(g.m, "cg2dKernel") == 4.0;
  g.cgLeads.clear();
  for (int i = 0; i < N; i++) {
    if (!g.cgLeads.empty() && g.sh[g.cgLeads.back().shard].gpu == g.sh[i].gpu) {
      g.cgLeads.back().nT += g.sh[i].nT;
      continue;
    }
    for (auto &c : g.cgLeads)
      if (g.sh[c.shard].gpu == g.sh[i].gpu) die(where, "the models of one GPU must own contiguous tiles (MGCM_AMD_DEVICES)");
    g.cgLeads.push_back(CgLead{i, g.sh[i].t0, g.sh[i].nT});
  }
  if (g.cgDevice && g.cgLeads.size() > 1)
    for (auto &c : g.cgLeads)
      if (mgcm_cg2d_share(g.sh[c.shard].m, g.sh[g.cgLeads[0].shard].m)) die(where);
  // peer access between the GPUs in use (device-to-device copies)
  for (auto &a : g.sh)
    for (auto &b : g.sh)
      if (a.dev != b.dev) {
        hipchk(hipSetDevice(a.dev), where);
        const hipError_t e = hipDeviceEnablePeerAccess(b.dev, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) die(where, hipGetErrorString(e));
        (void)hipGetLastError();
      }
  // links: for every model d, the sources its halos read in another model's tiles
  const int Nr = g.dims[4];
  int nfMax = 0;
  for (int grp = 0; grp < 3; grp++) nfMax = std::max(nfMax, mgcm_exchange_nfields_group(g.m, grp));
  const long per2 = n2();
  for (int d = 0; d < N; d++) {
    const Shard &sd = g.sh[d];
    const long cnt = mgcm_halo_sources(sd.m, sd.t0, sd.nT, nullptr, 0);
    if (cnt < 0) die(where);
    std::vector<long> src((size_t)cnt);
    if (cnt && mgcm_halo_sources(sd.m, sd.t0, sd.nT, src.data(), cnt) != cnt) die(where);
    for (int sIdx = 0; sIdx < N; sIdx++) {
      if (sIdx == d) continue;
      const Shard &ss = g.sh[sIdx];
      std::vector<long> mine;
      for (long v : src)
        if (v >= ss.t0 * per2 && v < (ss.t0 + ss.nT) * per2) mine.push_back(v);
      if (mine.empty()) continue;
      Link L;
      L.s = sIdx;
      L.d = d;
      L.n = (long)mine.size();
      const size_t ib = mine.size() * sizeof(long), bb = (size_t)std::max(1, nfMax) * Nr * mine.size() * sizeof(double);
      hipchk(hipSetDevice(ss.dev), where);
      hipchk(hipMalloc(&L.idxS, ib), where);
      hipchk(hipMalloc(&L.sbuf, bb), where);
      hipchk(hipMemcpy(L.idxS, mine.data(), ib, hipMemcpyHostToDevice), where);
      hipchk(hipEventCreateWithFlags(&L.ev, hipEventDisableTiming), where);
      hipchk(hipSetDevice(sd.dev), where);
      hipchk(hipMalloc(&L.idxD, ib), where);
      hipchk(hipMalloc(&L.rbuf, bb), where);
      hipchk(hipMemcpy(L.idxD, mine.data(), ib, hipMemcpyHostToDevice), where);
      g.links.push_back(L);
    }
  }
}

void free_links() {
  for (auto &L : g.links) {
    (void)hipSetDevice(g.sh[L.s].dev);
    (void)hipFree(L.idxS);
    (void)hipFree(L.sbuf);
    if (L.ev) (void)hipEventDestroy(L.ev);
    (void)hipSetDevice(g.sh[L.d].dev);
    (void)hipFree(L.idxD);
    (void)hipFree(L.rbuf);
  }
  g.links.clear();
  g.cgLeads.clear();
}
void seg_destroy(FortranSide::SegGraphs &S) {
  for (auto &v : S.seg)
    for (auto e : v)
      if (e) (void)hipGraphExecDestroy(e);
  S.seg.clear();
}
void free_shards() {
  free_links();
  for (auto &S : g.sgr) seg_destroy(S);
  for (auto &p : g.evPools) {
    (void)hipSetDevice(p.dev);
    for (auto e : p.ev) (void)hipEventDestroy(e);
  }
  g.evPools.clear();
  for (auto &s : g.sh) {
    if (s.ev) { (void)hipSetDevice(s.dev); (void)hipEventDestroy(s.ev); }
    if (s.m) mgcm_destroy(s.m);
  }
  g.sh.clear();
  g.m = nullptr;
}

// A drop-in FORWARD_STEP calls after it advances myIter / myTime (forward_step.F:806-807):
// the step's end time, for the host-reader test of DO_FIELDS_BLOCKING_EXCHANGES.
void advanced(int myIter, double myTime) {
  g.advValid = true;
  g.advIter = myIter;
  g.advTime = myTime;
}

// staggerTimeStep: THERMODYNAMICS after the pressure solve (forward_step.F:1003-1036)
bool staggered() { return mgcm_get_param(g.m, "staggerTimeStep") != 0.0; }

// Is the recorded step FORWARD_STEP's order, which mgcm_forward_step replays bit for bit
// (forward_step.F:656-1120; tests/test_gpu_refhost.py)?  Each routine once, in the order
// DO_OCEANIC_PHYS, THERMODYNAMICS, DYNAMICS, [UPDATE_R_STAR, UPDATE_CG2D],
// SOLVE_FOR_PRESSURE, MOMENTUM_CORRECTION_STEP, INTEGR_CONTINUITY, [CALC_R_STAR],
// DO_FIELDS_BLOCKING_EXCHANGES -- the bracketed ones iff the r* free surface -- or, under
// staggerTimeStep, THERMODYNAMICS moved after DO_STAGGER_FIELDS_EXCHANGES, which follows
// INTEGR_CONTINUITY / CALC_R_STAR.
bool canonical_step(const std::vector<std::string> &q) {
  const bool rstar = mgcm_get_param(g.m, "nonlinFreeSurf") > 0.0, st = staggered();
  if (mgcm_get_param(g.m, "momStepping") == 0.0) return false;
  std::vector<std::string> want = {"DO_OCEANIC_PHYS"};
  if (!st) want.push_back("THERMODYNAMICS");
  want.push_back("DYNAMICS");
  if (rstar) { want.push_back("UPDATE_R_STAR"); want.push_back("UPDATE_CG2D"); }
  want.push_back("SOLVE_FOR_PRESSURE");
  want.push_back("MOMENTUM_CORRECTION_STEP");
  want.push_back("INTEGR_CONTINUITY");
  if (rstar) want.push_back("CALC_R_STAR");
  if (st) { want.push_back("DO_STAGGER_FIELDS_EXCHANGES"); want.push_back("THERMODYNAMICS"); }
  want.push_back("DO_FIELDS_BLOCKING_EXCHANGES");
  return q == want;
}
// Replay: one model, N models on one GPU (captured onto one stream, multi_replay), or models
// over several GPUs (per-GPU segment graphs, seg_replay); MGCM_AMD_EAGER=1 steps routine by
// routine
bool fuse_allowed() {
  const char *e = getenv("MGCM_AMD_EAGER");
  if (e && atoi(e) == 1) return false;
  if (!multi()) return true;
  return !g.multiGraphOff;
}

// The device work of the recorded step's drop-ins, in their order, with the iteration
// counter advanced where FORWARD_STEP advances myIter (forward_step.F:806: every drop-in
// after DYNAMICS runs at myIter + 1 -- but THERMODYNAMICS, staggered or not, steps the
// tracers' Adams-Bashforth at the step's start, temp_integrate.F:154-155).
void run_recorded_step(const char *w, int myIter) {
  for (auto &nm : g.fusedSeq) {
    const bool late = nm != "DO_OCEANIC_PHYS" && nm != "THERMODYNAMICS" && nm != "DYNAMICS";
    set_iter(w, late ? myIter + 1 : myIter);
    if (nm == "DO_OCEANIC_PHYS") op_oceanic_phys(w);
    else if (nm == "THERMODYNAMICS") op_tracer_step(w);
    else if (nm == "DYNAMICS") op_dynamics(w);
    else if (nm == "UPDATE_R_STAR") op_update_r_star(w);
    else if (nm == "UPDATE_CG2D") continue;   // folded into UPDATE_R_STAR
    else if (nm == "SOLVE_FOR_PRESSURE") op_solve(w);
    else if (nm == "MOMENTUM_CORRECTION_STEP") op_correction(w);
    else if (nm == "INTEGR_CONTINUITY") op_continuity(w);
    else if (nm == "CALC_R_STAR") op_calc_r_star(w);
    else if (nm == "DO_STAGGER_FIELDS_EXCHANGES") op_stagger(w);
    else if (nm == "DO_FIELDS_BLOCKING_EXCHANGES") op_blocking(w);
    else die(w, "unknown drop-in in the recorded step");
  }
}

// model 0's stream waits for every other model's work so far (join), or every other model's
// stream for model 0's (fork)
void join_into_0(const char *w) {
  cap_op("join into model 0", -1);
  std::vector<hipEvent_t> ev(g.sh.size());
  for (size_t i = 1; i < g.sh.size(); i++) {
    hipchk(hipSetDevice(g.sh[i].dev), w);
    ev[i] = rec_event(g.sh[i].dev, g.sh[i].ev, w);
    hipchk(hipEventRecord(ev[i], stream_of(g.sh[i])), w);
  }
  hipchk(hipSetDevice(g.sh[0].dev), w);
  for (size_t i = 1; i < g.sh.size(); i++) hipchk(hipStreamWaitEvent(stream_of(g.sh[0]), ev[i], 0), w);
}
void fork_from_0(const char *w) {
  hipchk(hipSetDevice(g.sh[0].dev), w);
  const hipEvent_t e0 = rec_event(g.sh[0].dev, g.sh[0].ev, w);
  hipchk(hipEventRecord(e0, stream_of(g.sh[0])), w);
  for (size_t i = 1; i < g.sh.size(); i++) {
    hipchk(hipSetDevice(g.sh[i].dev), w);
    hipchk(hipStreamWaitEvent(stream_of(g.sh[i]), e0, 0), w);
  }
}

// One FORWARD_STEP of N device models (the recorded drop-in sequence) as a graph replay:
// the forcing goes up and myIter is set outside the graph; the graph of model 0's tracer
// parity is captured on first use -- every model's stream joins model 0's capture, the
// cross-model copies and event barriers of the ops become graph edges -- and launched; a
// replay then leaves every model at the parity its captured step's host-side CYCLE_TRACER
// swaps left (mgcm_tracer_parity).  false: the capture failed (the step then runs eagerly
// and later steps stay eager).
bool multi_replay(const char *w, int myIter) {
  const int q = mgcm_tracer_parity(g.m, -1);
  if (q < 0 || q > 3) die(w);
  auto &G = g.mg[q];
  std::vector<int> pre;
  for (auto &s : g.sh) pre.push_back(mgcm_tracer_parity(s.m, -1));
  join_into_0(w);   // the forcing uploads of every model before the graph
  if (!G.exec) {
    G.pre = pre;
    hipStream_t s0 = stream_of(g.sh[0]);
    // every model keeps its own stream in the capture (the graph then has a branch per model,
    // joined at the exchange points) from 4 models on, or with MGCM_AMD_CAPTURE=multi; else (or
    // with MGCM_AMD_CAPTURE=one) every model issues on model 0's stream.  Config 2's 36 tiles
    // over 60 steps (test_refhost_dropin_throughput): 4 models 0.76 against 1.42 ms/step, 6
    // models 1.35 against 3.40, 2 models 0.63 against 0.61 (profiles/r06/cap_repro/)
    const bool multiStream = cap_opt("multi") || (!cap_opt("one") && g.sh.size() >= 4);
    static const hipStreamCaptureMode mode = cap_opt("relaxed") ? hipStreamCaptureModeRelaxed : hipStreamCaptureModeGlobal;
    fill_pools(4096, w);
    // one stream: the graph is one chain of the models' work in the recorded order.  The
    // multi-stream form's barriers go through model 0 (barrier_all: the runtime's capture of an
    // all-to-all event barrier over 4 or more streams faults)
    if (!multiStream)
      for (size_t i = 1; i < g.sh.size(); i++)
        if (mgcm_set_stream(g.sh[i].m, s0)) die(w);
    hipchk(hipSetDevice(g.sh[0].dev), w);
    if (hipStreamBeginCapture(s0, mode) != hipSuccess) {
      (void)hipGetLastError();
      for (size_t i = 1; i < g.sh.size(); i++)
        if (mgcm_set_stream(g.sh[i].m, nullptr)) die(w);
      return false;
    }
    cap_dbg("begin capture", q);
    g.capturing = true;   // (the pool's events from here: the fork's record is the capture's first node)
    g.capMulti = multiStream;
    fork_from_0(w);
    g.devIter = myIter;   // the graph's increments are relative to this
    run_recorded_step(w, myIter);
    join_into_0(w);
    g.capturing = g.capMulti = false;
    cap_dbg("joined; ending capture", q);
    hipGraph_t gr = nullptr;
    hipchk(hipSetDevice(g.sh[0].dev), w);
    hipError_t e = hipStreamEndCapture(s0, &gr);
    cap_dbg("end capture", q);
    if (e == hipSuccess && cap_dbg_on()) {
      size_t nn = 0;
      (void)hipGraphGetNodes(gr, nullptr, &nn);
      fprintf(stderr, "MGCM_AMD capture[%d]: %zu nodes\n", q, nn);
    }
    if (e == hipSuccess) e = hipGraphInstantiate(&G.exec, gr, nullptr, nullptr, 0);
    cap_dbg("instantiated", q);
    if (gr) (void)hipGraphDestroy(gr);
    for (size_t i = 1; i < g.sh.size(); i++)   // each model back on its own stream
      if (mgcm_set_stream(g.sh[i].m, nullptr)) die(w);
    // the capture ran the step's host side (the CYCLE_TRACER swaps) without its device work:
    // nothing consistent to fall back to
    if (e != hipSuccess) die(w, hipGetErrorString(e));
    G.post.clear();
    for (auto &s : g.sh) G.post.push_back(mgcm_tracer_parity(s.m, -1));
  } else {
    // the graph holds the theta/salt buffer pointers of the parities it was captured at: every
    // model must start there (a model stepped apart -- eagerly -- would drift)
    if (pre != G.pre) die(w, "a device model's tracer parity differs from the captured step's");
    for (size_t i = 0; i < g.sh.size(); i++)
      if (mgcm_tracer_parity(g.sh[i].m, G.post[i]) < 0) die(w);
  }
  hipchk(hipSetDevice(g.sh[0].dev), w);
  cap_dbg("launch", q);
  hipchk(hipGraphLaunch(G.exec, stream_of(g.sh[0])), w);
  if (cap_dbg_on()) {
    hipchk(hipStreamSynchronize(stream_of(g.sh[0])), w);
    cap_dbg("replay done", q);
  }
  fork_from_0(w);   // every model's later work (downloads, the next step) after the graph
  g.devIter = -1;   // the graph advanced the counters: set again before the next use
  return true;
}
bool spans_gpus() {
  for (auto &s : g.sh)
    if (s.gpu != g.sh[0].gpu) return true;
  return false;
}
hipStream_t lead_stream(size_t j) { return stream_of(g.sh[g.cgLeads[j].shard]); }
int lead_dev(size_t j) { return g.sh[g.cgLeads[j].shard].dev; }
// open one capture per GPU group (Relaxed: several captures in flight on this thread)
void seg_begin(const char *w) {
  for (size_t j = 0; j < g.cgLeads.size(); j++) {
    hipchk(hipSetDevice(lead_dev(j)), w);
    if (hipStreamBeginCapture(lead_stream(j), hipStreamCaptureModeRelaxed) != hipSuccess) {
      (void)hipGetLastError();
      g.segFail = true;
    }
  }
}
// close every group's capture into the open segment's graphs.  A group with nothing captured
// since the last cut gets no graph (nothing launched); a segment empty on every group is
// dropped -- the barriers either side of it are then one (two cuts in a row: the barrier after
// one gather and the one before the next)
void seg_end(const char *w) {
  std::vector<hipGraphExec_t> cur(g.cgLeads.size(), nullptr);
  bool any = false;
  for (size_t j = 0; j < g.cgLeads.size(); j++) {
    hipchk(hipSetDevice(lead_dev(j)), w);
    hipGraph_t gr = nullptr;
    hipError_t e = hipStreamEndCapture(lead_stream(j), &gr);
    size_t nn = 0;
    if (e == hipSuccess) e = hipGraphGetNodes(gr, nullptr, &nn);
    if (e == hipSuccess && nn > 0) e = hipGraphInstantiate(&cur[j], gr, nullptr, nullptr, 0);
    if (gr) (void)hipGraphDestroy(gr);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      g.segFail = true;
    }
    any = any || nn > 0;
  }
  if (any) g.segAll.push_back(cur);
}
void seg_boundary(const char *w) {
  cap_op("segment cut", (int)g.segAll.size());
  seg_end(w);
  seg_begin(w);
}
// every group's lead stream waits for every other's work so far (between segments)
void group_barrier(const char *w) {
  const size_t G = g.cgLeads.size();
  for (size_t j = 0; j < G; j++) {
    hipchk(hipSetDevice(lead_dev(j)), w);
    hipchk(hipEventRecord(g.sh[g.cgLeads[j].shard].ev, lead_stream(j)), w);
  }
  for (size_t j = 0; j < G; j++) {
    hipchk(hipSetDevice(lead_dev(j)), w);
    for (size_t i = 0; i < G; i++)
      if (i != j) hipchk(hipStreamWaitEvent(lead_stream(j), g.sh[g.cgLeads[i].shard].ev, 0), w);
  }
}
// within each group: the lead stream after the group's models' own streams (join), or they
// after it (fork)
void group_join(const char *w, bool fork) {
  for (size_t j = 0; j < g.cgLeads.size(); j++) {
    const int L = g.cgLeads[j].shard;
    for (size_t i = 0; i < g.sh.size(); i++) {
      if ((int)i == L || g.sh[i].gpu != g.sh[L].gpu) continue;
      const Shard &from = fork ? g.sh[L] : g.sh[i], &to = fork ? g.sh[i] : g.sh[L];
      hipchk(hipSetDevice(from.dev), w);
      hipchk(hipEventRecord(from.ev, stream_of(from)), w);
      hipchk(hipSetDevice(to.dev), w);
      hipchk(hipStreamWaitEvent(stream_of(to), from.ev, 0), w);
    }
  }
}
// One FORWARD_STEP of models over several GPUs as per-GPU segment graphs (the recorded drop-in
// sequence, captured on first use per tracer-buffer parity of model 0).  false: the capture
// failed -- every model is put back at the tracer parity it had, and this and later steps run
// routine by routine.
bool seg_replay(const char *w, int myIter) {
  const int q = mgcm_tracer_parity(g.m, -1);
  if (q < 0 || q > 3) die(w);
  auto &S = g.sgr[q];
  std::vector<int> pre;
  for (auto &s : g.sh) pre.push_back(mgcm_tracer_parity(s.m, -1));
  const size_t G = g.cgLeads.size();
  group_join(w, false);   // the forcing uploads of every model before its group's graphs
  group_barrier(w);       // and the previous step's work of every group
  if (S.seg.empty()) {
    S.pre = pre;
    for (size_t i = 0; i < g.sh.size(); i++) {   // every model issues on its group's lead stream
      const int L = g.cgLeads[0].shard;
      (void)L;
      for (size_t j = 0; j < G; j++)
        if (g.sh[g.cgLeads[j].shard].gpu == g.sh[i].gpu && (int)i != g.cgLeads[j].shard)
          if (mgcm_set_stream(g.sh[i].m, lead_stream(j))) die(w);
    }
    g.segAll.clear();
    g.segFail = false;
    cap_dbg("begin segmented capture", q);
    seg_begin(w);
    g.capturing = g.segMode = true;
    g.devIter = myIter;
    if (!g.segFail) run_recorded_step(w, myIter);
    g.capturing = g.segMode = false;
    seg_end(w);
    for (size_t i = 0; i < g.sh.size(); i++)   // each model back on its own stream
      if (mgcm_set_stream(g.sh[i].m, nullptr)) die(w);
    if (g.segFail) {
      for (auto &v : g.segAll)
        for (auto e : v)
          if (e) (void)hipGraphExecDestroy(e);
      g.segAll.clear();
      for (size_t i = 0; i < g.sh.size(); i++)
        if (mgcm_tracer_parity(g.sh[i].m, pre[i]) < 0) die(w);
      g.devIter = -1;
      return false;
    }
    S.seg = g.segAll;
    g.segAll.clear();
    S.post.clear();
    for (auto &s : g.sh) S.post.push_back(mgcm_tracer_parity(s.m, -1));
    if (cap_dbg_on()) fprintf(stderr, "MGCM_AMD capture[%d]: %zu segments x %zu GPUs\n", q, S.seg.size(), G);
  } else {
    if (pre != S.pre) die(w, "a device model's tracer parity differs from the captured step's");
    for (size_t i = 0; i < g.sh.size(); i++)
      if (mgcm_tracer_parity(g.sh[i].m, S.post[i]) < 0) die(w);
  }
  for (size_t k = 0; k < S.seg.size(); k++) {
    if (k > 0) group_barrier(w);
    for (size_t j = 0; j < G; j++) {
      if (!S.seg[k][j]) continue;   // nothing of this GPU's in the segment
      hipchk(hipSetDevice(lead_dev(j)), w);
      hipchk(hipGraphLaunch(S.seg[k][j], lead_stream(j)), w);
    }
  }
  group_barrier(w);
  group_join(w, true);   // every model's later work (downloads, the next step) after the graphs
  g.devIter = -1;
  return true;
}
// A routine drop-in of a device-authoritative step: true when its work already ran inside
// the step's replay (then it only checks its place in the recorded order).
bool absorbed(const char *name) {
  if (!g.fused) {
    if (g.recording) g.seq.push_back(name);
    return false;
  }
  if (g.fusedPos >= g.fusedSeq.size() || g.fusedSeq[g.fusedPos] != name) {
    fprintf(stderr, "ABNORMAL END: %s_AMD: the step's drop-ins left the recorded FORWARD_STEP order while the step "
                    "ran as one graph replay (MGCM_AMD_EAGER=1 steps routine by routine)\n", name);
    abort();
  }
  g.fusedPos++;
  return true;
}

// eesupp/src/different_multiple.F: is val1 the step nearest to a multiple of freq?
bool different_multiple(double freq, double val1, double step) {
  if (freq == 0.0) return false;
  if (fabs(step) > freq) return true;
  const double v1 = val1, v2 = val1 - step, v3 = val1 + step;
  const double v4 = round(v1 / freq) * freq;   // NINT: half away from zero
  const double d1 = v1 - v4, d2 = v2 - v4, d3 = v3 - v4;
  return fabs(d1) < fabs(d2) && fabs(d1) <= fabs(d3);
}

// Does a host routine read the state at the end of this step?  MONITOR
// (monitor.F:48), DO_THE_MODEL_IO (do_the_model_io.F:106), DO_WRITE_PICKUP
// (do_write_pickup.F:61-63, modelEnd) -- a superset is harmless, a miss is not.
bool host_reads_state(double myTime, int myIter) {
  const Readers &r = g.rd;
  return r.everyStep || myIter == r.nEndIter || different_multiple(r.monitorFreq, myTime, r.deltaTClock) ||
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
 * process and thread: the MPI decomposition of eesupp is not taken over, SURVEY.md 8(b)
 * "Threading"; the tiles go over GPUs inside the process instead: MGCM_AMD_MODELS device
 * models, see the top of this file).  Re-creates the models when the sizes change. */
void mgcm_amd_setup_(const int *sNx, const int *sNy, const int *OLx, const int *OLy, const int *Nr, const int *nSx,
                     const int *nSy, const int *nProcs, const int *nThreads) {
  if (*nProcs != 1 || *nThreads != 1)
    die("MGCM_AMD_SETUP", "the drop-ins need nPx*nPy = nTx*nTy = 1 (tiles go over GPUs by MGCM_AMD_MODELS)");
  const int d[7] = {*sNx, *sNy, *OLx, *OLy, *Nr, *nSx, *nSy};
  if (g.m && memcmp(d, g.dims, sizeof d) == 0) return;
  if (g.m) free_shards();
  g = FortranSide{};
  const int nt = d[5] * d[6];
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) die("MGCM_AMD_SETUP", "no HIP device");
  int N = 1;
  if (const char *e = getenv("MGCM_AMD_MODELS")) N = strcmp(e, "auto") == 0 ? std::min(nt, ndev) : atoi(e);
  if (N < 1 || N > nt) die("MGCM_AMD_SETUP", "MGCM_AMD_MODELS must be 1 .. the number of tiles (or auto)");
  std::vector<int> devs((size_t)N);
  for (int i = 0; i < N; i++) devs[i] = (int)(((long)i * ndev) / N);   // contiguous blocks of models per GPU
  // MGCM_AMD_DEVICES=virtual[:ids] (test hook): the GPU ids are logical -- every model runs on
  // device 0, but the models are grouped, sharded, solved and stepped exactly as on that many
  // GPUs (per-GPU CG2D leads, cross-GPU copies, the multi-GPU step and its segment graphs), so
  // the code an 8-GPU node runs is exercised on one; "virtual" alone: one GPU per model
  const char *dv = getenv("MGCM_AMD_DEVICES");
  const bool virt = dv && !strncmp(dv, "virtual", 7);
  if (virt) {
    for (int i = 0; i < N; i++) devs[i] = i;
    dv = dv[7] == ':' ? dv + 8 : nullptr;
  }
  if (const char *e = dv) {
    std::string l(e);
    size_t pos = 0;
    for (int i = 0; i < N; i++) {
      if (pos > l.size()) die("MGCM_AMD_SETUP", "MGCM_AMD_DEVICES: one GPU per model (comma separated)");
      const size_t c = l.find(',', pos);
      devs[i] = atoi(l.substr(pos, c == std::string::npos ? std::string::npos : c - pos).c_str());
      pos = c == std::string::npos ? l.size() + 1 : c + 1;
      if (devs[i] < 0 || (!virt && devs[i] >= ndev)) die("MGCM_AMD_SETUP", "MGCM_AMD_DEVICES names a GPU that does not exist");
    }
  }
  for (int i = 0; i < N; i++) {
    Shard s;
    s.gpu = devs[i];
    s.dev = virt ? 0 : devs[i];
    s.m = mgcm_create(d[0], d[1], d[2], d[3], d[4], d[5], d[6], s.dev);
    if (!s.m) die("MGCM_AMD_SETUP");
    s.nT = nt;
    g.sh.push_back(s);
  }
  g.m = g.sh[0].m;
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
  for (auto &s : g.sh) {
    if (mgcm_set_halo_map(s.m, src.data(), n)) die("MGCM_AMD_SET_MAPS");
    if (mgcm_set_uv_map(s.m, cu1.data(), cv1.data(), cu0.data(), cv0.data(), tFace, tEdge, n)) die("MGCM_AMD_SET_MAPS");
  }
  g.ready = false;
}

/* The halo maps of a pkg/exch2 topology from the W2_EXCH2_TOPOLOGY.h arrays
 * (mods/mgcm_amd_exch2.F; the derivation: exch2_maps.hip), set on every device model with
 * the tile faces and facet-edge flags (N=1 S=2 E=4 W=8) of the cube-corner vorticity. */
void mgcm_amd_set_w2_(const int *nTilesW2, const int *ldNb, const int *ldT, const int *myFace, const int *tBasex,
                      const int *tBasey, const int *isN, const int *isS, const int *isE, const int *isW, const int *nNb,
                      const int *nbId, const int *opp, const int *pij, const int *oi, const int *oj, const int *iLo,
                      const int *iHi, const int *jLo, const int *jHi, const int *useCS) {
  model("MGCM_AMD_SET_W2");
  const int nt = *nTilesW2;
  if (nt != (int)nTiles()) die("MGCM_AMD_SET_W2", "exch2_nTiles differs from nSx*nSy");
  const long n = (long)nt * n2();
  std::vector<long> src(n), cu1(n), cv1(n), cu0(n), cv0(n);
  if (mgcm_exch2_maps(g.dims[0], g.dims[1], g.dims[2], nt, *ldNb, *ldT, tBasex, tBasey, isN, isS, isE, isW, nNb, nbId,
                      opp, pij, oi, oj, iLo, iHi, jLo, jHi, *useCS != 0, src.data(), cu1.data(), cv1.data(), cu0.data(),
                      cv0.data()))
    die("MGCM_AMD_SET_W2", "inconsistent W2_EXCH2_TOPOLOGY arrays");
  std::vector<int> face(nt), edge(nt);
  for (int t = 0; t < nt; t++) {
    face[t] = myFace[t];
    edge[t] = isN[t] + 2 * isS[t] + 4 * isE[t] + 8 * isW[t];
  }
  for (auto &s : g.sh) {
    if (mgcm_set_halo_map(s.m, src.data(), n)) die("MGCM_AMD_SET_W2");
    if (mgcm_set_uv_map(s.m, cu1.data(), cv1.data(), cu0.data(), cv0.data(), face.data(), edge.data(), n))
      die("MGCM_AMD_SET_W2");
  }
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
  if (n == "useSBO") { r.everyStep = r.everyStep || *value != 0.0; return; }
  if (n == "useDiagnostics") {
    if (*value == 0.0) return;
    // DO_STATEVARS_DIAGS (forward_step.F:513) reads the state each step; the fills inside the
    // shadowed routines (DYNAMICS, THERMODYNAMICS, DO_OCEANIC_PHYS) are not made on the device
    const char *e = getenv("MGCM_AMD_DIAGNOSTICS");
    if (!e || strcmp(e, "state") != 0)
      die("MGCM_AMD_PARAM", "useDiagnostics: the device routines do not fill diagnostics (set "
                            "MGCM_AMD_DIAGNOSTICS=state for the state variables only, downloaded every step)");
    fprintf(stderr, "MGCM_AMD: useDiagnostics with MGCM_AMD_DIAGNOSTICS=state: state diagnostics only, "
                    "the state comes down after every step\n");
    r.everyStep = true;
    return;
  }
  if (n == "deltaTClock") r.deltaTClock = *value;
  for (auto &s : g.sh)
    if (mgcm_set_param(s.m, n.c_str(), *value)) die("MGCM_AMD_PARAM");
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
  install_fault_report();
  // device options with no PARAMS.h counterpart, from the environment:
  // MGCM_CG2D_REFORDER=1 sums CG2D in the reference's order (cg2dRefOrder, parity runs)
  // (several models: each is set up on the whole domain -- the CG2D tables too -- and only
  // then restricted to its tiles, setup_shards)
  free_links();
  for (auto &s : g.sh) {
    if (const char *e = getenv("MGCM_CG2D_REFORDER"))
      if (mgcm_set_param(s.m, "cg2dRefOrder", atof(e))) die("MGCM_AMD_INIT");
    // MGCM_CG2D_MWG=1: the multi-workgroup CG2D where a single-CU kernel would solve (the
    // device-sharded solve on a small grid: tests, rehearsals)
    if (const char *e = getenv("MGCM_CG2D_MWG"))
      if (mgcm_set_param(s.m, "cg2dForceMwg", atof(e))) die("MGCM_AMD_INIT");
    if (multi() && mgcm_set_tile_range(s.m, 0, (int)nTiles())) die("MGCM_AMD_INIT");
  }
  upload("MGCM_AMD_INIT", K_STATIC | K_STATE | K_INPUT);
  for (auto &s : g.sh) {
    if (mgcm_set_param(s.m, "myIter", (double)*myIter)) die("MGCM_AMD_INIT");
    if (mgcm_init(s.m)) die("MGCM_AMD_INIT");
  }
  upload("MGCM_AMD_INIT", K_STATE | K_INPUT);
  for (auto &s : g.sh)
    if (mgcm_set_param(s.m, "myIter", (double)*myIter)) die("MGCM_AMD_INIT");
  if (multi()) setup_shards("MGCM_AMD_INIT");
  g.canFuse = g.fused = g.recording = false;   // the step is learned again
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
  model("MGCM_AMD_STEP_FENCE");
  static const bool off = getenv("MGCM_AMD_STEP_FENCE") && atoi(getenv("MGCM_AMD_STEP_FENCE")) == 0;
  if (off) return;   // per-step times then measure the host's side (the steps pipeline)
  sync_all("MGCM_AMD_STEP_FENCE");
  static unsigned nFence = 0;
  if ((nFence++ & 7u) == 0) check_solve("MGCM_AMD_STEP_FENCE");   // every 8th fence (one small copy)
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
  g.advValid = false;   // a new step: its end time is not known yet
  if (g.fused) die("DO_OCEANIC_PHYS_AMD", "a step began before the previous one's DO_FIELDS_BLOCKING_EXCHANGES");
  if (g.canFuse && fuse_allowed() && g.ready) {
    // the whole step as one replay of the captured FORWARD_STEP (mgcm_forward_step; with N
    // models multi_replay), after this step's forcing; the counter the device advances at the
    // step's end is known
    g.lastIter = *myIter;
    g.lastTime = *myTime;
    upload("DO_OCEANIC_PHYS_AMD", K_INPUT);
    set_iter("DO_OCEANIC_PHYS_AMD", *myIter);
    bool replayed = true;
    if (multi()) {
      replayed = spans_gpus() ? seg_replay("DO_OCEANIC_PHYS_AMD", *myIter) : multi_replay("DO_OCEANIC_PHYS_AMD", *myIter);
      if (!replayed) {   // the stream refused the capture: stay eager
        fprintf(stderr, "MGCM_AMD: stream capture of the %zu-model step refused; steps run routine by routine\n",
                g.sh.size());
        g.multiGraphOff = true;
      }
    } else {
      if (mgcm_forward_step(g.m, 1)) die("DO_OCEANIC_PHYS_AMD");
      g.devIter = *myIter + 1;
    }
    if (replayed) {
      g.fused = true;
      g.fusedPos = 1;
      return;
    }
  }
  g.seq.assign(1, "DO_OCEANIC_PHYS");
  g.recording = g.deviceAuth && fuse_allowed();
  routine("DO_OCEANIC_PHYS_AMD", op_oceanic_phys, *myIter, *myTime, true);
}
/* SUBROUTINE THERMODYNAMICS(myTime, myIter, myThid)      model/src/thermodynamics.F:25
 * Under staggerTimeStep FORWARD_STEP calls it after advancing myIter (forward_step.F:806,
 * 1032) and TEMP/SALT_INTEGRATE step the Adams-Bashforth terms at iterNb = myIter - 1
 * (temp_integrate.F:154-155) while everything else keeps the advanced myIter / myTime
 * (temp_integrate.F:275-543): only the device's AB counter is lagged, to the step's start.
 * The advanced values are the step's end, as after forward_step.F:806. */
void thermodynamics_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  enter_time_loop("THERMODYNAMICS_AMD");
  const bool late = staggered();
  if (late) advanced(*myIter, *myTime);
  if (absorbed("THERMODYNAMICS")) return;
  routine("THERMODYNAMICS_AMD", op_tracer_step, *myIter, *myTime, false, late ? *myIter - 1 : kNoIter);
}
/* SUBROUTINE DYNAMICS(myTime, myIter, myThid)            model/src/dynamics.F:21 */
void dynamics_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  enter_time_loop("DYNAMICS_AMD");
  if (absorbed("DYNAMICS")) return;
  routine("DYNAMICS_AMD", op_dynamics, *myIter, *myTime);
}
/* SUBROUTINE UPDATE_R_STAR(useLatest, myTime, myIter, myThid)   model/src/update_r_star.F:6
 * useLatest = .TRUE. (forward_step.F:838): the new r* factors and hFac, and UPDATE_CG2D's
 * operator (update_cg2d.F:7, forward_step.F:868) with them -- one device pass.
 * useLatest = .FALSE. (RESET_NLFS_VARS + UPDATE_R_STAR at the start of the step,
 * forward_step.F:469-477) restores the hFac of the previous step's end, which the mirror
 * already holds: nothing to do. */
void update_r_star_amd_(const int *useLatest, const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  if (*useLatest) {
    advanced(*myIter, *myTime);
    if (absorbed("UPDATE_R_STAR")) return;
    routine("UPDATE_R_STAR_AMD", op_update_r_star, *myIter, *myTime);
  }
}
/* SUBROUTINE UPDATE_CG2D(myTime, myIter, myThid)         model/src/update_cg2d.F:7
 * Folded into UPDATE_R_STAR_AMD(.TRUE.), which FORWARD_STEP calls just before it. */
void update_cg2d_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myTime; (void)myIter; (void)myThid;
  model("UPDATE_CG2D_AMD");
  (void)absorbed("UPDATE_CG2D");
}
/* SUBROUTINE CALC_R_STAR(etaFld, myTime, myIter, myThid)  model/src/calc_r_star.F:10
 * FORWARD_STEP passes etaH (forward_step.F:976): the bound array. */
void calc_r_star_amd_(const double *etaFld, const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  const Bound *b = bound_at(etaFld);
  if (!b || b->name != "etaH") die("CALC_R_STAR_AMD", "etaFld must be the bound etaH");
  advanced(*myIter, *myTime);
  if (absorbed("CALC_R_STAR")) return;
  routine("CALC_R_STAR_AMD", op_calc_r_star, *myIter, *myTime);
}
/* SUBROUTINE SOLVE_FOR_PRESSURE(myTime, myIter, myThid)  model/src/solve_for_pressure.F:7 */
void solve_for_pressure_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  advanced(*myIter, *myTime);
  if (absorbed("SOLVE_FOR_PRESSURE")) return;
  routine("SOLVE_FOR_PRESSURE_AMD", op_solve, *myIter, *myTime);
}
/* SUBROUTINE MOMENTUM_CORRECTION_STEP(myTime, myIter, myThid)
 *                                                   model/src/momentum_correction_step.F:7 */
void momentum_correction_step_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  advanced(*myIter, *myTime);
  if (absorbed("MOMENTUM_CORRECTION_STEP")) return;
  routine("MOMENTUM_CORRECTION_STEP_AMD", op_correction, *myIter, *myTime);
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
  advanced(*myIter, *myTime);
  if (absorbed("INTEGR_CONTINUITY")) return;
  routine("INTEGR_CONTINUITY_AMD", op_continuity, *myIter, *myTime);
}
/* SUBROUTINE DO_FIELDS_BLOCKING_EXCHANGES(myThid)   model/src/do_fields_blocking_exchanges.F:7 */
/* The last device routine of a step: the state comes down when a host routine reads it
 * next (MONITOR / DO_THE_MODEL_IO / DO_WRITE_PICKUP at this step's end time: the advanced
 * myTime / myIter of the step's drop-ins after forward_step.F:806, or, when none of them ran
 * -- momStepping and calc_wVelocity both off -- one deltaTClock past the step's start). */
void do_fields_blocking_exchanges_amd_(const int *myThid) {
  (void)myThid;
  const int it = g.advValid ? g.advIter : g.lastIter + 1;
  const double t = g.advValid ? g.advTime : g.lastTime + g.rd.deltaTClock;
  if (absorbed("DO_FIELDS_BLOCKING_EXCHANGES")) {
    if (g.fusedPos != g.fusedSeq.size()) die("DO_FIELDS_BLOCKING_EXCHANGES_AMD", "drop-ins of the replayed step missing");
    g.fused = false;
    g.lastIter = it;
    g.lastTime = t;
  } else {
    routine("DO_FIELDS_BLOCKING_EXCHANGES_AMD", op_blocking, it, t);
    // a step that ran routine by routine in FORWARD_STEP's order: later ones replay it
    if (g.recording && canonical_step(g.seq)) {
      g.fusedSeq = g.seq;
      g.canFuse = true;
    }
    g.recording = false;
  }
  if (g.deviceAuth && host_reads_state(t, it)) download("DO_FIELDS_BLOCKING_EXCHANGES_AMD");
}

/* SUBROUTINE DO_STAGGER_FIELDS_EXCHANGES(myTime, myIter, myThid)
 *                                            model/src/do_stagger_fields_exchanges.F:7
 * staggerTimeStep (forward_step.F:1010): the new uVel, vVel, wVel exchanged before the
 * staggered THERMODYNAMICS reads them. */
void do_stagger_fields_exchanges_amd_(const double *myTime, const int *myIter, const int *myThid) {
  (void)myThid;
  model("DO_STAGGER_FIELDS_EXCHANGES_AMD");
  if (!staggered()) return;   // do_stagger_fields_exchanges.F:37 (implicitIntGravWave: refused)
  advanced(*myIter, *myTime);
  if (absorbed("DO_STAGGER_FIELDS_EXCHANGES")) return;
  routine("DO_STAGGER_FIELDS_EXCHANGES_AMD", op_stagger, *myIter, *myTime);
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
