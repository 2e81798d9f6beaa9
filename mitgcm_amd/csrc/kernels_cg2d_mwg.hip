// kernels_cg2d_mwg.hip -- CG2D (model/src/cg2d.F:13-415) as one persistent multi-workgroup
// launch, for solves that do not fit one CU: the cube's 6 faces (6 144 points), the LLC
// facets (105 300 points), anything past the single-workgroup kernels' 4 096 / 8 192.
//
// Decomposition.  Every tile is cut into parts (row strips) of <= OPT*NT points; one
// workgroup owns one part (mgcm_model::mwg, built by build_mwg in model.hip).  A thread
// holds OPT owned points: x, r, s, q and their 10 operator coefficients in VGPRs; r and s
// of the part live in LDS.  The points of the neighbouring parts that the stencils reach
// form two rings around the part:
//   ring 1 = neighbours of owned points (through the halo map, EXCH_S3D_RL's copies),
//   ring 2 = neighbours of ring-1 points.
// A thread also holds RPT ring-1 points, for which the workgroup recomputes r redundantly
// (r -= alpha*A s needs s on rings 1 and 2): the owner and the neighbour evaluate the same
// expression on the same bytes, so the copies stay bit-identical and the exchange of r that
// cg2d.F does after each update (EXCH_S3D_RL(cg2d_r), :337) needs no synchronisation.
//
// Per iteration two grid-wide hand-offs, each in the data-is-the-flag form (Guideline 16,
// R2): every handed-off f64 travels as two 8-byte granules {tag, half}, each written by ONE
// relaxed agent-scope (sc1) store; a consumer re-reads its granules (relaxed, sc1) until every
// tag equals the phase number.  No counter, no drain, no fence: one fabric round trip per
// hand-off instead of a store-drain, an atomic add, a poll and a load.  Tags restart at 1 in
// each launch (the hand-off block is zeroed before it); partials alternate between two
// buffers (a part can run at most one phase ahead of the slowest reader):
//   sync B  partials of (r,r) of iteration n and (M r, r) of n+1 (the reference's err_sq and
//           eta_qrN, reduced together: same values, cg2d.F:211-243, 321-337), and the
//           q = M r of the owned points other parts' rings hold;
//   sync D  partials of (s, A s) -> alpha (cg2d.F:268-301).
// EXCH_S3D_RL(cg2d_s) (cg2d.F:260) needs no hand-off of its own: a part keeps the s of its
// rings and updates them itself, s = q + beta*s with the q imported at sync B -- the
// owner's expression on the owner's bytes, so the ring copies stay bit-identical.
// Global sums in a fixed order, independent of placement and of how many GPUs share the
// tiles: thread partials (OPT terms in order) -> pairwise tree over the NT threads -> per
// workgroup partial; lane l of every wave adds partials l, l+64, ... in order, then the
// pairwise tree over the 64 lanes.  mgcm_cg2d_sum_plan exports it for the oracle.
#include "common.h"

namespace mgcm {

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
// SYS: the hand-off block is shared with other processes' launches (the tile-sharded
// device CG2D, parallel.py cg2d="device"; mapped by IPC, possibly on a peer GPU): every
// granule access at system scope
#define RLX_SCOPE(SYS) __ATOMIC_RELAXED, ((SYS) ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT)

// ---- DPP sums (the same operations as kernels_solve.hip's block reductions) ----
template <int CTRL>
__device__ __forceinline__ double mw_dpp(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double mw_bcast(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), CTRL, ROWMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWMASK, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double mw_lane(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double mw_row16(double v) {
  v = v + mw_dpp<0xB1>(v);
  v = v + mw_dpp<0x4E>(v);
  v = v + mw_dpp<0x141>(v);
  v = v + mw_dpp<0x140>(v);
  return v;
}
__device__ __forceinline__ double mw_rowmax16(double v) {
  v = fmax(v, mw_dpp<0xB1>(v));
  v = fmax(v, mw_dpp<0x4E>(v));
  v = fmax(v, mw_dpp<0x141>(v));
  v = fmax(v, mw_dpp<0x140>(v));
  return v;
}
// pairwise tree over the 64 lanes, uniform result
__device__ __forceinline__ double mw_wave_sum(double v) {
  v = mw_row16(v);
  v = v + mw_bcast<0x142, 0xA>(v);
  v = v + mw_bcast<0x143, 0xC>(v);
  return mw_lane(v, 63);
}
__device__ __forceinline__ double mw_wave_max(double v) {
  v = mw_rowmax16(v);
  return fmax(fmax(mw_lane(v, 0), mw_lane(v, 16)), fmax(mw_lane(v, 32), mw_lane(v, 48)));
}

// workgroup geometry: NT threads x OPT points per thread = 1024 points per part.  Swept with
// tools/mwg_geom_ab.sh (profiles/r02/mwg_geometry.txt): 1024 x 1 (16 waves, 104 VGPRs) hides
// the hand-off and LDS latencies best -- 4.25 / 7.39 us per iteration on cs32x15 / LLC-90
// against 6.02 / 8.70 for 256 x 4; the MGCM_MW_* macros build the other variants
#ifndef MGCM_MW_NT
#define MGCM_MW_NT 1024
#endif
#ifndef MGCM_MW_OPT
#define MGCM_MW_OPT 1
#endif
constexpr int MW_NT = MGCM_MW_NT, MW_OPT = MGCM_MW_OPT, MW_RPT = 1, MW_NW = MW_NT / 64;
constexpr int MW_NV = 3;   // values per reduction

// ---- granule hand-offs (Guideline 16 R2) -------------------------------------------
template <bool SYS = false>
__device__ __forceinline__ void gran_put(gu64 *g, unsigned tag, double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v), t = (unsigned long long)tag << 32;
  __hip_atomic_store(g, t | (b & 0xffffffffull), RLX_SCOPE(SYS));
  __hip_atomic_store(g + 1, t | (b >> 32), RLX_SCOPE(SYS));
}
template <bool SYS = false>
__device__ __forceinline__ bool gran_get(gu64 *g, unsigned tag, double &v) {
  const unsigned long long lo = __hip_atomic_load(g, RLX_SCOPE(SYS)), hi = __hip_atomic_load(g + 1, RLX_SCOPE(SYS));
  v = __builtin_bit_cast(double, ((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull));
  return (unsigned)(lo >> 32) == tag && (unsigned)(hi >> 32) == tag;
}
// Launch epochs: each process keeps its own epoch word (T.epoch, never shared), read by its
// parts at their start and advanced by its launch's first part g0 after the last hand-off
// (every part of the solve has read its epoch by then: g0's last hand-off needs every part's
// partial).  Every process launches the same solves in the same order, so the epochs agree
// without any process reading another's counter (a shared counter advanced by one process
// could be read stale by a process whose next launch starts first).  A granule's tag is
// (epoch mod 2^16) << 16 | phase, so no memset is needed between launches.  The timeout word
// ctr[1] (shared) holds epoch + 1 of a launch that gave up (the epoch then advances by 2).
__device__ __forceinline__ unsigned mw_tag(unsigned ep, int phase) { return ((ep & 0xffffu) << 16) | (unsigned)phase; }
// bounded spin: after ~2^22 passes every part gives up (timeout word), so no wave hangs.
// The timeout word is read every MGCM_MW_TMO_EVERY-th pass only: read every pass, its load
// (a second memory round trip behind the granule loads) doubled each poll's period.
// MGCM_MW_SLEEP: the s_sleep argument between passes (0: none): 2 by default -- cs32x15's
// one-XCD parts 4.13 against 4.22 us/iteration at 1 and worse at 0, LLC-90 unchanged
// (6.12 against 6.02-6.19), 4 slower there (profiles/r04/mwsleep/, profiles/r04/mwpoll/).
// Build-time switches (A/B libraries, tools/lib_ab.sh).
#ifndef MGCM_MW_TMO_EVERY
#define MGCM_MW_TMO_EVERY 64
#endif
#ifndef MGCM_MW_SLEEP
#define MGCM_MW_SLEEP 2
#endif
template <bool SYS = false>
__device__ __forceinline__ bool spin_fail(unsigned &spins, gu32 *tmo, unsigned ep) {
  ++spins;
  if (spins % MGCM_MW_TMO_EVERY == 0u || spins > (1u << 22)) {
    if (__hip_atomic_load(tmo, RLX_SCOPE(SYS)) == ep + 1u || spins > (1u << 22)) {
      __hip_atomic_store(tmo, ep + 1u, RLX_SCOPE(SYS));
      return true;
    }
  }
  if (MGCM_MW_SLEEP > 0) __builtin_amdgcn_s_sleep(MGCM_MW_SLEEP);
  return false;
}

// One grid-wide reduction: NV workgroup partials (a pairwise tree over the threads of
// v[0..NV-1]) published as granules and combined by wave 0 in the fixed order, the results
// broadcast through LDS; MAXOP: combine by max instead.
// The q of this part's ring points (ring 1, then ring 2), handed off with a reduction: the
// waves other than wave 0 sweep their granules into LDS while wave 0 combines the partials.
struct MwImport {
  size_t gi;       // first import slot of this part
  int nImp;
  double *imp_l;   // LDS staging, nImp doubles
  const gu64 *src; // the export granules read (T.xs; CG2D_SR alternates two buffers)
};

template <int NV, bool MAXOP, bool SYS = false>
__device__ __forceinline__ bool mw_sync(double *v, const MwgTables &T, int g, int &nsync, double *red, unsigned ep,
                                        const MwImport *imp = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  nsync++;
  const unsigned tag = mw_tag(ep, nsync);
  gu64 *P = (gu64 *)(T.part + (size_t)(nsync & 1) * MW_NV * T.G * 2);
  // workgroup partial: the pairwise tree over its threads (wave tree, then the row-16 tree
  // over the zero-padded wave values: the operations of block_sum_nw)
#pragma unroll
  for (int q = 0; q < NV; q++) {
    const double w = MAXOP ? mw_wave_max(v[q]) : mw_wave_sum(v[q]);
    if (lane == 0) red[q * 16 + wv] = w;
  }
  __syncthreads();
  if (wv == 0) {
    const int l = lane & 15;
#pragma unroll
    for (int q = 0; q < NV; q++) {
      const double xw = l < MW_NW ? red[q * 16 + l] : 0.0;
      const double wgp = MAXOP ? mw_rowmax16(xw) : mw_row16(xw);
      if (lane == 0) gran_put<SYS>(P + ((size_t)q * T.G + g) * 2, tag, wgp);
    }
    // combine: lane l adds partials l, l+64, ... in order, then the pairwise tree over the
    // lanes; the whole sweep is repeated until every granule carries this phase's tag.  Up
    // to MW_KG partials per lane (G <= 64*MW_KG) the sweep is unrolled: every granule load
    // of a sweep is issued before the first is used, so a sweep costs one round trip rather
    // than one per partial (a run-time loop waits for each load before its add)
    double acc[NV];
    unsigned spins = 0;
    bool ok = true;
    constexpr int MW_KG = 2;
    if (T.G <= 64 * MW_KG) {
      for (;;) {
        double xs[NV][MW_KG];
        bool gd[NV][MW_KG];
#pragma unroll
        for (int q = 0; q < NV; q++)
#pragma unroll
          for (int r = 0; r < MW_KG; r++) {
            const int gg = lane + 64 * r;
            xs[q][r] = 0.0;
            gd[q][r] = gg < T.G ? gran_get<SYS>(P + ((size_t)q * T.G + gg) * 2, tag, xs[q][r]) : true;
          }
        bool good = true;
#pragma unroll
        for (int q = 0; q < NV; q++) {
          acc[q] = 0.0;
#pragma unroll
          for (int r = 0; r < MW_KG; r++) {
            good = good && gd[q][r];
            if (lane + 64 * r < T.G) acc[q] = MAXOP ? fmax(acc[q], xs[q][r]) : acc[q] + xs[q][r];
          }
        }
        if (__all(good)) break;
        if (spin_fail<SYS>(spins, (gu32 *)T.ctr + 1, ep)) { ok = false; break; }
      }
    } else {
      for (;;) {
        bool good = true;
#pragma unroll
        for (int q = 0; q < NV; q++) {
          acc[q] = 0.0;
          for (int gg = lane; gg < T.G; gg += 64) {
            double xg;
            good = gran_get<SYS>(P + ((size_t)q * T.G + gg) * 2, tag, xg) && good;
            acc[q] = MAXOP ? fmax(acc[q], xg) : acc[q] + xg;
          }
        }
        if (__all(good)) break;
        if (spin_fail<SYS>(spins, (gu32 *)T.ctr + 1, ep)) { ok = false; break; }
      }
    }
#pragma unroll
    for (int q = 0; q < NV; q++) {
      const double rv = MAXOP ? mw_wave_max(acc[q]) : mw_wave_sum(acc[q]);
      if (lane == 0) red[(8 + q) * 16] = rv;
    }
    if (lane == 0) red[15 * 16] = ok ? 1.0 : 0.0;
  } else if (imp) {
    for (int q0 = 0; q0 < imp->nImp; q0 += MW_NT - 64) {
      const int qq = q0 + tid - 64;
      const bool act = qq < imp->nImp;
      gu64 *src = (gu64 *)imp->src + (size_t)2 * (act ? T.impC[imp->gi + qq] : 0);
      double xv = 0.0;
      unsigned spins = 0;
      for (;;) {
        const bool good = !act || gran_get<SYS>(src, tag, xv);
        if (__all(good)) break;
        if (spin_fail<SYS>(spins, (gu32 *)T.ctr + 1, ep)) break;   // the timeout word fails the solve
      }
      if (act) imp->imp_l[qq] = xv;
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV; q++) v[q] = red[(8 + q) * 16];
  return red[15 * 16] != 0.0;
}

#ifdef MGCM_CG_STAMPS   // diagnostic build only: per-phase shader-cycle totals of part 0
#define MW_STAMP(k)                                                                   \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    unsigned long long t_;                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
    __builtin_amdgcn_sched_barrier(0);                                                \
    if ((k) > 0) stampAcc[(k) - 1] += t_ - stampPrev;                                 \
    stampPrev = t_;                                                                   \
  } while (0)
#else
#define MW_STAMP(k) \
  do {              \
  } while (0)
#endif

// g0, gN: this launch runs parts g0 .. g0+gN-1 of the T.G (all of them in one process; a
// process's tiles' parts in the tile-sharded device CG2D, whose other parts run in the other
// processes' launches on the same hand-off block)
template <bool PINNED, bool SYS>
__global__ void __launch_bounds__(MW_NT) k_cg2d_mwg(Dims d, Params p, Fields f, MwgTables T, int maxIters,
                                                    int nIterMinIn, SolveRecord *rec, int *stepCounter, int g0, int gN) {
  int g = (int)blockIdx.x;
  if (PINNED) {
    if (g % MG_NXCD) return;   // parts on XCD 0 only: their hand-offs stay in one L2
    g /= MG_NXCD;
  }
  if (g >= gN) return;
  g += g0;
  constexpr int NO = MW_OPT * MW_NT, NR = MW_RPT * MW_NT;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int SZ = T.SZ;            // own + ring 1 + ring 2 slots; ZERO slot = SZ
  double *s_l = lds;              // SZ + 1
  double *r_l = lds + (SZ + 1);   // NO + NR used, + ZERO at SZ
  double *red = lds + 2 * (SZ + 1);   // 16 x 16 scratch
  double *imp_l = red + 16 * 16;      // IMAX: the ring q handed off at the last reduction
  const int tid = threadIdx.x;
  int nsync = 0;
  const unsigned ep = __hip_atomic_load((gu32 *)T.epoch, RLX_AGENT);
  const size_t go = (size_t)g * NO, gr = (size_t)g * NR, gi = (size_t)g * T.IMAX;
  // ---- owned points: offsets, neighbour slots, coefficients (cg2d.F operator rows)
  int G2[MW_OPT];
  unsigned nwe[MW_OPT], nsn[MW_OPT];
  double aW0[MW_OPT], aW1[MW_OPT], aS0[MW_OPT], aS1[MW_OPT], aC[MW_OPT];
  double pC[MW_OPT], pW0[MW_OPT], pW1[MW_OPT], pS0[MW_OPT], pS1[MW_OPT];
  double x[MW_OPT], r[MW_OPT], s[MW_OPT], q[MW_OPT], b[MW_OPT];
  const unsigned exp = T.ownExp[(size_t)g * MW_NT + tid];
  const long nx = d.nx;
#pragma unroll
  for (int m = 0; m < MW_OPT; m++) {
    const int sl = m * MW_NT + tid;
    G2[m] = T.ownG[go + sl];
    nwe[m] = T.ownNb[2 * (go + sl)];
    nsn[m] = T.ownNb[2 * (go + sl) + 1];
    const bool act = G2[m] >= 0;
    const long gg = act ? G2[m] : 0;
    const double az = act ? 1.0 : 0.0;
    aW0[m] = az * f.aW2d[gg]; aW1[m] = az * f.aW2d[gg + 1]; aS0[m] = az * f.aS2d[gg]; aS1[m] = az * f.aS2d[gg + nx];
    aC[m] = az * f.aC2d[gg];
    pC[m] = az * f.pC[gg]; pW0[m] = az * f.pW[gg]; pW1[m] = az * f.pW[gg + 1]; pS0[m] = az * f.pS[gg];
    pS1[m] = az * f.pS[gg + nx];
    b[m] = act ? f.cg2d_b[gg] : 0.0;
    x[m] = act ? f.cg2d_x[gg] : 0.0;
    s[m] = 0.0;
  }
  // ---- ring-1 points (r kept redundantly)
  int RG[MW_RPT];
  unsigned rwe[MW_RPT], rsn[MW_RPT];
  double raW0[MW_RPT], raW1[MW_RPT], raS0[MW_RPT], raS1[MW_RPT], raC[MW_RPT], rr[MW_RPT], rb[MW_RPT];
#pragma unroll
  for (int m = 0; m < MW_RPT; m++) {
    const int sl = m * MW_NT + tid;
    RG[m] = T.ringG[gr + sl];
    rwe[m] = T.ringNb[2 * (gr + sl)];
    rsn[m] = T.ringNb[2 * (gr + sl) + 1];
    const bool act = RG[m] >= 0;
    const long gg = act ? RG[m] : 0;
    const double az = act ? 1.0 : 0.0;
    raW0[m] = az * f.aW2d[gg]; raW1[m] = az * f.aW2d[gg + 1]; raS0[m] = az * f.aS2d[gg]; raS1[m] = az * f.aS2d[gg + nx];
    raC[m] = az * f.aC2d[gg];
    rb[m] = act ? f.cg2d_b[gg] : 0.0;
  }
  // CG2D_SR forms y = M r on ring 1 too: the ring points' preconditioner rows
  const bool SR = p.useSRCGSolver != 0;
  double rpC[MW_RPT], rpW0[MW_RPT], rpW1[MW_RPT], rpS0[MW_RPT], rpS1[MW_RPT];
#pragma unroll
  for (int m = 0; m < MW_RPT; m++) {
    const bool act = SR && RG[m] >= 0;
    const long gg = act ? RG[m] : 0;
    const double az = act ? 1.0 : 0.0;
    rpC[m] = az * f.pC[gg]; rpW0[m] = az * f.pW[gg]; rpW1[m] = az * f.pW[gg + 1]; rpS0[m] = az * f.pS[gg];
    rpS1[m] = az * f.pS[gg + nx];
  }
  const int nImp = T.nImp[g];
  const MwImport imp{gi, nImp, imp_l, (const gu64 *)T.xs};
#define LO(w) ((w) & 0xFFFFu)
#define HI(w) ((w) >> 16)

  // cg2d.F:104-133: normalise the RHS by its global max
  double rhsMaxV[1] = {0.0};
#pragma unroll
  for (int m = 0; m < MW_OPT; m++) { b[m] = b[m] * p.cg2dNorm; rhsMaxV[0] = fmax(fabs(b[m]), rhsMaxV[0]); }
  bool ok = mw_sync<1, true, SYS>(rhsMaxV, T, g, nsync, red, ep);
  const double rhsMax = rhsMaxV[0];
  double rhsNorm = 1.0;
  if (p.cg2dNormaliseRHS) {
    if (rhsMax != 0.0) rhsNorm = 1.0 / rhsMax;
#pragma unroll
    for (int m = 0; m < MW_OPT; m++) { b[m] = b[m] * rhsNorm; x[m] = x[m] * rhsNorm; }
  }
#pragma unroll
  for (int m = 0; m < MW_RPT; m++) rb[m] = (rb[m] * p.cg2dNorm) * (p.cg2dNormaliseRHS ? rhsNorm : 1.0);
  // cgUseMinResSol (cg2d.F:148-155, 190-193, 338-347, 358-368): the lowest-residual solution,
  // saved from the normalised first guess on (every part tests the same reduced err_sq)
  const bool minRes = nIterMinIn >= 0;
  double xmin[MW_OPT];
#pragma unroll
  for (int m = 0; m < MW_OPT; m++) xmin[m] = x[m];
  // EXCH_XY_RL(cg2d_x): x of owned points and of both rings into s_l (the ring values are read
  // from cg2d_x, written before this launch, and scaled with the owner's arithmetic)
#pragma unroll
  for (int m = 0; m < MW_OPT; m++) s_l[m * MW_NT + tid] = x[m];
  for (int qq = tid; qq < nImp; qq += MW_NT) {
    const double xv = f.cg2d_x[T.impG[gi + qq]];
    s_l[NO + qq] = p.cg2dNormaliseRHS ? xv * rhsNorm : xv;
  }
  if (tid == 0) { s_l[SZ] = 0.0; r_l[SZ] = 0.0; }
  __syncthreads();
  // cg2d.F:139-180: r = b - A x on owned points and ring 1
  double v3[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int m = 0; m < MW_OPT; m++) {
    r[m] = b[m] - (aW0[m] * s_l[LO(nwe[m])] + aW1[m] * s_l[HI(nwe[m])] + aS0[m] * s_l[LO(nsn[m])] +
                   aS1[m] * s_l[HI(nsn[m])] + aC[m] * x[m]);
    v3[0] = v3[0] + r[m] * r[m];
    v3[1] = v3[1] + b[m];
  }
#pragma unroll
  for (int m = 0; m < MW_RPT; m++)
    rr[m] = rb[m] - (raW0[m] * s_l[LO(rwe[m])] + raW1[m] * s_l[HI(rwe[m])] + raS0[m] * s_l[LO(rsn[m])] +
                     raS1[m] * s_l[HI(rsn[m])] + raC[m] * s_l[NO + m * MW_NT + tid]);
#pragma unroll
  for (int m = 0; m < MW_OPT; m++)
    if (G2[m] >= 0) f.cg2d_b[G2[m]] = b[m];   // cg2d_b is INOUT (normalised in place)
#pragma unroll
  for (int m = 0; m < MW_OPT; m++) r_l[m * MW_NT + tid] = r[m];
#pragma unroll
  for (int m = 0; m < MW_RPT; m++) r_l[NO + m * MW_NT + tid] = rr[m];
  __syncthreads();
  gu64 *xs = (gu64 *)T.xs;
  double err_sq, sumRHS, firstResidual;
  int actualIts = 0;
  int nIterMin = nIterMinIn;
  double minResidualSq = -1.0;
  if (SR) {
    // CG2D_SR (cg2d_sr.F:100-440; the oracle's cg2d_sr): ONE grid hand-off per iteration.
    // Each part keeps r and q on both rings as copies (r -= sigma*q, q = v + beta*q: the
    // owner's expressions on the owner's bytes), forms y = M r on its points and ring 1 and
    // v = A y on its points, and hands off v of its exported points with the three partials
    // (y.r, y.v, r.r): the rings' v arrive with the sums.  The exports alternate between two
    // buffers (a fast part exports for the next hand-off while a slow one still reads this one).
    // The ring-2 r cannot be formed locally (it needs x on ring 3): it arrives with the first
    // residual's sums.
    gu64 *xsb[2] = {xs, xs + (size_t)2 * T.nExp};
    double *qr_l = imp_l + T.IMAX;   // the rings' q (nImp)
    auto exportv = [&](const double (&val)[MW_OPT]) {
#pragma unroll
      for (int m = 0; m < MW_OPT; m++)
        if ((exp >> m) & 1u)
          gran_put<SYS>(xsb[(nsync + 1) & 1] + (size_t)2 * T.ownC[go + m * MW_NT + tid], mw_tag(ep, nsync + 1), val[m]);
    };
    auto impOf = [&]() { return MwImport{gi, nImp, imp_l, (const gu64 *)xsb[(nsync + 1) & 1]}; };
    exportv(r);
    double v2[2] = {v3[0], v3[1]};
    {
      const MwImport ir = impOf();
      ok = ok && mw_sync<2, false, SYS>(v2, T, g, nsync, red, ep, &ir);
    }
    err_sq = v2[0];
    sumRHS = v2[1];
    firstResidual = sqrt(err_sq);
    if (minRes) { nIterMin = 0; minResidualSq = err_sq; }
    for (int qq = tid; qq < nImp; qq += MW_NT) r_l[NO + qq] = imp_l[qq];
    __syncthreads();
    // y = M r on the owned points and ring 1, into s_l
    double y[MW_OPT];
    auto form_y = [&]() {
#pragma unroll
      for (int m = 0; m < MW_OPT; m++) {
        y[m] = pC[m] * r[m] + pW0[m] * r_l[LO(nwe[m])] + pW1[m] * r_l[HI(nwe[m])] + pS0[m] * r_l[LO(nsn[m])] +
               pS1[m] * r_l[HI(nsn[m])];
        s_l[m * MW_NT + tid] = y[m];
      }
#pragma unroll
      for (int m = 0; m < MW_RPT; m++)
        s_l[NO + m * MW_NT + tid] = rpC[m] * r_l[NO + m * MW_NT + tid] + rpW0[m] * r_l[LO(rwe[m])] +
                                    rpW1[m] * r_l[HI(rwe[m])] + rpS0[m] * r_l[LO(rsn[m])] + rpS1[m] * r_l[HI(rsn[m])];
    };
    auto apply_A = [&](double (&out)[MW_OPT]) {   // A (s_l) on the owned points
#pragma unroll
      for (int m = 0; m < MW_OPT; m++)
        out[m] = aW0[m] * s_l[LO(nwe[m])] + aW1[m] * s_l[HI(nwe[m])] + aS0[m] * s_l[LO(nsn[m])] +
                 aS1[m] * s_l[HI(nsn[m])] + aC[m] * y[m];
    };
    int it2d = 0;
    bool conv = false;
    if (ok && !(err_sq < p.cg2dTolerance_sq)) {
      // the standard first step (cg2d_sr.F:190-260): y = M r, s = y, eta = y.r, q = A s,
      // alpha = s.q -- both sums in one hand-off, with the rings' q
      form_y();
      double ev[2] = {0.0, 0.0};
#pragma unroll
      for (int m = 0; m < MW_OPT; m++) { s[m] = y[m]; ev[0] = ev[0] + y[m] * r[m]; }
      __syncthreads();
      apply_A(q);
#pragma unroll
      for (int m = 0; m < MW_OPT; m++) ev[1] = ev[1] + s[m] * q[m];
      exportv(q);
      {
        const MwImport iq = impOf();
        ok = mw_sync<2, false, SYS>(ev, T, g, nsync, red, ep, &iq);
      }
      double eta_qrN = ev[0], eta_qrNM1 = eta_qrN, alpha = ev[1];
      double sigma = eta_qrN / alpha;
#pragma unroll
      for (int m = 0; m < MW_OPT; m++) {
        x[m] = x[m] + sigma * s[m];
        r[m] = r[m] - sigma * q[m];
        r_l[m * MW_NT + tid] = r[m];
      }
      for (int qq = tid; qq < nImp; qq += MW_NT) {
        qr_l[qq] = imp_l[qq];
        r_l[NO + qq] = r_l[NO + qq] - sigma * qr_l[qq];
      }
      __syncthreads();
      for (it2d = 1; ok && it2d <= maxIters - 1; it2d++) {   // cg2d_sr.F:262-370
        form_y();
        __syncthreads();
        double v[MW_OPT];
        apply_A(v);
        double sv[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int m = 0; m < MW_OPT; m++) sv[0] = sv[0] + y[m] * r[m];
#pragma unroll
        for (int m = 0; m < MW_OPT; m++) sv[1] = sv[1] + y[m] * v[m];
#pragma unroll
        for (int m = 0; m < MW_OPT; m++) sv[2] = sv[2] + r[m] * r[m];
        exportv(v);
        {
          const MwImport iv = impOf();
          ok = mw_sync<3, false, SYS>(sv, T, g, nsync, red, ep, &iv);
        }
        if (!ok) break;
        eta_qrN = sv[0];
        const double delta = sv[1];
        err_sq = sv[2];
        if (err_sq < p.cg2dTolerance_sq) { conv = true; break; }
        if (minRes && err_sq < minResidualSq) {
          minResidualSq = err_sq;
          nIterMin = it2d;
#pragma unroll
          for (int m = 0; m < MW_OPT; m++) xmin[m] = x[m];
        }
        const double cgBeta = eta_qrN / eta_qrNM1;
        eta_qrNM1 = eta_qrN;
        alpha = delta - (cgBeta * cgBeta) * alpha;
        sigma = eta_qrN / alpha;
#pragma unroll
        for (int m = 0; m < MW_OPT; m++) {
          s[m] = y[m] + cgBeta * s[m];
          x[m] = x[m] + sigma * s[m];
          q[m] = v[m] + cgBeta * q[m];
          r[m] = r[m] - sigma * q[m];
          r_l[m * MW_NT + tid] = r[m];
        }
        for (int qq = tid; qq < nImp; qq += MW_NT) {
          const double qn = imp_l[qq] + cgBeta * qr_l[qq];
          qr_l[qq] = qn;
          r_l[NO + qq] = r_l[NO + qq] - sigma * qn;
        }
        __syncthreads();
      }
      if (ok && !conv) {   // cg2d_sr.F:372-382: the residual of the last update
        double e1[1] = {0.0};
#pragma unroll
        for (int m = 0; m < MW_OPT; m++) e1[0] = e1[0] + r[m] * r[m];
        ok = mw_sync<1, false, SYS>(e1, T, g, nsync, red, ep);
        err_sq = e1[0];
      }
    }
    actualIts = it2d;   // cg2d_sr.F:410: the loop index at exit
  } else {
    // q = M r and (q, r) of iteration 1, reduced with err_sq and sumRHS; q exported for the
    // parts whose rings hold these points; the ring copies of s start at s = 0 like the owners'
  #pragma unroll
    for (int m = 0; m < MW_OPT; m++) {
      q[m] = pC[m] * r[m] + pW0[m] * r_l[LO(nwe[m])] + pW1[m] * r_l[HI(nwe[m])] + pS0[m] * r_l[LO(nsn[m])] +
             pS1[m] * r_l[HI(nsn[m])];
      v3[2] = v3[2] + q[m] * r[m];
      if ((exp >> m) & 1u) gran_put<SYS>(xs + (size_t)2 * T.ownC[go + m * MW_NT + tid], mw_tag(ep, nsync + 1), q[m]);
    }
    for (int qq = tid; qq < nImp; qq += MW_NT) s_l[NO + qq] = 0.0;
    ok = ok && mw_sync<3, false, SYS>(v3, T, g, nsync, red, ep, &imp);
    err_sq = v3[0];
    sumRHS = v3[1];
    double eta_qrN = v3[2], eta_qrNM1 = 1.0;
    firstResidual = sqrt(err_sq);
    if (minRes) { nIterMin = 0; minResidualSq = err_sq; }
    if (ok && !(err_sq < p.cg2dTolerance_sq)) {
  #ifdef MGCM_CG_STAMPS
      unsigned long long stampAcc[6] = {0, 0, 0, 0, 0, 0}, stampPrev = 0;
      const unsigned long long stampT0 = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_s_waitcnt(0xC07F);
  #endif
      for (int it2d = 1; it2d <= maxIters; it2d++) {
        const double cgBeta = eta_qrN / eta_qrNM1;
        eta_qrNM1 = eta_qrN;
        // s = q + beta*s on the owned points and, with the q handed off at sync B, on both rings
        // (EXCH_S3D_RL(cg2d_s)); the next export of q comes after sync D, when every part has
        // read this one
  #pragma unroll
        for (int m = 0; m < MW_OPT; m++) {
          s[m] = q[m] + cgBeta * s[m];
          s_l[m * MW_NT + tid] = s[m];
        }
        MW_STAMP(0);
        for (int qq = tid; qq < nImp; qq += MW_NT) s_l[NO + qq] = imp_l[qq] + cgBeta * s_l[NO + qq];
        __syncthreads();
        MW_STAMP(1);
        // q = A s (owned + ring 1); alpha = eta_qrN / (s, A s)
        double av[1] = {0.0};
  #pragma unroll
        for (int m = 0; m < MW_OPT; m++) {
          q[m] = aW0[m] * s_l[LO(nwe[m])] + aW1[m] * s_l[HI(nwe[m])] + aS0[m] * s_l[LO(nsn[m])] + aS1[m] * s_l[HI(nsn[m])] +
                 aC[m] * s[m];
          av[0] = av[0] + s[m] * q[m];
        }
        double rq[MW_RPT];
  #pragma unroll
        for (int m = 0; m < MW_RPT; m++)
          rq[m] = raW0[m] * s_l[LO(rwe[m])] + raW1[m] * s_l[HI(rwe[m])] + raS0[m] * s_l[LO(rsn[m])] +
                  raS1[m] * s_l[HI(rsn[m])] + raC[m] * s_l[NO + m * MW_NT + tid];
        MW_STAMP(2);
        ok = mw_sync<1, false, SYS>(av, T, g, nsync, red, ep);
        MW_STAMP(3);
        if (!ok) break;
        const double alpha = eta_qrN / av[0];
        // x += alpha s ; r -= alpha q (owned and ring 1); err_sq and the next (M r, r)
        double v2[2] = {0.0, 0.0};
  #pragma unroll
        for (int m = 0; m < MW_OPT; m++) {
          x[m] = x[m] + alpha * s[m];
          r[m] = r[m] - alpha * q[m];
          v2[0] = v2[0] + r[m] * r[m];
          r_l[m * MW_NT + tid] = r[m];
        }
  #pragma unroll
        for (int m = 0; m < MW_RPT; m++) {
          rr[m] = rr[m] - alpha * rq[m];
          r_l[NO + m * MW_NT + tid] = rr[m];
        }
        actualIts = it2d;
        __syncthreads();
  #pragma unroll
        for (int m = 0; m < MW_OPT; m++) {
          q[m] = pC[m] * r[m] + pW0[m] * r_l[LO(nwe[m])] + pW1[m] * r_l[HI(nwe[m])] + pS0[m] * r_l[LO(nsn[m])] +
                 pS1[m] * r_l[HI(nsn[m])];
          v2[1] = v2[1] + q[m] * r[m];
          if ((exp >> m) & 1u) gran_put<SYS>(xs + (size_t)2 * T.ownC[go + m * MW_NT + tid], mw_tag(ep, nsync + 1), q[m]);
        }
        MW_STAMP(4);
        ok = mw_sync<2, false, SYS>(v2, T, g, nsync, red, ep, &imp);
        MW_STAMP(5);
        if (!ok) break;
        err_sq = v2[0];
        eta_qrN = v2[1];
        if (err_sq < p.cg2dTolerance_sq) break;
        if (minRes && err_sq < minResidualSq) {
          minResidualSq = err_sq;
          nIterMin = it2d;
  #pragma unroll
          for (int m = 0; m < MW_OPT; m++) xmin[m] = x[m];
        }
      }
  #ifdef MGCM_CG_STAMPS
      if (g == 0 && threadIdx.x == 0)
        printf("MWSTAMP G %d its %d total %llu | import %llu applyA %llu syncD %llu upd+applyM %llu syncB %llu\n", T.G,
               actualIts, __builtin_amdgcn_s_memtime() - stampT0, stampAcc[0], stampAcc[1], stampAcc[2], stampAcc[3],
               stampAcc[4]);
  #endif
    }
  }
  const bool useMin = minRes && err_sq > minResidualSq;
#pragma unroll
  for (int m = 0; m < MW_OPT; m++) {
    double xv = useMin ? xmin[m] : x[m];
    if (p.cg2dNormaliseRHS) xv = xv / rhsNorm;
    if (G2[m] >= 0) f.cg2d_x[G2[m]] = xv;
  }
  // the record and this process's next epoch by the launch's first part (every part holds the
  // same reduced values)
  if (g == g0 && tid == 0) {
    const int st = stepCounter ? *stepCounter : 0;
    SolveRecord &R = rec[st];
    R.firstResidual = firstResidual;
    R.lastResidual = sqrt(err_sq);
    R.minResidualSq = minResidualSq;
    R.rhsMax = rhsMax;
    R.sumRHS = sumRHS;
    const bool tmo = __hip_atomic_load((gu32 *)T.ctr + 1, RLX_SCOPE(SYS)) == ep + 1u;
    R.numIters = (ok && !tmo) ? actualIts : -1;   // -1: a grid hand-off timed out
    R.nIterMin = nIterMin;
    // the next launch's epoch; after a timeout it skips one, so a part of this launch that
    // starts late (reading ep + 1, tagging with it, failing into the timeout word as ep + 2)
    // can neither match the next launch's tags nor fail it
    __hip_atomic_store((gu32 *)T.epoch, R.numIters < 0 ? ep + 2u : ep + 1u, RLX_AGENT);
  }
#undef LO
#undef HI
}

int cg2d_mwg_geometry(int *nt, int *opt, int *rpt) { *nt = MW_NT; *opt = MW_OPT; *rpt = MW_RPT; return 0; }

hipError_t launch_cg2d_mwg(const Dims &d, const Params &p, const Fields &f, const MwgTables &T, int maxIters,
                           int nIterMin, SolveRecord *rec, int *stepCounter, hipStream_t s, int g0, int gN) {
  // phases per launch: 2 + 2 per iteration, below 2^16 (the tag's phase field)
  if (maxIters < 0 || maxIters > 30000) return hipErrorInvalidValue;
  if (gN < 0) { g0 = 0; gN = T.G; }
  if (g0 < 0 || gN < 1 || g0 + gN > T.G) return hipErrorInvalidValue;
  hipError_t e = hipSuccess;
  size_t lds = (size_t)(2 * (T.SZ + 1) + 16 * 16 + (p.useSRCGSolver ? 2 : 1) * T.IMAX) * sizeof(double);
  // a part may claim its CU's whole LDS so that no other kernel's workgroup shares the CU
  // (THERMODYNAMICS running beside the solve, model.hip one_step)
  if (T.exclusive) lds = 160 * 1024;
  const bool pinned = T.pinned && !T.sys && gN == T.G;
  const int v = (pinned ? 1 : 0) + (T.sys ? 2 : 0);
  auto kern = v == 3 ? k_cg2d_mwg<true, true> : v == 2 ? k_cg2d_mwg<false, true>
            : v == 1 ? k_cg2d_mwg<true, false> : k_cg2d_mwg<false, false>;
  static bool attrSet[4] = {false, false, false, false};
  if (!attrSet[v]) {
    e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attrSet[v] = true;
  }
  const unsigned grid = (unsigned)(pinned ? gN * MG_NXCD : gN);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(MW_NT), lds, s, d, p, f, T, maxIters, nIterMin, rec, stepCounter, g0, gN);
  return hipGetLastError();
}

}  // namespace mgcm
