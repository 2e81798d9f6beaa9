// kernels_solve.hip -- SOLVE_FOR_PRESSURE on the MI355X.
//
// Reference: model/src/solve_for_pressure.F:7-468, model/src/calc_div_ghat.F:6-201,
//            model/src/cg2d.F:13-415, eesupp/src/global_sum_tile.F:14-237,
//            model/src/momentum_correction_step.F:7-131, correction_step.F:150-234,
//            model/src/integr_continuity.F:276-314, integrate_for_w.F:61-195.
//
// CG2D is latency-bound at the BASELINE grids (3.6k-6k points, ~100 iterations
// per solve, 3 global sums + 2 halo exchanges per iteration in the reference):
// a launch per phase would cost more than the arithmetic.  k_cg2d_block runs
// the WHOLE solve in ONE workgroup of 1024 threads:
//   * r and s live in LDS (interior points only, compact); the halo exchange
//     of EXCH_S3D_RL becomes a neighbour-index table (halo point -> the interior
//     point it is a copy of), so an exchange costs nothing;
//   * x, s, r and (as register room allows) the 10 operator coefficients of
//     each point stay in VGPRs;
//   * each global sum is a DPP row reduction + 4 readlanes per wave, one LDS
//     slot per wave, one barrier, and a DPP row reduction of the 16 wave
//     partials; every lane ends with the bit-identical sum (no broadcast,
//     run-to-run deterministic).
#include <cstdlib>

#include "common.h"

namespace mgcm {

constexpr int CG_THREADS = 1024;
constexpr int CG_WAVES = CG_THREADS / 64;

// ---- wave64 reductions on the DPP path (no LDS round trips) --------------
// One DPP step moves a 64-bit value between lanes of a 16-lane row as two
// v_mov_b32_dpp.  Butterfly xor1 (quad_perm 1,0,3,2), xor2 (quad_perm 2,3,0,1),
// row_half_mirror, row_mirror: after the four steps every lane of a row holds
// the row's sum, bit-identical across the row (each step adds a commuted pair).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  // every pattern used here reads a valid lane for every lane (row/bank masks 0xF),
  // so the "old" operand is dead: tie it to the source instead of a zeroed register
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
// row_bcast15 (rows 1,3 <- lane 15 of rows 0,2) / row_bcast31 (rows 2,3 <- lane 31);
// rows outside ROWMASK receive +0.0, which leaves their partial unchanged.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_bcast_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), CTRL, ROWMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWMASK, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double row_sum16(double v) {
  v = v + dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v = v + dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v = v + dpp_f64<0x141>(v);  // row_half_mirror
  v = v + dpp_f64<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ double row_max16(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  v = fmax(v, dpp_f64<0x140>(v));
  return v;
}
__device__ __forceinline__ double lane_f64(double v, int l) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
// wave sum, uniform (SGPR) result: rows by DPP, then row1 += row0, row3 += row2
// (row_bcast15) and rows 2,3 += lane 31 (row_bcast31): lane 63 holds
// (r3+r2)+(r1+r0), the same value as (r0+r1)+(r2+r3).
__device__ __forceinline__ double wave_sum(double v) {
  v = row_sum16(v);
  v = v + dpp_bcast_f64<0x142, 0xA>(v);
  v = v + dpp_bcast_f64<0x143, 0xC>(v);
  return lane_f64(v, 63);
}
__device__ __forceinline__ double wave_max(double v) {
  v = row_max16(v);
  return fmax(fmax(lane_f64(v, 0), lane_f64(v, 16)), fmax(lane_f64(v, 32), lane_f64(v, 48)));
}

// Block-wide sum over the 16 waves; `slot` selects one of 4 rotating LDS
// partial buffers so consecutive reductions need only one barrier each.  After
// the barrier lane l of every wave reads partial[l & 15] and reduces its row:
// every lane of the block ends with the same, bit-identical sum.
__device__ __forceinline__ double block_sum(double v, double *red, int slot) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[slot * CG_WAVES + wv] = v;
  __syncthreads();
  return row_sum16(red[slot * CG_WAVES + (lane & 15)]);
}
__device__ __forceinline__ double block_max(double v, double *red, int slot) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[slot * CG_WAVES + wv] = v;
  __syncthreads();
  return row_max16(red[slot * CG_WAVES + (lane & 15)]);
}

// GLOBAL_SUM_TILE_RL in the reference's own order (cg2d.F:211-243 / 305-337 +
// global_sum_tile.F:161-191): every tile's interior terms added sequentially, j outer and
// i inner, from 0.0, then the tile partials added in tile order (bi fastest), from 0.0.
// The per-point terms go through LDS at their compact index (tile, j, i: build_nbr's
// order), one thread per tile sums them, and every thread adds the tile partials itself
// (identical values, no broadcast).  Costs two barriers and a serial chain of sNx*sNy adds
// per sum: the parity mode, not the performance path (cg2dRefOrder).
template <int PPT>
__device__ __forceinline__ double ref_sum(const double (&v)[PPT], double *term_l, double *tile_l, int nTiles,
                                          int tilePts) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int m = 0; m < PPT; m++) term_l[tid + m * CG_THREADS] = v[m];
  __syncthreads();
  for (int t = tid; t < nTiles; t += CG_THREADS) {
    const double *tp = term_l + (size_t)t * tilePts;
    double e = 0.0;
    for (int q = 0; q < tilePts; q++) e = e + tp[q];
    tile_l[t] = e;
  }
  __syncthreads();
  double sum = 0.0;
  for (int t = 0; t < nTiles; t++) sum = sum + tile_l[t];
  return sum;
}

// CALC_DIV_GHAT over k = Nr..1 + free-surface term; cg2d_x = Bo_surf*etaN (full range).
// With useRealFreshWaterFlux the RHS starts from the E-P-R volume flux
// (solve_for_pressure.F:142-151); with the CD scheme etaNm1 = etaN
// (solve_for_pressure.F:126-128) and CD_CODE_SCHEME's uNM1, vNM1 = u, v
// (cd_code_scheme.F:228-234) are saved here, after every k_cd_scheme read.
__global__ void __launch_bounds__(256) k_sfp_rhs(Dims d, Params p, Fields f, int nc) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  MG_COLF(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, nc)
  const int NS = d.Nr * NC_;
  double *sE = lds, *sW = lds + NS, *sN = lds + 2 * NS, *sS = lds + 3 * NS;
  const bool inner = i >= 1 && i <= d.sNx && j >= 1 && j <= d.sNy;
  const long q = MG_I2(d, i, j, t);
  if (valid && p.useCDscheme) MG_COLF_K(k) {
    const long q3 = MG_I3(d, i, j, k, t);
    f.uNM1[q3] = f.uVel[q3];
    f.vNM1[q3] = f.vVel[q3];
  }
  if (valid && inner) MG_COLF_K(k) {
    const int me = (k - 1) * NC_ + cc;
    {   // CALC_DIV_GHAT flux terms of level k
      const double drF = f.drF[k - 1];
      sE[me] = f.dyG[MG_I2(d, i + 1, j, t)] * drF * f.hFacW[MG_I3(d, i + 1, j, k, t)] *
               f.gU[MG_I3(d, i + 1, j, k, t)] / p.deltaTMom;
      sW[me] = f.dyG[q] * drF * f.hFacW[MG_I3(d, i, j, k, t)] * f.gU[MG_I3(d, i, j, k, t)] / p.deltaTMom;
      sN[me] = f.dxG[MG_I2(d, i, j + 1, t)] * drF * f.hFacS[MG_I3(d, i, j + 1, k, t)] *
               f.gV[MG_I3(d, i, j + 1, k, t)] / p.deltaTMom;
      sS[me] = f.dxG[q] * drF * f.hFacS[MG_I3(d, i, j, k, t)] * f.gV[MG_I3(d, i, j, k, t)] / p.deltaTMom;
    }
  }
  __syncthreads();
  if (!valid || kk != 0) return;
  sfp_rhs_column(d, p, f, q, inner, sE, sW, sN, sS, NC_, cc);
}

// k_sfp_rhs as a k-march at a fixed depth NR: one thread per column, k = NR..1 fully unrolled
// (sfp_rhs_column's order), each batch of levels' operands loaded before its sums (about 40
// loads in flight per wave: the 105 300 columns of LLC-90 give only 1.6 waves per SIMD), the
// four face terms in registers.  The same expression trees as k_sfp_rhs + sfp_rhs_column:
// bit-identical.
template <int NR>
__device__ __forceinline__ double sfp_column_sum(double b, long q3b, long nx, long n2, double dyW, double dyE, double dxS,
                                                 double dxN, double dT, const double *__restrict__ drFv,
                                                 const double *__restrict__ hFacW, const double *__restrict__ hFacS,
                                                 const double *__restrict__ gU, const double *__restrict__ gV) {
  // batches of SB levels: the batch's 8*SB operands are loaded before its first sum
  constexpr int SB = 10;
  static_assert(NR % SB == 0, "whole batches");
#pragma unroll
  for (int k0 = NR; k0 >= 1; k0 -= SB) {
    double hWe[SB], hWw[SB], uE[SB], uW[SB], hSn[SB], hSs[SB], vN[SB], vS[SB];
#pragma unroll
    for (int m = 0; m < SB; m++) {
      const long q3 = q3b + (long)(k0 - m - 1) * n2;
      hWe[m] = hFacW[q3 + 1]; uE[m] = gU[q3 + 1]; hWw[m] = hFacW[q3]; uW[m] = gU[q3];
      hSn[m] = hFacS[q3 + nx]; vN[m] = gV[q3 + nx]; hSs[m] = hFacS[q3]; vS[m] = gV[q3];
    }
#pragma unroll
    for (int m = 0; m < SB; m++) {
      const double drF = drFv[k0 - m - 1];
      const double sE = dyE * drF * hWe[m] * uE[m] / dT;
      const double sW = dyW * drF * hWw[m] * uW[m] / dT;
      const double sN = dxN * drF * hSn[m] * vN[m] / dT;
      const double sS = dxS * drF * hSs[m] * vS[m] / dT;
      b = b + sE - sW;
      b = b + sN - sS;
    }
  }
  return b;
}
template <int NR>
__global__ void __launch_bounds__(256) k_sfp_rhs_march(Dims d, Params p, Fields f) {
  const long g = (long)mg_xcd_block() * 256 + threadIdx.x;
  if (g >= d.n2 * d.nT) return;
  const int t = d.t0 + (int)(g / d.n2);
  const long r = g % d.n2, nx = d.nx, n2 = d.n2;
  const int i = (int)(r % nx) + 1 - d.OLx, j = (int)(r / nx) + 1 - d.OLy;
  const long q = (long)t * n2 + r;
  // the point's own 2-D operands read up front (every 2-D field spans the whole slab), so none
  // waits behind the column sum's batches
  const double rAq = f.rA[q], emp = f.EmPmR[q], mIn = f.maskInC[q], etaNq = f.etaN[q], Bo = f.Bo_surf[q];
  const double etaB = (p.exactConserv ? f.etaH : f.etaN)[q];
  double b = 0.0;
  if (i >= 1 && i <= d.sNx && j >= 1 && j <= d.sNy) {
    if (p.useRealFreshWaterFlux) {
      const double tmpFac = p.freeSurfFac * (1.0 / p.rhoConst) * p.implicDiv2DFlow;
      b = tmpFac * rAq * emp / p.deltaTMom * mIn;
    }
    b = sfp_column_sum<NR>(b, (long)t * d.n3 + r, nx, n2, f.dyG[q], f.dyG[q + 1], f.dxG[q], f.dxG[q + nx], p.deltaTMom,
                           f.drF, f.hFacW, f.hFacS, f.gU, f.gV);
    b = b - p.freeSurfFac * rAq / p.deltaTMom / p.deltaTFreeSurf * etaB;
  }
  f.cg2d_x[q] = Bo * etaNq;
  f.cg2d_b[q] = b;
}

// Whole-solve CG2D in one workgroup.  PPT = interior points per thread.
// Points are padded to NP = PPT*1024: a padding point has x = b = 0, every
// neighbour index pointing at the ZERO slot (index NP, never written), so it
// stays exactly 0 through every phase and the per-point code is branch-free.
// nbr[2*NP]: packed compact neighbour indices (W | E<<16), (S | N<<16); when the
// neighbour is a halo point, the index is the interior point the halo is a copy
// of (EXCH_S3D_RL / EXCH_XY_RL).  CREG: how many of the two 5-coefficient sets
// (A, then M) stay in VGPRs; the rest is re-read each use from L2.
template <int PPT, bool MINRES, int CREG, bool REFSUM = false>
__global__ void __launch_bounds__(CG_THREADS) k_cg2d_block(Dims d, Params p, Fields f, const unsigned *__restrict__ nbr,
                                                          const int *__restrict__ gofs, int nPts, int maxIters,
                                                          int nIterMinIn, SolveRecord *rec, int *stepCounter) {
  constexpr int NP = PPT * CG_THREADS;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double *r_l = lds;                // NP + 1 (last = ZERO slot)
  double *s_l = lds + (NP + 1);     // NP + 1
  double *red = lds + 2 * (NP + 1); // 4 * CG_WAVES
  // REFSUM (cg2dRefOrder): per-point terms and tile partials of the reference-order sums
  double *term_l = red + 4 * CG_WAVES;   // NP
  double *tile_l = term_l + NP;          // nTiles
  const int nTilesR = d.nTiles, tilePts = d.sNx * d.sNy;
  const int tid = threadIdx.x;
  constexpr int RA = (CREG >= 1) ? PPT : 1, RM = (CREG >= 2) ? PPT : 1, RX = MINRES ? PPT : 1;

  unsigned g[PPT];  // BYTE offset of the point in a 2-D field (32-bit: saddr-mode loads)
  unsigned nwe[PPT], nsn[PPT];
  double x[PPT], s[PPT], r[PPT], xmin[RX];
  double aW0r[RA], aW1r[RA], aS0r[RA], aS1r[RA], aCr[RA];
  double pCr[RM], pW0r[RM], pW1r[RM], pS0r[RM], pS1r[RM];
  const unsigned dE = 8u, dN = 8u * (unsigned)d.nx;
  // buffer descriptors (32-bit voffset + immediate offsets: one VGPR per point
  // addresses all ten coefficient loads; guide T8)
  const unsigned fbytes = (unsigned)(8 * d.n2 * d.nTiles);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc((void *)f.aW2d, 0, fbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsS = __builtin_amdgcn_make_buffer_rsrc((void *)f.aS2d, 0, fbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc((void *)f.aC2d, 0, fbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rpW = __builtin_amdgcn_make_buffer_rsrc((void *)f.pW, 0, fbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rpS = __builtin_amdgcn_make_buffer_rsrc((void *)f.pS, 0, fbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rpC = __builtin_amdgcn_make_buffer_rsrc((void *)f.pC, 0, fbytes, 0x00020000);
#define BLD(rs, off) __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, (off), 0, 0))
#define LDO(base, off) (*(const double *)((const char *)(base) + (off)))
#define STO(base, off) (*(double *)((char *)(base) + (off)))
#define aW0(m) ((CREG >= 1) ? aW0r[(CREG >= 1) ? m : 0] : BLD(rsW, g[m]))
#define aW1(m) ((CREG >= 1) ? aW1r[(CREG >= 1) ? m : 0] : BLD(rsW, g[m] + dE))
#define aS0(m) ((CREG >= 1) ? aS0r[(CREG >= 1) ? m : 0] : BLD(rsS, g[m]))
#define aS1(m) ((CREG >= 1) ? aS1r[(CREG >= 1) ? m : 0] : BLD(rsS, g[m] + dN))
#define aC(m) ((CREG >= 1) ? aCr[(CREG >= 1) ? m : 0] : BLD(rsC, g[m]))
#define pC(m) ((CREG >= 2) ? pCr[(CREG >= 2) ? m : 0] : BLD(rpC, g[m]))
#define pW0(m) ((CREG >= 2) ? pW0r[(CREG >= 2) ? m : 0] : BLD(rpW, g[m]))
#define pW1(m) ((CREG >= 2) ? pW1r[(CREG >= 2) ? m : 0] : BLD(rpW, g[m] + dE))
#define pS0(m) ((CREG >= 2) ? pS0r[(CREG >= 2) ? m : 0] : BLD(rpS, g[m]))
#define pS1(m) ((CREG >= 2) ? pS1r[(CREG >= 2) ? m : 0] : BLD(rpS, g[m] + dN))
#define LO(w) ((w) & 0xFFFFu)
#define HI(w) ((w) >> 16)
#define ACT(m) (tid + (m) * CG_THREADS < nPts)

  if (tid == 0) { r_l[NP] = 0.0; s_l[NP] = 0.0; }
  double b[PPT];
#pragma unroll
  for (int m = 0; m < PPT; m++) {
    const int pt = tid + m * CG_THREADS;
    g[m] = 8u * (unsigned)gofs[pt];
    nwe[m] = nbr[2 * pt];
    nsn[m] = nbr[2 * pt + 1];
    if (CREG >= 1) {
      const int mm = (CREG >= 1) ? m : 0;
      aW0r[mm] = BLD(rsW, g[m]); aW1r[mm] = BLD(rsW, g[m] + dE); aS0r[mm] = BLD(rsS, g[m]); aS1r[mm] = BLD(rsS, g[m] + dN);
      aCr[mm] = BLD(rsC, g[m]);
    }
    if (CREG >= 2) {
      const int mm = (CREG >= 2) ? m : 0;
      pCr[mm] = BLD(rpC, g[m]); pW0r[mm] = BLD(rpW, g[m]); pW1r[mm] = BLD(rpW, g[m] + dE); pS0r[mm] = BLD(rpS, g[m]);
      pS1r[mm] = BLD(rpS, g[m] + dN);
    }
    b[m] = ACT(m) ? LDO(f.cg2d_b, g[m]) : 0.0;
    x[m] = ACT(m) ? LDO(f.cg2d_x, g[m]) : 0.0;
    s[m] = 0.0;
  }

  // cg2d.F:104-133: normalise the RHS
  double rhsMax = 0.0;
#pragma unroll
  for (int m = 0; m < PPT; m++) { b[m] = b[m] * p.cg2dNorm; rhsMax = fmax(fabs(b[m]), rhsMax); }
  rhsMax = block_max(rhsMax, red, 0);
  double rhsNorm = 1.0;
  if (p.cg2dNormaliseRHS) {
    if (rhsMax != 0.0) rhsNorm = 1.0 / rhsMax;
#pragma unroll
    for (int m = 0; m < PPT; m++) { b[m] = b[m] * rhsNorm; x[m] = x[m] * rhsNorm; }
  }
  // EXCH_XY_RL(cg2d_x): the neighbours' x values come through LDS
#pragma unroll
  for (int m = 0; m < PPT; m++) s_l[tid + m * CG_THREADS] = x[m];
  __syncthreads();
  // cg2d.F:139-180: r = b - A x ; err_sq, sumRHS
  double err = 0.0, sumB = 0.0, tq[PPT];
#pragma unroll
  for (int m = 0; m < PPT; m++) {
    r[m] = b[m] - (aW0(m) * s_l[LO(nwe[m])] + aW1(m) * s_l[HI(nwe[m])] + aS0(m) * s_l[LO(nsn[m])] +
                   aS1(m) * s_l[HI(nsn[m])] + aC(m) * x[m]);
    err = err + r[m] * r[m];
    sumB = sumB + b[m];
    tq[m] = r[m] * r[m];
    if (MINRES) xmin[MINRES ? m : 0] = x[m];
  }
#pragma unroll
  for (int m = 0; m < PPT; m++)
    if (ACT(m)) STO(f.cg2d_b, g[m]) = b[m];  // cg2d_b is INOUT (normalised in place)
  double err_sq, sumRHS;
  if (REFSUM) {
    err_sq = ref_sum<PPT>(tq, term_l, tile_l, nTilesR, tilePts);
    sumRHS = ref_sum<PPT>(b, term_l, tile_l, nTilesR, tilePts);
  } else {
    err_sq = block_sum(err, red, 1);
    sumRHS = block_sum(sumB, red, 2);
  }
  // EXCH_S3D_RL(cg2d_r): r into LDS; s_l re-zeroed for s = q + beta*s
#pragma unroll
  for (int m = 0; m < PPT; m++) { r_l[tid + m * CG_THREADS] = r[m]; s_l[tid + m * CG_THREADS] = 0.0; }
  const double firstResidual = sqrt(err_sq);
  int nIterMin = nIterMinIn;
  double minResidualSq = -1.0;
  if (MINRES && nIterMin >= 0) { nIterMin = 0; minResidualSq = err_sq; }
  int actualIts = 0;
  double eta_qrNM1 = 1.0;
  __syncthreads();
  int slot = 3;
  if (!(err_sq < p.cg2dTolerance_sq)) {
    for (int it2d = 1; it2d <= maxIters; it2d++) {
      // keep L2-resident coefficients out of VGPRs: forbid hoisting their loads
      if (CREG < 2) asm volatile("" ::: "memory");
      // q = M r ; eta_qrN = sum q*r   (cg2d.F:211-243)
      double q[PPT];
      double e = 0.0;
#pragma unroll
      for (int m = 0; m < PPT; m++) {
        q[m] = pC(m) * r[m] + pW0(m) * r_l[LO(nwe[m])] + pW1(m) * r_l[HI(nwe[m])] + pS0(m) * r_l[LO(nsn[m])] +
               pS1(m) * r_l[HI(nsn[m])];
        e = e + q[m] * r[m];
        tq[m] = q[m] * r[m];
      }
      slot = (slot + 1) & 3;
      const double eta_qrN = REFSUM ? ref_sum<PPT>(tq, term_l, tile_l, nTilesR, tilePts) : block_sum(e, red, slot);
      const double cgBeta = eta_qrN / eta_qrNM1;
      eta_qrNM1 = eta_qrN;
      // s = q + beta*s ; EXCH_S3D_RL(cg2d_s)
#pragma unroll
      for (int m = 0; m < PPT; m++) { s[m] = q[m] + cgBeta * s[m]; s_l[tid + m * CG_THREADS] = s[m]; }
      __syncthreads();
      // q = A s ; alpha = sum s*q   (cg2d.F:268-301)
      double a = 0.0;
#pragma unroll
      for (int m = 0; m < PPT; m++) {
        q[m] = aW0(m) * s_l[LO(nwe[m])] + aW1(m) * s_l[HI(nwe[m])] + aS0(m) * s_l[LO(nsn[m])] +
               aS1(m) * s_l[HI(nsn[m])] + aC(m) * s[m];
        a = a + s[m] * q[m];
        tq[m] = s[m] * q[m];
      }
      slot = (slot + 1) & 3;
      double alpha = REFSUM ? ref_sum<PPT>(tq, term_l, tile_l, nTilesR, tilePts) : block_sum(a, red, slot);
      alpha = eta_qrN / alpha;
      // x += alpha s ; r -= alpha q ; err_sq   (cg2d.F:305-328)
      double e2 = 0.0;
#pragma unroll
      for (int m = 0; m < PPT; m++) {
        x[m] = x[m] + alpha * s[m];
        r[m] = r[m] - alpha * q[m];
        e2 = e2 + r[m] * r[m];
        tq[m] = r[m] * r[m];
        r_l[tid + m * CG_THREADS] = r[m];
      }
      actualIts = it2d;
      slot = (slot + 1) & 3;
      // the barrier of either sum also publishes r_l (EXCH_S3D_RL(cg2d_r))
      err_sq = REFSUM ? ref_sum<PPT>(tq, term_l, tile_l, nTilesR, tilePts) : block_sum(e2, red, slot);
      if (err_sq < p.cg2dTolerance_sq) break;
      if (MINRES && err_sq < minResidualSq) {
        minResidualSq = err_sq;
        nIterMin = it2d;
#pragma unroll
        for (int m = 0; m < PPT; m++) xmin[MINRES ? m : 0] = x[m];
      }
    }
  }
  if (MINRES && nIterMin >= 0 && err_sq > minResidualSq) {
#pragma unroll
    for (int m = 0; m < PPT; m++) x[m] = xmin[MINRES ? m : 0];
  }
#pragma unroll
  for (int m = 0; m < PPT; m++) {
    if (p.cg2dNormaliseRHS) x[m] = x[m] / rhsNorm;
    if (ACT(m)) STO(f.cg2d_x, g[m]) = x[m];
  }
  if (tid == 0) {
    const int st = stepCounter ? *stepCounter : 0;
    SolveRecord &R = rec[st];
    R.firstResidual = firstResidual;
    R.lastResidual = sqrt(err_sq);
    R.minResidualSq = minResidualSq;
    R.rhsMax = rhsMax;
    R.sumRHS = sumRHS;
    R.numIters = actualIts;
    R.nIterMin = nIterMin;
  }
#undef LO
#undef HI
#undef ACT
#undef LDO
#undef BLD
#undef STO
#undef aW0
#undef aW1
#undef aS0
#undef aS1
#undef aC
#undef pC
#undef pW0
#undef pW1
#undef pS0
#undef pS1
}

// 2x2-blocked whole-solve CG2D (<= 4096 points): each thread owns a 2x2 block of
// mutually adjacent interior points P[b][a] (row b, column a; P[0][1] east of
// P[0][0], P[1][*] north of P[0][*]).  Blocks are formed on the global lat-lon
// index space, so a block may straddle a tile edge and odd tile sizes work as
// long as the global Nx, Ny are even; each point carries its own 2-D offset.
// The block's four in-block neighbour values come from its own registers; only
// the eight out-of-block ones (two per side) are LDS reads through the
// neighbour table, and all 32 operator coefficients of the block (aW/pW of the
// three W-E faces of each row, aS/pS of the three S-N faces of each column, aC,
// pC) stay in VGPRs (pS, pC in LDS).  No FMA contraction (built -ffp-contract=off like
// every kernel): each operator row is the reference's expression tree, so only the
// order of the global sums differs from cg2d.F.
// nb4[4*T]: packed 16-bit compact indices (W0|W1<<16), (E0|E1<<16),
// (S0|S1<<16), (N0|N1<<16); blk[4*T] = 2-D offsets of P00, P10(east), P01(north),
// P11 (T = #blocks; padding blocks: offsets of a real block, inactive).
template <bool MINRES>
__global__ void __launch_bounds__(CG_THREADS) k_cg2d_blk2(Dims d, Params p, Fields f, const unsigned *__restrict__ nb4,
                                                         const int *__restrict__ blk, int nBlk, int maxIters,
                                                         int nIterMinIn, SolveRecord *rec, int *stepCounter) {
  constexpr int NP = 4 * CG_THREADS;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double *r_l = lds;                // NP + 1 (last = ZERO slot)
  double *s_l = lds + (NP + 1);
  double *red = lds + 2 * (NP + 1);
  const int tid = threadIdx.x;
  const bool act = tid < nBlk;
  const int bt = act ? tid : 0;
  const long nx = d.nx;
  // G[b][a]: 2-D offset of point P[b][a]; compact LDS slot: tile-major, row-major in the tile
  const long G[2][2] = {{blk[4 * bt], blk[4 * bt + 1]}, {blk[4 * bt + 2], blk[4 * bt + 3]}};
  auto slot_of = [&](long gg) {
    const int tt = (int)(gg / d.n2), ll = (int)(gg % d.n2);
    return tt * d.sNx * d.sNy + (ll / d.nx - d.OLy) * d.sNx + (ll % d.nx - d.OLx);
  };
  const int c00 = act ? slot_of(G[0][0]) : NP, c10 = act ? slot_of(G[0][1]) : NP;
  const int c01 = act ? slot_of(G[1][0]) : NP, c11 = act ? slot_of(G[1][1]) : NP;
  const unsigned wW = nb4[4 * bt], wE = nb4[4 * bt + 1], wS = nb4[4 * bt + 2], wN = nb4[4 * bt + 3];
#define LO(w) ((w) & 0xFFFFu)
#define HI(w) ((w) >> 16)
  // coefficients (halo-inclusive arrays: the i0+2 / j0+2 entries may be halo values,
  // exactly what the reference reads after EXCH_UV_XY_RS / EXCH_XY_RS)
  const double az = act ? 1.0 : 0.0;
  // A (aW, aS, aC) and pW stay in VGPRs; pS and pC (10 values) live in LDS,
  // structure-of-arrays over threads (conflict-free), to stay under 128 VGPRs.
  double *pl = red + 4 * CG_WAVES;  // 10 * CG_THREADS
  double aW[2][3], pW[2][3], aS[2][3], aC[2][2];
  // W-E faces of row b: west faces of P[b][0], P[b][1], and the east face of P[b][1]
  // (its i+1 entry: the halo copy of the eastern neighbour's coefficient when P[b][1]
  // is on a tile edge, exactly what the reference reads after EXCH_UV_XY_RS)
#pragma unroll
  for (int b = 0; b < 2; b++)
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const long gw = a < 2 ? G[b][a] : G[b][1] + 1;
      const long gs = a < 2 ? G[a][b] : G[1][b] + nx;
      aW[b][a] = az * f.aW2d[gw];
      pW[b][a] = az * f.pW[gw];
      aS[b][a] = az * f.aS2d[gs];  // [column b][row a]
      pl[(b * 3 + a) * CG_THREADS + tid] = az * f.pS[gs];
    }
#pragma unroll
  for (int b = 0; b < 2; b++)
#pragma unroll
    for (int a = 0; a < 2; a++) {
      aC[b][a] = az * f.aC2d[G[b][a]];   // [row b][col a]
      pl[(6 + b * 2 + a) * CG_THREADS + tid] = az * f.pC[G[b][a]];
    }
#define pS(b, a) pl[((b) * 3 + (a)) * CG_THREADS + tid]
#define pC(b, a) pl[(6 + (b) * 2 + (a)) * CG_THREADS + tid]
  // state of the 4 points, index [row b][col a]
  double x[2][2], r[2][2], s[2][2], b_[2][2];
#pragma unroll
  for (int b = 0; b < 2; b++)
#pragma unroll
    for (int a = 0; a < 2; a++) {
      b_[b][a] = act ? f.cg2d_b[G[b][a]] : 0.0;
      x[b][a] = act ? f.cg2d_x[G[b][a]] : 0.0;
      s[b][a] = 0.0;
    }
  if (tid == 0) { r_l[NP] = 0.0; s_l[NP] = 0.0; }
  const int cs[2][2] = {{c00, c10}, {c01, c11}};

  // 5-point operator on the block: out[b][a] = sum of coef*value (reference order C?:
  // A: aW*v(i-1)+aW(i+1)*v(i+1)+aS*v(j-1)+aS(j+1)*v(j+1)+aC*v ; M: pC*v+pW*..+pS*..)
#define NEIGH(arr, v, vW0, vW1, vE0, vE1, vS0, vS1, vN0, vN1)                                              \
  const double vW0 = arr[LO(wW)], vW1 = arr[HI(wW)], vE0 = arr[LO(wE)], vE1 = arr[HI(wE)];                \
  const double vS0 = arr[LO(wS)], vS1 = arr[HI(wS)], vN0 = arr[LO(wN)], vN1 = arr[HI(wN)];
#define APPLY_A(out, v, vW0, vW1, vE0, vE1, vS0, vS1, vN0, vN1)                                            \
  out[0][0] = aW[0][0] * vW0 + aW[0][1] * v[0][1] + aS[0][0] * vS0 + aS[0][1] * v[1][0] + aC[0][0] * v[0][0]; \
  out[0][1] = aW[0][1] * v[0][0] + aW[0][2] * vE0 + aS[1][0] * vS1 + aS[1][1] * v[1][1] + aC[0][1] * v[0][1]; \
  out[1][0] = aW[1][0] * vW1 + aW[1][1] * v[1][1] + aS[0][1] * v[0][0] + aS[0][2] * vN0 + aC[1][0] * v[1][0]; \
  out[1][1] = aW[1][1] * v[1][0] + aW[1][2] * vE1 + aS[1][1] * v[0][1] + aS[1][2] * vN1 + aC[1][1] * v[1][1];
#define APPLY_M(out, v, vW0, vW1, vE0, vE1, vS0, vS1, vN0, vN1)                                            \
  out[0][0] = pC(0, 0) * v[0][0] + pW[0][0] * vW0 + pW[0][1] * v[0][1] + pS(0, 0) * vS0 + pS(0, 1) * v[1][0]; \
  out[0][1] = pC(0, 1) * v[0][1] + pW[0][1] * v[0][0] + pW[0][2] * vE0 + pS(1, 0) * vS1 + pS(1, 1) * v[1][1]; \
  out[1][0] = pC(1, 0) * v[1][0] + pW[1][0] * vW1 + pW[1][1] * v[1][1] + pS(0, 1) * v[0][0] + pS(0, 2) * vN0; \
  out[1][1] = pC(1, 1) * v[1][1] + pW[1][1] * v[1][0] + pW[1][2] * vE1 + pS(1, 1) * v[0][1] + pS(1, 2) * vN1;

  // cg2d.F:104-133: normalise the RHS
  double rhsMax = 0.0;
#pragma unroll
  for (int b = 0; b < 2; b++)
#pragma unroll
    for (int a = 0; a < 2; a++) { b_[b][a] = b_[b][a] * p.cg2dNorm; rhsMax = fmax(fabs(b_[b][a]), rhsMax); }
  rhsMax = block_max(rhsMax, red, 0);
  double rhsNorm = 1.0;
  if (p.cg2dNormaliseRHS) {
    if (rhsMax != 0.0) rhsNorm = 1.0 / rhsMax;
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int a = 0; a < 2; a++) { b_[b][a] = b_[b][a] * rhsNorm; x[b][a] = x[b][a] * rhsNorm; }
  }
  // EXCH_XY_RL(cg2d_x) through LDS
#pragma unroll
  for (int b = 0; b < 2; b++)
#pragma unroll
    for (int a = 0; a < 2; a++) s_l[cs[b][a]] = x[b][a];
  if (tid == 0) s_l[NP] = 0.0;
  __syncthreads();
  double err = 0.0, sumB = 0.0;
  {
    double ax[2][2];
    NEIGH(s_l, x, xW0, xW1, xE0, xE1, xS0, xS1, xN0, xN1)
    APPLY_A(ax, x, xW0, xW1, xE0, xE1, xS0, xS1, xN0, xN1)
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int a = 0; a < 2; a++) {
        r[b][a] = b_[b][a] - ax[b][a];
        err = err + r[b][a] * r[b][a];
        sumB = sumB + b_[b][a];
      }
  }
  double xmin[2][2];
  if (MINRES) {
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int a = 0; a < 2; a++) xmin[b][a] = x[b][a];
  }
  if (act) {
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int a = 0; a < 2; a++) f.cg2d_b[G[b][a]] = b_[b][a];
  }
  double err_sq = block_sum(err, red, 1);
  const double sumRHS = block_sum(sumB, red, 2);
#pragma unroll
  for (int b = 0; b < 2; b++)
#pragma unroll
    for (int a = 0; a < 2; a++) { r_l[cs[b][a]] = r[b][a]; s_l[cs[b][a]] = 0.0; }
  if (tid == 0) { r_l[NP] = 0.0; s_l[NP] = 0.0; }
  const double firstResidual = sqrt(err_sq);
  int nIterMin = nIterMinIn;
  double minResidualSq = -1.0;
  if (MINRES && nIterMin >= 0) { nIterMin = 0; minResidualSq = err_sq; }
  int actualIts = 0;
  double eta_qrNM1 = 1.0;
  __syncthreads();
  int slot = 3;
  if (!(err_sq < p.cg2dTolerance_sq)) {
    for (int it2d = 1; it2d <= maxIters; it2d++) {
      asm volatile("" ::: "memory");  // re-read pS/pC from LDS every iteration (no hoisting into VGPRs)
      double q[2][2];
      double e = 0.0;
      {
        NEIGH(r_l, r, rW0, rW1, rE0, rE1, rS0, rS1, rN0, rN1)
        APPLY_M(q, r, rW0, rW1, rE0, rE1, rS0, rS1, rN0, rN1)
      }
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int a = 0; a < 2; a++) e = e + q[b][a] * r[b][a];
      slot = (slot + 1) & 3;
      const double eta_qrN = block_sum(e, red, slot);
      const double cgBeta = eta_qrN / eta_qrNM1;
      eta_qrNM1 = eta_qrN;
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int a = 0; a < 2; a++) { s[b][a] = q[b][a] + cgBeta * s[b][a]; s_l[cs[b][a]] = s[b][a]; }
      __syncthreads();
      double aa = 0.0;
      {
        NEIGH(s_l, s, sW0, sW1, sE0, sE1, sS0, sS1, sN0, sN1)
        APPLY_A(q, s, sW0, sW1, sE0, sE1, sS0, sS1, sN0, sN1)
      }
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int a = 0; a < 2; a++) aa = aa + s[b][a] * q[b][a];
      slot = (slot + 1) & 3;
      double alpha = block_sum(aa, red, slot);
      alpha = eta_qrN / alpha;
      double e2 = 0.0;
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int a = 0; a < 2; a++) {
          x[b][a] = x[b][a] + alpha * s[b][a];
          r[b][a] = r[b][a] - alpha * q[b][a];
          e2 = e2 + r[b][a] * r[b][a];
          r_l[cs[b][a]] = r[b][a];
        }
      actualIts = it2d;
      slot = (slot + 1) & 3;
      err_sq = block_sum(e2, red, slot);
      if (err_sq < p.cg2dTolerance_sq) break;
      if (MINRES && err_sq < minResidualSq) {
        minResidualSq = err_sq;
        nIterMin = it2d;
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
          for (int a = 0; a < 2; a++) xmin[b][a] = x[b][a];
      }
    }
  }
  if (MINRES && nIterMin >= 0 && err_sq > minResidualSq) {
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int a = 0; a < 2; a++) x[b][a] = xmin[b][a];
  }
  if (act) {
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int a = 0; a < 2; a++) {
        double xv = x[b][a];
        if (p.cg2dNormaliseRHS) xv = xv / rhsNorm;
        f.cg2d_x[G[b][a]] = xv;
      }
  }
  if (tid == 0) {
    const int st = stepCounter ? *stepCounter : 0;
    SolveRecord &R = rec[st];
    R.firstResidual = firstResidual;
    R.lastResidual = sqrt(err_sq);
    R.minResidualSq = minResidualSq;
    R.rhsMax = rhsMax;
    R.sumRHS = sumRHS;
    R.numIters = actualIts;
    R.nIterMin = nIterMin;
  }
#undef LO
#undef HI
#undef NEIGH
#undef APPLY_A
#undef APPLY_M
#undef pS
#undef pC
}

// ---------------------------------------------------------------------------
// k_cg2d_bxy<BX, BY, NT>: the same whole-solve CG2D with BX x BY points per thread
// (i x j) and NT threads.  Fewer, fatter threads: the per-wave reduction cost
// (DPP row sums, row broadcasts, the LDS partials and the barrier) is paid by
// NT/64 waves instead of 16, more neighbours come from registers, and every
// operator coefficient of the block (aW/pW of the BX+1 W-E faces of each row,
// aS/pS of the BY+1 S-N faces of each column, aC, pC) stays in VGPRs
// (NT = 512: 2 waves per SIMD, 256 VGPRs each).  Blocks are formed on the global
// lat-lon index space as for k_cg2d_blk2; r and s live in LDS point-major
// (slot = p*NT + block, p = b*BX + a), conflict-free for the thread-contiguous
// gathers and scatters.  nbx[NB/2 per block] packs the
// 2(BX+BY) out-of-block neighbour slots as 16-bit pairs in the order
// W[0..BY-1], E[0..BY-1], S[0..BX-1], N[0..BX-1]; blkx[BX*BY per block] = the
// 2-D offsets of P[b][a] (row b = j, column a = i).
// The block sums of k_cg2d_bxy (NW waves): the pairwise tree over the wave's 64 lanes, then
// the pairwise tree over the 16 wave slots (slots >= NW are +0.0) -- the order
// mgcm_cg2d_sum_plan exports.  Cheaper evaluation of the same tree, bit for bit:
//   * wave stage: the row trees (row_sum16), then row 3 += lane 47 (row_bcast15) and
//     row 3 += lane 31 (row_bcast31) by plain DPP moves: only lane 63's value is used, so the
//     other rows' lanes may take any source and need no zeroed "old" operand; lane 63 stores
//     its own value (no readlane to a scalar and back);
//   * slot stage: every lane reads the NW slots (LDS broadcast, 16-byte reads) and adds them in
//     the tree's order in registers -- the row_sum16 of the zero-padded slots computes
//     (((s0+s1)+(s2+s3))+((s4+s5)+(s6+s7))) + (upper half) in every lane, each addition
//     commuted at most, which is exact -- instead of four DPP steps.
__device__ __forceinline__ double wave_tree63(double v) {
  v = row_sum16(v);
  v = v + dpp_f64<0x142>(v);   // lanes 48..63 += lane 47 (row 2's sum)
  v = v + dpp_f64<0x143>(v);   // lanes 48..63 += lane 31 (rows 0+1)
  return v;                    // lane 63: (r3 + r2) + (r1 + r0)
}
template <int NW>
__device__ __forceinline__ double slot_tree(const double *red_slot) {
  static_assert(NW >= 1 && NW <= 16 && (NW % 2 == 0 || NW == 1), "slot_tree: NW");
  double s[16];
#pragma unroll
  for (int q = 0; q < 16; q += 2) {
    if (q + 1 < NW) {
      const double2 w = *reinterpret_cast<const double2 *>(red_slot + q);
      s[q] = w.x; s[q + 1] = w.y;
    } else {
      s[q] = q < NW ? red_slot[q] : 0.0;
      s[q + 1] = 0.0;
    }
  }
  double t8[8], t4[4];
#pragma unroll
  for (int q = 0; q < 8; q++) t8[q] = s[2 * q] + s[2 * q + 1];
#pragma unroll
  for (int q = 0; q < 4; q++) t4[q] = t8[2 * q] + t8[2 * q + 1];
  return (t4[0] + t4[1]) + (t4[2] + t4[3]);
}
template <int NW>
__device__ __forceinline__ double block_sum_nw(double v, double *red, int slot) {
  v = wave_tree63(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 63) red[slot * 16 + wv] = v;
  __syncthreads();
  return slot_tree<NW>(red + slot * 16);
}
// two sums in one reduction (independent chains interleave), each as block_sum_nw
template <int NW>
__device__ __forceinline__ void block_sum2_nw(double &v0, double &v1, double *red, int slot) {
  v0 = row_sum16(v0);
  v1 = row_sum16(v1);
  v0 = v0 + dpp_f64<0x142>(v0);
  v1 = v1 + dpp_f64<0x142>(v1);
  v0 = v0 + dpp_f64<0x143>(v0);
  v1 = v1 + dpp_f64<0x143>(v1);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 63) { red[slot * 16 + wv] = v0; red[(slot ^ 1) * 16 + wv] = v1; }
  __syncthreads();
  v0 = slot_tree<NW>(red + slot * 16);
  v1 = slot_tree<NW>(red + (slot ^ 1) * 16);
}
// three sums in one reduction (slots 0, 1, 2), each as block_sum_nw
template <int NW>
__device__ __forceinline__ void block_sum3_nw(double &v0, double &v1, double &v2, double *red) {
  v0 = row_sum16(v0);
  v1 = row_sum16(v1);
  v2 = row_sum16(v2);
  v0 = v0 + dpp_f64<0x142>(v0);
  v1 = v1 + dpp_f64<0x142>(v1);
  v2 = v2 + dpp_f64<0x142>(v2);
  v0 = v0 + dpp_f64<0x143>(v0);
  v1 = v1 + dpp_f64<0x143>(v1);
  v2 = v2 + dpp_f64<0x143>(v2);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 63) { red[wv] = v0; red[16 + wv] = v1; red[32 + wv] = v2; }
  __syncthreads();
  v0 = slot_tree<NW>(red);
  v1 = slot_tree<NW>(red + 16);
  v2 = slot_tree<NW>(red + 32);
}
__device__ __forceinline__ double wave_max_u(double v) {
  v = row_max16(v);
  return fmax(fmax(lane_f64(v, 0), lane_f64(v, 16)), fmax(lane_f64(v, 32), lane_f64(v, 48)));
}
template <int NW>
__device__ __forceinline__ double block_max_nw(double v, double *red, int slot) {
  v = wave_max_u(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[slot * 16 + wv] = v;
  __syncthreads();
  const int l = lane & 15;
  return row_max16(l < NW ? red[slot * 16 + l] : 0.0);
}

#ifdef MGCM_CG_STAMPS   // diagnostic build only: per-phase shader-cycle totals of one solve
#define CG_NSTAMP 12
#define CG_STAMP(k)                                                                   \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    unsigned long long t_;                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
    __builtin_amdgcn_sched_barrier(0);                                                \
    if ((k) > 0) stampAcc[(k) - 1] += t_ - stampPrev;                                 \
    stampPrev = t_;                                                                   \
  } while (0)
#else
#define CG_STAMP(k) \
  do {              \
  } while (0)
#endif
// FMA: the operator rows, dot products and vector updates as fused multiply-adds in a fixed
// order (cg2dUseFMA; the oracle's device-order mode evaluates the same fma chains)
// (round 3 measured a recompute form without the barrier before the two operator
// applications -- out-of-block neighbour values re-derived from their inputs: bit-identical
// but 2.54 us/iteration against 1.82, 256 VGPRs + 29 spilled; removed in round 5)
// SR: CG2D_SR (cg2d_sr.F, useSRCGSolver) -- one standard step, then per iteration y = M r,
// v = A y and the three sums (y.r, y.v, r.r) in one reduction: three barriers per iteration
// (y, the reduction, r) instead of four; s_l holds y.
// (round 6 measured k_cg2d_hr, the same blocks with two barriers per iteration -- every
// thread advancing its own copies of the out-of-block neighbours' s and r from the q = M r and
// A s the owners publish before the reductions, aC / pC in LDS: bit-identical, 1.705 against
// 1.64 us/iteration, 20-26 VGPRs spilled; removed, profiles/r06/ab_hr_vi/)
// (round 5 measured lifting the s- and r-update barriers by re-deriving the out-of-block
// neighbours' s_n = beta*s_{n-1} + M r and r_n = r_{n-1} - alpha*A s from values published
// before the reductions: bit-identical, but the extra live values spill -- 2.89-4.30 against
// 1.64 us/iteration, profiles/r05/cg_lb/)
template <int BX, int BY, int NT, bool MINRES, bool FMA, bool SR = false>
__global__ void __launch_bounds__(NT) k_cg2d_bxy(Dims d, Params p, Fields f, const unsigned *__restrict__ nbx,
                                                 const int *__restrict__ blkx, int nBlk, int maxIters, int nIterMinIn,
                                                 SolveRecord *rec, int *stepCounter, const int *__restrict__ slot2,
                                                 const long *__restrict__ srcOf) {
  constexpr int NPT = BX * BY, NP = NPT * NT, NB = 2 * (BX + BY), NW = NT / 64;
  extern __shared__ __attribute__((aligned(16))) double lds[];
  double *r_l = lds;               // NP + 1 (last = ZERO slot)
  double *s_l = lds + (NP + 1);
  double *red = lds + 2 * (NP + 1);  // 4 x 16 partial slots
  const int tid = threadIdx.x;
  const bool act = tid < nBlk;
  const int bt = act ? tid : 0;
  const double az = act ? 1.0 : 0.0;
  long G[BY][BX];
  int cs[BY][BX];
#pragma unroll
  for (int b = 0; b < BY; b++)
#pragma unroll
    for (int a = 0; a < BX; a++) {
      G[b][a] = blkx[NPT * bt + BX * b + a];
      // point-major LDS slots (see build_nbr); an idle thread (tid >= nBlk, all its values 0)
      // keeps its own slots, which no block's neighbour table names
      cs[b][a] = (BX * b + a) * NT + tid;
    }
  unsigned nbp[NB / 2];
#pragma unroll
  for (int q = 0; q < NB / 2; q++) nbp[q] = nbx[(NB / 2) * bt + q];
  auto nbi = [&](int q) -> int { return (q & 1) ? (int)(nbp[q >> 1] >> 16) : (int)(nbp[q >> 1] & 0xFFFFu); };
  // coefficients: W-E faces of row b (a = 0..BX: west face of P[b][a], a = BX: east face of
  // P[b][BX-1], its i+1 entry), S-N faces of column a (b = 0..BY)
  double aW[BY][BX + 1], pW[BY][BX + 1], aS[BX][BY + 1], pS[BX][BY + 1], aC[BY][BX], pC[BY][BX];
  const long nx = d.nx;
#pragma unroll
  for (int b = 0; b < BY; b++)
#pragma unroll
    for (int a = 0; a <= BX; a++) {
      const long g = a < BX ? G[b][a] : G[b][BX - 1] + 1;
      aW[b][a] = az * f.aW2d[g];
      pW[b][a] = az * f.pW[g];
    }
#pragma unroll
  for (int a = 0; a < BX; a++)
#pragma unroll
    for (int b = 0; b <= BY; b++) {
      const long g = b < BY ? G[b][a] : G[BY - 1][a] + nx;
      aS[a][b] = az * f.aS2d[g];
      pS[a][b] = az * f.pS[g];
    }
#pragma unroll
  for (int b = 0; b < BY; b++)
#pragma unroll
    for (int a = 0; a < BX; a++) {
      aC[b][a] = az * f.aC2d[G[b][a]];
      pC[b][a] = az * f.pC[G[b][a]];
    }
  double x[BY][BX], r[BY][BX], sv[BY][BX], bb[BY][BX];
#pragma unroll
  for (int b = 0; b < BY; b++)
#pragma unroll
    for (int a = 0; a < BX; a++) {
      bb[b][a] = act ? f.cg2d_b[G[b][a]] : 0.0;
      x[b][a] = act ? f.cg2d_x[G[b][a]] : 0.0;
      sv[b][a] = 0.0;
    }
  // operator application: out-of-block neighbours from LDS, in-block from registers
  // (cg2d.F order: A = aW*vW + aW(i+1)*vE + aS*vS + aS(j+1)*vN + aC*v; M = pC*v + pW*vW + ...)
  auto apply_nb = [&](auto nbv, const double (&v)[BY][BX], double (&out)[BY][BX], bool isM) {
    double vW[BY], vE[BY], vS[BX], vN[BX];
#pragma unroll
    for (int b = 0; b < BY; b++) { vW[b] = nbv(nbi(b)); vE[b] = nbv(nbi(BY + b)); }
#pragma unroll
    for (int a = 0; a < BX; a++) { vS[a] = nbv(nbi(2 * BY + a)); vN[a] = nbv(nbi(2 * BY + BX + a)); }
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) {
        const double w = a > 0 ? v[b][a - 1] : vW[b];
        const double e = a < BX - 1 ? v[b][a + 1] : vE[b];
        const double so = b > 0 ? v[b - 1][a] : vS[a];
        const double no = b < BY - 1 ? v[b + 1][a] : vN[a];
        if (FMA) {   // the same terms, accumulated left to right by fma
          if (isM)
            out[b][a] = __builtin_fma(pS[a][b + 1], no, __builtin_fma(pS[a][b], so, __builtin_fma(pW[b][a + 1], e,
                                      __builtin_fma(pW[b][a], w, pC[b][a] * v[b][a]))));
          else
            out[b][a] = __builtin_fma(aC[b][a], v[b][a], __builtin_fma(aS[a][b + 1], no, __builtin_fma(aS[a][b], so,
                                      __builtin_fma(aW[b][a + 1], e, aW[b][a] * w))));
        } else if (isM)
          out[b][a] = pC[b][a] * v[b][a] + pW[b][a] * w + pW[b][a + 1] * e + pS[a][b] * so + pS[a][b + 1] * no;
        else
          out[b][a] = aW[b][a] * w + aW[b][a + 1] * e + aS[a][b] * so + aS[a][b + 1] * no + aC[b][a] * v[b][a];
      }
  };
  auto apply = [&](const double *arr, const double (&v)[BY][BX], double (&out)[BY][BX], bool isM) {
    apply_nb([&](int sl) { return arr[sl]; }, v, out, isM);
  };
  // cg2d.F:104-133: normalise the RHS
  double rhsMax = 0.0;
#pragma unroll
  for (int b = 0; b < BY; b++)
#pragma unroll
    for (int a = 0; a < BX; a++) { bb[b][a] = bb[b][a] * p.cg2dNorm; rhsMax = fmax(fabs(bb[b][a]), rhsMax); }
  rhsMax = block_max_nw<NW>(rhsMax, red, 0);
  double rhsNorm = 1.0;
  if (p.cg2dNormaliseRHS) {
    if (rhsMax != 0.0) rhsNorm = 1.0 / rhsMax;
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) { bb[b][a] = bb[b][a] * rhsNorm; x[b][a] = x[b][a] * rhsNorm; }
  }
#pragma unroll
  for (int b = 0; b < BY; b++)
#pragma unroll
    for (int a = 0; a < BX; a++) s_l[cs[b][a]] = x[b][a];
  if (tid == 0) { s_l[NP] = 0.0; r_l[NP] = 0.0; }
  __syncthreads();
  double err = 0.0, sumB = 0.0;
  {
    double ax[BY][BX];
    apply(s_l, x, ax, false);
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) {
        r[b][a] = bb[b][a] - ax[b][a];
        err = FMA ? __builtin_fma(r[b][a], r[b][a], err) : err + r[b][a] * r[b][a];
        sumB = sumB + bb[b][a];
      }
  }
  double xmin[BY][BX];
  if (MINRES) {
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) xmin[b][a] = x[b][a];
  }
  if (act) {
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) f.cg2d_b[G[b][a]] = bb[b][a];
  }
  double err_sq = block_sum_nw<NW>(err, red, 1);
  const double sumRHS = block_sum_nw<NW>(sumB, red, 2);
#pragma unroll
  for (int b = 0; b < BY; b++)
#pragma unroll
    for (int a = 0; a < BX; a++) { r_l[cs[b][a]] = r[b][a]; s_l[cs[b][a]] = 0.0; }
  if (tid == 0) { r_l[NP] = 0.0; s_l[NP] = 0.0; }
  const double firstResidual = sqrt(err_sq);
  int nIterMin = nIterMinIn;
  double minResidualSq = -1.0;
  if (MINRES && nIterMin >= 0) { nIterMin = 0; minResidualSq = err_sq; }
  int actualIts = 0;
  double eta_qrNM1 = 1.0;
  __syncthreads();
  // slots: {0,1} for the paired (err_sq of iteration n, eta_qrN of n+1) sum, 2/3 alternate
  // for alpha; the r_l writes of iteration n are fenced by an explicit barrier.  Same
  // values and the same exit test as cg2d.F:211-352, one reduction fewer per iteration.
  int aslot = 2;
  if (SR && !(err_sq < p.cg2dTolerance_sq)) {
    // the standard first step (cg2d_sr.F:190-260): y = M r, s = y, eta = y.r, q = A s
    double q[BY][BX], y[BY][BX];
    apply(r_l, r, y, true);
    double e = 0.0;
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) {
        sv[b][a] = y[b][a];
        s_l[cs[b][a]] = y[b][a];
        e = FMA ? __builtin_fma(y[b][a], r[b][a], e) : e + y[b][a] * r[b][a];
      }
    double eta_qrN = block_sum_nw<NW>(e, red, 0);   // also fences s_l
    eta_qrNM1 = eta_qrN;
    apply(s_l, sv, q, false);
    double aa = 0.0;
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) aa = FMA ? __builtin_fma(sv[b][a], q[b][a], aa) : aa + sv[b][a] * q[b][a];
    double alpha = block_sum_nw<NW>(aa, red, 1);
    double sigma = eta_qrN / alpha;
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) {
        x[b][a] = FMA ? __builtin_fma(sigma, sv[b][a], x[b][a]) : x[b][a] + sigma * sv[b][a];
        r[b][a] = FMA ? __builtin_fma(-sigma, q[b][a], r[b][a]) : r[b][a] - sigma * q[b][a];
        r_l[cs[b][a]] = r[b][a];
      }
    __syncthreads();
    bool conv = false;
    int it2d = 1;
    for (; it2d <= maxIters - 1; it2d++) {   // cg2d_sr.F:262-370
      apply(r_l, r, y, true);
#pragma unroll
      for (int b = 0; b < BY; b++)
#pragma unroll
        for (int a = 0; a < BX; a++) s_l[cs[b][a]] = y[b][a];
      __syncthreads();
      double v[BY][BX];
      apply(s_l, y, v, false);
      double eyr = 0.0, eyv = 0.0, err = 0.0;
#pragma unroll
      for (int b = 0; b < BY; b++)
#pragma unroll
        for (int a = 0; a < BX; a++) {
          eyr = FMA ? __builtin_fma(y[b][a], r[b][a], eyr) : eyr + y[b][a] * r[b][a];
          eyv = FMA ? __builtin_fma(y[b][a], v[b][a], eyv) : eyv + y[b][a] * v[b][a];
          err = FMA ? __builtin_fma(r[b][a], r[b][a], err) : err + r[b][a] * r[b][a];
        }
      block_sum3_nw<NW>(eyr, eyv, err, red);
      err_sq = err;
      if (err_sq < p.cg2dTolerance_sq) { conv = true; break; }
      if (MINRES && err_sq < minResidualSq) {
        minResidualSq = err_sq;
        nIterMin = it2d;
#pragma unroll
        for (int b = 0; b < BY; b++)
#pragma unroll
          for (int a = 0; a < BX; a++) xmin[b][a] = x[b][a];
      }
      eta_qrN = eyr;
      const double cgBeta = eta_qrN / eta_qrNM1;
      eta_qrNM1 = eta_qrN;
      alpha = eyv - (cgBeta * cgBeta) * alpha;
      sigma = eta_qrN / alpha;
#pragma unroll
      for (int b = 0; b < BY; b++)
#pragma unroll
        for (int a = 0; a < BX; a++) {
          sv[b][a] = FMA ? __builtin_fma(cgBeta, sv[b][a], y[b][a]) : y[b][a] + cgBeta * sv[b][a];
          x[b][a] = FMA ? __builtin_fma(sigma, sv[b][a], x[b][a]) : x[b][a] + sigma * sv[b][a];
          q[b][a] = FMA ? __builtin_fma(cgBeta, q[b][a], v[b][a]) : v[b][a] + cgBeta * q[b][a];
          r[b][a] = FMA ? __builtin_fma(-sigma, q[b][a], r[b][a]) : r[b][a] - sigma * q[b][a];
          r_l[cs[b][a]] = r[b][a];
        }
      __syncthreads();
    }
    if (!conv) {   // cg2d_sr.F:372-382: the residual of the last update
      double err = 0.0;
#pragma unroll
      for (int b = 0; b < BY; b++)
#pragma unroll
        for (int a = 0; a < BX; a++) err = FMA ? __builtin_fma(r[b][a], r[b][a], err) : err + r[b][a] * r[b][a];
      err_sq = block_sum_nw<NW>(err, red, 0);
    }
    actualIts = it2d;
  }
  if (!SR && !(err_sq < p.cg2dTolerance_sq)) {
    double q[BY][BX];
    apply(r_l, r, q, true);
    double e = 0.0;
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) e = FMA ? __builtin_fma(q[b][a], r[b][a], e) : e + q[b][a] * r[b][a];
    double eta_qrN = block_sum_nw<NW>(e, red, 0);
#ifdef MGCM_CG_STAMPS
    unsigned long long stampAcc[CG_NSTAMP] = {0};
    const unsigned long long stampT0 = __builtin_amdgcn_s_memtime(), stampR0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long stampPrev = stampT0;
    __builtin_amdgcn_s_waitcnt(0xC07F);
#endif
    // the standard iteration, unrolled by two: the loop-carried s and q then need no register
    // copies at the back edge (each copy of the body may hold them in the other's registers)
    auto iter = [&](int it2d) -> bool {
      const double cgBeta = eta_qrN / eta_qrNM1;
      eta_qrNM1 = eta_qrN;
#pragma unroll
      for (int b = 0; b < BY; b++)
#pragma unroll
        for (int a = 0; a < BX; a++) {
          sv[b][a] = FMA ? __builtin_fma(cgBeta, sv[b][a], q[b][a]) : q[b][a] + cgBeta * sv[b][a];
          s_l[cs[b][a]] = sv[b][a];
        }
      CG_STAMP(12);
      __syncthreads();
      CG_STAMP(1);
      apply(s_l, sv, q, false);
      double aa = 0.0;
#pragma unroll
      for (int b = 0; b < BY; b++)
#pragma unroll
        for (int a = 0; a < BX; a++) aa = FMA ? __builtin_fma(sv[b][a], q[b][a], aa) : aa + sv[b][a] * q[b][a];
      aslot = aslot ^ 1;
      CG_STAMP(2);
#ifdef MGCM_CG_STAMPS
      double alpha;
      {   // block_sum_nw, stamped: wave tree | LDS store + barrier | slot tree
        double v = wave_tree63(aa);
        CG_STAMP(6);
        if ((tid & 63) == 63) red[aslot * 16 + (tid >> 6)] = v;
        __syncthreads();
        CG_STAMP(7);
        alpha = slot_tree<NW>(red + aslot * 16);
      }
#else
      double alpha = block_sum_nw<NW>(aa, red, aslot);
#endif
      CG_STAMP(3);
      alpha = eta_qrN / alpha;
      double e2 = 0.0;
#pragma unroll
      for (int b = 0; b < BY; b++)
#pragma unroll
        for (int a = 0; a < BX; a++) {
          x[b][a] = FMA ? __builtin_fma(alpha, sv[b][a], x[b][a]) : x[b][a] + alpha * sv[b][a];
          r[b][a] = FMA ? __builtin_fma(-alpha, q[b][a], r[b][a]) : r[b][a] - alpha * q[b][a];
          e2 = FMA ? __builtin_fma(r[b][a], r[b][a], e2) : e2 + r[b][a] * r[b][a];
          r_l[cs[b][a]] = r[b][a];
        }
      actualIts = it2d;
      CG_STAMP(4);
      __syncthreads();
      CG_STAMP(8);
      // next iteration's q = M r and (q, r), reduced together with this iteration's r.r
      apply(r_l, r, q, true);
      double en = 0.0;
#pragma unroll
      for (int b = 0; b < BY; b++)
#pragma unroll
        for (int a = 0; a < BX; a++) en = FMA ? __builtin_fma(q[b][a], r[b][a], en) : en + q[b][a] * r[b][a];
      CG_STAMP(9);
      block_sum2_nw<NW>(e2, en, red, 0);
      CG_STAMP(5);
      err_sq = e2;
      eta_qrN = en;
      if (err_sq < p.cg2dTolerance_sq) return true;
      if (MINRES && err_sq < minResidualSq) {
        minResidualSq = err_sq;
        nIterMin = it2d;
#pragma unroll
        for (int b = 0; b < BY; b++)
#pragma unroll
          for (int a = 0; a < BX; a++) xmin[b][a] = x[b][a];
      }
      return false;
    };
    {
      bool done = false;
      int it2d = 1;
      for (; !done && it2d + 1 <= maxIters; it2d += 2) done = iter(it2d) || iter(it2d + 1);
      if (!done && it2d <= maxIters) iter(it2d);
    }
#ifdef MGCM_CG_STAMPS
    if (tid == 0)
      printf("CGSTAMP its %d total %llu real100MHz %llu | beta+s+store %llu barS %llu applyA+dot %llu sumA(slot tree) %llu "
             "div+upd+store %llu sum2 %llu sumA.wave %llu sumA.bar %llu barR %llu applyM+dot %llu\n",
             actualIts, __builtin_amdgcn_s_memtime() - stampT0, __builtin_amdgcn_s_memrealtime() - stampR0,
             stampAcc[11], stampAcc[0], stampAcc[1], stampAcc[2], stampAcc[3], stampAcc[4], stampAcc[5], stampAcc[6],
             stampAcc[7], stampAcc[8]);
#endif
  }
  if (MINRES && nIterMin >= 0 && err_sq > minResidualSq) {
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) x[b][a] = xmin[b][a];
  }
  if (slot2) {
    // SOLVE_FOR_PRESSURE's EXCH_XY_RL(cg2d_x) + etaN = recip_Bo*cg2d_x (k_exch_eta) as the
    // epilogue: the solution through LDS (r_l, every reader of it is past the last barrier of
    // the loop once this one is passed), then every 2-D point takes its own value or its
    // interior source's and is stored with its etaN
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) {
        double xv = x[b][a];
        if (p.cg2dNormaliseRHS) xv = xv / rhsNorm;
        if (act) r_l[cs[b][a]] = xv;
      }
    __syncthreads();
    const long n2 = d.n2 * d.nTiles;
    for (long q = tid; q < n2; q += NT) {
      const int sl = slot2[q];
      double xq;
      if (sl >= 0) xq = r_l[sl];
      else {   // neither in a block nor mapped onto one: as k_exch_eta, from global memory
        const long sq = srcOf[q];
        xq = f.cg2d_x[sq >= 0 ? sq : q];
      }
      f.cg2d_x[q] = xq;
      f.etaN[q] = f.recip_Bo[q] * xq;
    }
  } else if (act) {
#pragma unroll
    for (int b = 0; b < BY; b++)
#pragma unroll
      for (int a = 0; a < BX; a++) {
        double xv = x[b][a];
        if (p.cg2dNormaliseRHS) xv = xv / rhsNorm;
        f.cg2d_x[blkx[NPT * bt + BX * b + a]] = xv;   // re-read: G is not kept live across the solve
      }
  }
  if (tid == 0) {
    const int st = stepCounter ? *stepCounter : 0;
    SolveRecord &R = rec[st];
    R.firstResidual = firstResidual;
    R.lastResidual = sqrt(err_sq);
    R.minResidualSq = minResidualSq;
    R.rhsMax = rhsMax;
    R.sumRHS = sumRHS;
    R.numIters = actualIts;
    R.nIterMin = nIterMin;
  }
}

// Halo exchange of `nz` levels through a precomputed map (EXCH1 / EXCH2 scalar).
// map[2*h] = destination 2-D flat offset (t*n2+local), map[2*h+1] = source.
__global__ void __launch_bounds__(256) k_exchange(Dims d, double *a, const long *__restrict__ map, int nHalo, int nz) {
  const int h = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int k = (int)blockIdx.y;
  if (h >= nHalo || k >= nz) return;
  const long dst = map[2 * h], src = map[2 * h + 1];
  const long dt = dst / d.n2, dl = dst % d.n2, st = src / d.n2, sl = src % d.n2;
  const long lvl = (long)d.n2 * nz;
  a[dt * lvl + (long)k * d.n2 + dl] = a[st * lvl + (long)k * d.n2 + sl];
}

// MOMENTUM_CORRECTION_STEP over i=2-OLx..sNx+OLx, j=2-OLy..sNy+OLy, all k.
__global__ void __launch_bounds__(256) k_correction(Dims d, Params p, Fields f) {
  MG_PLANE(2 - d.OLx, d.nx - 1, 2 - d.OLy, d.ny - 1, tz)
  const int t = d.t0 + tz;
  if (i > d.sNx + d.OLx || j > d.sNy + d.OLy) return;
  const double psFac = p.pfFacMom * p.implicSurfPress;
  const long q = MG_I2(d, i, j, t);
  const double phiSurfX =
      f.recip_dxC[q] * (f.Bo_surf[q] * f.etaN[q] - f.Bo_surf[MG_I2(d, i - 1, j, t)] * f.etaN[MG_I2(d, i - 1, j, t)]);
  const double phiSurfY =
      f.recip_dyC[q] * (f.Bo_surf[q] * f.etaN[q] - f.Bo_surf[MG_I2(d, i, j - 1, t)] * f.etaN[MG_I2(d, i, j - 1, t)]);
  for (int k = 1; k <= d.Nr; k++) {
    const long q3 = MG_I3(d, i, j, k, t);
    const double mW = f.maskW[q3], mS = f.maskS[q3];
    const double gU_dpx = -psFac * phiSurfX * mW;
    const double gV_dpy = -psFac * phiSurfY * mS;
    f.uVel[q3] = (f.gU[q3] + p.deltaTMom * gU_dpx) * mW;
    f.vVel[q3] = (f.gV[q3] + p.deltaTMom * gV_dpy) * mS;
  }
}

// DO_FIELDS_BLOCKING_EXCHANGES in one launch: up to MG_XMAX fields of nz[f] levels
// through the halo map (exchange_multi_body, common.h).
__global__ void __launch_bounds__(256) k_exchange_multi(Dims d, XFields x, const long *__restrict__ map, int nHalo,
                                                        int *ctr) {
  exchange_multi_body(d, x, map, nHalo, ctr, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z);
}

// EXCH2 C-grid vector exchange (EXCH2_UV_3D_RX, pkg/exch2/exch2_uv_3d_rx.template) as one
// gather: entry h < nU writes u, the rest v; code = +-(src+1) with src indexing [u | v].
// The maps only ever source interior points, so the gather runs in place.
__global__ void __launch_bounds__(256) k_exchange_uv(Dims d, double *u, double *v, const long *__restrict__ map,
                                                     int nU, int nV) {
  const int h = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int k = (int)blockIdx.y;
  if (h >= nU + nV) return;
  const long dst = map[2 * h], code = map[2 * h + 1];
  const long N2 = d.n2 * d.nTiles, s = (code > 0 ? code : -code) - 1;
  const long lvl = (long)k * d.n2;
  auto at = [&](long g) -> long { return (g / d.n2) * d.n3 + lvl + g % d.n2; };
  // nz levels per tile: d.n3 = n2*Nr; a 2-D field is the nz = 1 case of the same layout
  const double val = s < N2 ? u[at(s)] : v[at(s - N2)];
  (h < nU ? u : v)[at(dst)] = code > 0 ? val : -val;
}

// Several 2-D C-grid vector pairs through the same map in one launch (blockIdx.y = pair):
// CALC_R_STAR's three EXCH_UV_XY_RL calls (calc_r_star.F:256-257 and the Dh/Exp pairs)
struct UVPairs {
  double *u[3], *v[3];
  int n;
};
__global__ void __launch_bounds__(256) k_exchange_uv_pairs(Dims d, UVPairs pr, const long *__restrict__ map, int nU,
                                                           int nV) {
  const int h = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int c = (int)blockIdx.y;
  if (h >= nU + nV || c >= pr.n) return;
  double *u = pr.u[c], *v = pr.v[c];
  const long dst = map[2 * h], code = map[2 * h + 1];
  const long N2 = d.n2 * d.nTiles, s = (code > 0 ? code : -code) - 1;
  const double val = s < N2 ? u[s] : v[s - N2];
  (h < nU ? u : v)[dst] = code > 0 ? val : -val;
}

// EXCH2 vector pair (u, v; nz levels, vector map) and the scalar fields x (scalar map) in one
// launch: blockIdx.z = 0 the pair, z = 1.. field z-1 (the bodies of k_exchange_uv and
// k_exchange_multi, counter bump included).  DO_FIELDS_BLOCKING_EXCHANGES on a cube/LLC
// topology and DO_STAGGER_FIELDS_EXCHANGES (u, v and w).
__global__ void __launch_bounds__(256) k_exchange_mixed(Dims d, double *u, double *v, int nzUV,
                                                        const long *__restrict__ uvMap, int nU, int nV, XFields x,
                                                        const long *__restrict__ map, int nHalo, int *ctr) {
  exchange_mixed_body(d, u, v, nzUV, uvMap, nU, nV, x, map, nHalo, ctr, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z);
}

// EXCH_XY_RL(cg2d_x) + etaN = recip_Bo*cg2d_x (solve_for_pressure.F:316, 377-385) in
// one pass over every 2-D point; srcOf[q] = interior source of halo point q, or -1.
__global__ void __launch_bounds__(256) k_exch_eta(Dims d, Fields f, const long *__restrict__ srcOf) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= d.n2 * d.nTiles) return;
  const long sq = srcOf[q];
  double x = f.cg2d_x[q];
  if (sq >= 0) { x = f.cg2d_x[sq]; f.cg2d_x[q] = x; }
  f.etaN[q] = f.recip_Bo[q] * x;
}

// exactConserv end of INTEGR_CONTINUITY: EXCH_XY_RL of the new eta (held in cg2d_b
// by k_corr_cont) into etaN, and UPDATE_ETAH (etaH = etaN) in one pass.
// Under the non-linear free surface with real fresh-water flux (not at initialisation)
// PmEpR = -EmPmR over the whole tile (integr_continuity.F:137-143) is set here too.
// fromX: SOLVE_FOR_PRESSURE's k_exch_eta was skipped (one_step), so the etaN it would have left at
// points neither interior nor mapped is formed here: recip_Bo*cg2d_x of the point.
__global__ void __launch_bounds__(256) k_exch_etaH(Dims d, Params p, Fields f, const long *__restrict__ srcOf, int atInit,
                                                   int fromX) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= d.n2 * d.nTiles) return;
  if (!atInit && p.nonlinFreeSurf > 0 && p.useRealFreshWaterFlux) f.PmEpR[q] = -f.EmPmR[q];
  const long sq = srcOf[q];
  const double *e = f.cg2d_b;
  double x;
  if (sq >= 0) x = e[sq];
  else {
    // interior: the new eta; points that are neither interior nor mapped keep etaN
    const long l = q % d.n2;
    const int i = (int)(l % d.nx) - d.OLx + 1, j = (int)(l / d.nx) - d.OLy + 1;
    x = (i >= 1 && i <= d.sNx && j >= 1 && j <= d.sNy) ? e[q] : fromX ? f.recip_Bo[q] * f.cg2d_x[q] : f.etaN[q];
  }
  f.etaHnm1[q] = f.etaH[q];   // update_etah.F:49-53: the etaH being replaced (pickup EtaH record)
  f.etaN[q] = x;
  f.etaH[q] = x;
}

// MOMENTUM_CORRECTION_STEP fused with INTEGR_CONTINUITY for one interior column:
// u, v = (u* + dt*gdPx)*mask (correction_step.F:152-234) for this column, the
// east/north neighbours' corrected velocities recomputed inline (identical
// expressions), then exactConserv's eta (into cg2d_b, see k_exch_etaH) and
// INTEGRATE_FOR_W.  Halo velocities are left to the end-of-step EXCH.
// atInit: the INTEGR_CONTINUITY call of INITIALISE_VARIA (myIter = nIter0): no
// correction (uVel, vVel as they are), dEtaHdt / PmEpR per integr_continuity.F:117-152,
// no eta update (cg2d_b = etaN, so k_exch_etaH makes etaH = etaN: UPDATE_ETAH).
// atInit = 2: INTEGR_CONTINUITY alone (the routine-level C-ABI, after a separate
// MOMENTUM_CORRECTION_STEP): divergence of uVel, vVel as they are, stepping formulas.
// r* (select_rStar > 0): w includes -rStarDhDt*drF*h0FacC (integrate_for_w.F:117-140).
// Column frame (MG_COLF): NC columns x KW level slots per workgroup, the levels of a
// column staged k-parallel into LDS and its serial parts (the exactConserv column sum, the
// upward w recurrence) run by one thread per column out of LDS; the corrected velocities go
// through LDS too, so no global store sits between a level's loads and the next level's.
// etaSrc (the step path): the surface-pressure gradient reads recip_Bo * cg2d_x at the
// exchange source of each point -- exactly the etaN that SOLVE_FOR_PRESSURE's EXCH_XY_RL +
// etaN = recip_Bo*cg2d_x (k_exch_eta) stores -- so k_exch_eta runs beside this kernel instead
// of before it (it writes only etaN and cg2d_x's halo, which this kernel then does not read).
__global__ void __launch_bounds__(256) k_corr_cont(Dims d, Params p, Fields f, int atInit, int nc,
                                                   const long *__restrict__ etaSrc) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  MG_COLF(1, d.sNx, 1, d.sNy, nc)
  const int NS = d.Nr * NC_;
  // sH0 (r* only) last: launch_corr_cont allocates it only under r*
  double *sDiv = lds, *sMask = lds + NS, *sU = lds + 2 * NS, *sV = lds + 3 * NS, *sH0 = lds + 4 * NS;
  const long q = MG_I2(d, i, j, t);
  const bool rstar = p.nonlinFreeSurf > 0 && p.select_rStar != 0;
  if (valid && atInit != 0) MG_COLF_K(k) {   // divergence of the velocities already in uVel, vVel
    const int me = (k - 1) * NC_ + cc;
    const double drF = f.drF[k - 1];
    const double u0 = f.uVel[MG_I3(d, i, j, k, t)], u1 = f.uVel[MG_I3(d, i + 1, j, k, t)];
    const double v0 = f.vVel[MG_I3(d, i, j, k, t)], v1 = f.vVel[MG_I3(d, i, j + 1, k, t)];
    const double uT1 = u1 * f.dyG[MG_I2(d, i + 1, j, t)] * drF * f.hFacW[MG_I3(d, i + 1, j, k, t)];
    const double uT0 = u0 * f.dyG[q] * drF * f.hFacW[MG_I3(d, i, j, k, t)];
    const double vT1 = v1 * f.dxG[MG_I2(d, i, j + 1, t)] * drF * f.hFacS[MG_I3(d, i, j + 1, k, t)];
    const double vT0 = v0 * f.dxG[q] * drF * f.hFacS[MG_I3(d, i, j, k, t)];
    sDiv[me] = uT1 - uT0 + vT1 - vT0;
    sMask[me] = f.maskC[MG_I3(d, i, j, k, t)];
    if (rstar) sH0[me] = f.h0FacC[MG_I3(d, i, j, k, t)];
  } else if (valid) {
    const double psFac = p.pfFacMom * p.implicSurfPress;
    auto eta = [&](long qq) {
      if (!etaSrc) return f.etaN[qq];
      const long sq = etaSrc[qq];
      return f.recip_Bo[qq] * f.cg2d_x[sq >= 0 ? sq : qq];
    };
    auto phiX = [&](int ii, int jj) {
      const long qq = MG_I2(d, ii, jj, t);
      return f.recip_dxC[qq] * (f.Bo_surf[qq] * eta(qq) - f.Bo_surf[MG_I2(d, ii - 1, jj, t)] * eta(MG_I2(d, ii - 1, jj, t)));
    };
    auto phiY = [&](int ii, int jj) {
      const long qq = MG_I2(d, ii, jj, t);
      return f.recip_dyC[qq] * (f.Bo_surf[qq] * eta(qq) - f.Bo_surf[MG_I2(d, ii, jj - 1, t)] * eta(MG_I2(d, ii, jj - 1, t)));
    };
    // the column's surface-pressure gradients (2-D, the same at every level)
    const double pX0 = phiX(i, j), pX1 = phiX(i + 1, j), pY0 = phiY(i, j), pY1 = phiY(i, j + 1);
    MG_COLF_K(k) {
      const int me = (k - 1) * NC_ + cc;
      // maskW / maskS are hFacW / hFacS != 0 at every point (ini_masks_etc.F:467-479, after the
      // hFac exchange; r* rescales hFac by positive factors): taken from the thicknesses the
      // transports read anyway -- two fewer 3-D streams
      const long q3c = MG_I3(d, i, j, k, t), q3e = MG_I3(d, i + 1, j, k, t), q3n = MG_I3(d, i, j + 1, k, t);
      const double hW0 = f.hFacW[q3c], hW1 = f.hFacW[q3e], hS0 = f.hFacS[q3c], hS1 = f.hFacS[q3n];
      auto uCor = [&](long q3, double hW, double phiSurfX) {
        const double mW = hW != 0.0 ? 1.0 : 0.0;
        return (f.gU[q3] + p.deltaTMom * (-psFac * phiSurfX * mW)) * mW;
      };
      auto vCor = [&](long q3, double hS, double phiSurfY) {
        const double mS = hS != 0.0 ? 1.0 : 0.0;
        return (f.gV[q3] + p.deltaTMom * (-psFac * phiSurfY * mS)) * mS;
      };
      const double u0 = uCor(q3c, hW0, pX0), u1 = uCor(q3e, hW1, pX1);
      const double v0 = vCor(q3c, hS0, pY0), v1 = vCor(q3n, hS1, pY1);
      sU[me] = u0;
      sV[me] = v0;
      const double drF = f.drF[k - 1];
      const double uT1 = u1 * f.dyG[MG_I2(d, i + 1, j, t)] * drF * hW1;
      const double uT0 = u0 * f.dyG[q] * drF * hW0;
      const double vT1 = v1 * f.dxG[MG_I2(d, i, j + 1, t)] * drF * hS1;
      const double vT0 = v0 * f.dxG[q] * drF * hS0;
      sDiv[me] = uT1 - uT0 + vT1 - vT0;
      sMask[me] = f.maskC[MG_I3(d, i, j, k, t)];
      if (rstar) sH0[me] = f.h0FacC[MG_I3(d, i, j, k, t)];
    }
  }
  __syncthreads();
  if (valid && kk == 0) {
    double rStarDhDt = 0.0;
    if (p.exactConserv) {
      double hDiv = 0.0;
      for (int k2 = 1; k2 <= d.Nr; k2++) hDiv = hDiv + sMask[(k2 - 1) * NC_ + cc] * sDiv[(k2 - 1) * NC_ + cc];
      double dEtaHdt;
      if (atInit == 1 && p.nIter0 != 0 && p.useRealFreshWaterFlux) {
        // integr_continuity.F:117-136: PmEpR consistent with the pickup's dEtaHdt
        dEtaHdt = f.dEtaHdt[q];
        double pm = dEtaHdt + hDiv * f.recip_rA[q];
        f.PmEpR[q] = pm * p.rhoConst;
        f.cg2d_b[q] = f.etaN[q];
      } else if (atInit == 1) {
        dEtaHdt = -(hDiv * f.recip_rA[q]);
        if (f.PmEpR) f.PmEpR[q] = 0.0;
        f.cg2d_b[q] = f.etaN[q];
      } else {
        const double facEmP = p.useRealFreshWaterFlux ? 1.0 / p.rhoConst : 0.0;   // integr_continuity.F:183-188
        dEtaHdt = -(hDiv * f.recip_rA[q]) - facEmP * f.EmPmR[q];
        f.cg2d_b[q] = f.etaH[q] + p.implicDiv2DFlow * dEtaHdt * p.deltaTFreeSurf;
      }
      if (f.dEtaHdt) f.dEtaHdt[q] = dEtaHdt;
      if (rstar) rStarDhDt = dEtaHdt * f.recip_Rcol[q];   // integr_continuity.F:171-183
    }
    double wBelow = 0.0;
    const double rA1 = f.recip_rA[q];
    for (int k2 = d.Nr; k2 >= 1; k2--) {
      const int s2 = (k2 - 1) * NC_ + cc;
      const double conv2d = -sDiv[s2];
      double w;
      if (rstar) {
        const double dh = rStarDhDt * f.drF[k2 - 1] * sH0[s2];
        if (k2 == d.Nr) w = (conv2d * rA1 - dh) * sMask[s2];
        else w = (wBelow + conv2d * rA1 - dh) * sMask[s2];
      } else if (k2 == d.Nr) {
        w = conv2d * rA1 * sMask[s2];
      } else {
        w = (wBelow + conv2d * rA1) * sMask[s2];
      }
      sDiv[s2] = w;
      wBelow = w;
    }
  }
  __syncthreads();
  if (valid) MG_COLF_K(k) {
    const int me = (k - 1) * NC_ + cc;
    const long q3 = MG_I3(d, i, j, k, t);
    f.wVel[q3] = sDiv[me];
    if (atInit == 0) { f.uVel[q3] = sU[me]; f.vVel[q3] = sV[me]; }
  }
}

// k_corr_cont as a k-march (deep grids, the step's call: atInit = 0, no r*): one thread per
// interior column walks k = Nr..1 -- INTEGRATE_FOR_W's upward order -- forming the level's
// corrected u, v (and the east / north neighbours', the same expressions), its divergence and w
// in registers and storing them at once; the exactConserv column sum runs k = 1..Nr over the
// maskC * divergence terms kept in registers (NRM slots, the unrolled loop's constant
// indices).  No LDS round trip, no serial phase with one thread in eight busy.  The column's
// operands arrive as __restrict__ parameters, so the next level's loads issue ahead of this
// level's stores.  The same expression trees as k_corr_cont: bit-identical.
template <int NR>
__device__ __forceinline__ void corr_cont_column(const Dims &d, const Params &p, long q, long q3b, long nx, long n2,
                                                 double pX0, double pX1, double pY0, double pY1, double dyG0, double dyG1,
                                                 double dxG0, double dxG1, double rA1, const double *__restrict__ gU,
                                                 const double *__restrict__ gV, const double *__restrict__ hFacW,
                                                 const double *__restrict__ hFacS, const double *__restrict__ maskC,
                                                 const double *__restrict__ drFv, double *__restrict__ uVel,
                                                 double *__restrict__ vVel, double *__restrict__ wVel, double &hDiv) {
  const double psFac = p.pfFacMom * p.implicSurfPress;
  auto uCor = [&](long q3, double hW, double phiSurfX) {
    const double mW = hW != 0.0 ? 1.0 : 0.0;
    return (gU[q3] + p.deltaTMom * (-psFac * phiSurfX * mW)) * mW;
  };
  auto vCor = [&](long q3, double hS, double phiSurfY) {
    const double mS = hS != 0.0 ? 1.0 : 0.0;
    return (gV[q3] + p.deltaTMom * (-psFac * phiSurfY * mS)) * mS;
  };
  double prod[NR];
  double wBelow = 0.0;
#pragma unroll
  for (int m = 0; m < NR; m++) {
    const int k = NR - m;
    const long q3c = q3b + (long)(k - 1) * n2, q3e = q3c + 1, q3n = q3c + nx;
    const double hW0 = hFacW[q3c], hW1 = hFacW[q3e], hS0 = hFacS[q3c], hS1 = hFacS[q3n];
    const double u0 = uCor(q3c, hW0, pX0), u1 = uCor(q3e, hW1, pX1);
    const double v0 = vCor(q3c, hS0, pY0), v1 = vCor(q3n, hS1, pY1);
    const double drF = drFv[k - 1];
    const double uT1 = u1 * dyG1 * drF * hW1;
    const double uT0 = u0 * dyG0 * drF * hW0;
    const double vT1 = v1 * dxG1 * drF * hS1;
    const double vT0 = v0 * dxG0 * drF * hS0;
    const double div = uT1 - uT0 + vT1 - vT0;
    const double mask = maskC[q3c];
    prod[m] = mask * div;
    const double conv2d = -div;
    const double w = (m == 0) ? conv2d * rA1 * mask : (wBelow + conv2d * rA1) * mask;
    wBelow = w;
    wVel[q3c] = w;
    uVel[q3c] = u0;
    vVel[q3c] = v0;
  }
  hDiv = 0.0;
#pragma unroll
  for (int m = NR - 1; m >= 0; m--) hDiv = hDiv + prod[m];
}
template <int NR>
__global__ void __launch_bounds__(256) k_corr_cont_march(Dims d, Params p, Fields f, const long *__restrict__ etaSrc) {
  const long g = (long)mg_xcd_block() * 256 + threadIdx.x;
  const long nI = (long)d.sNx * d.sNy;
  if (g >= nI * d.nT) return;
  const int t = d.t0 + (int)(g / nI), l = (int)(g % nI);
  const int i = 1 + l % d.sNx, j = 1 + l / d.sNx;
  const long q = MG_I2(d, i, j, t), nx = d.nx;
  // eta at the point and its four neighbours: the five source indices loaded together, then
  // the five values (one dependent round trip, not one per eta() evaluation)
  const long qs[5] = {q, q - 1, q + 1, q - nx, q + nx};
  double e[5];
  if (!etaSrc) {
#pragma unroll
    for (int n = 0; n < 5; n++) e[n] = f.etaN[qs[n]];
  } else {
    long sq[5];
#pragma unroll
    for (int n = 0; n < 5; n++) sq[n] = etaSrc[qs[n]];
#pragma unroll
    for (int n = 0; n < 5; n++) e[n] = f.recip_Bo[qs[n]] * f.cg2d_x[sq[n] >= 0 ? sq[n] : qs[n]];
  }
  auto phi = [&](const double *rdc, int a, int b) { return rdc[qs[a]] * (f.Bo_surf[qs[a]] * e[a] - f.Bo_surf[qs[b]] * e[b]); };
  const double pX0 = phi(f.recip_dxC, 0, 1), pX1 = phi(f.recip_dxC, 2, 0), pY0 = phi(f.recip_dyC, 0, 3),
               pY1 = phi(f.recip_dyC, 4, 0);
  const double rA1 = f.recip_rA[q];
  double hDiv;
  corr_cont_column<NR>(d, p, q, MG_I3(d, i, j, 1, t), nx, d.n2, pX0, pX1, pY0, pY1, f.dyG[q], f.dyG[q + 1], f.dxG[q],
                        f.dxG[q + nx], rA1, f.gU, f.gV, f.hFacW, f.hFacS, f.maskC, f.drF, f.uVel, f.vVel, f.wVel, hDiv);
  if (p.exactConserv) {
    const double facEmP = p.useRealFreshWaterFlux ? 1.0 / p.rhoConst : 0.0;   // integr_continuity.F:183-188
    const double dEtaHdt = -(hDiv * rA1) - facEmP * f.EmPmR[q];
    f.cg2d_b[q] = f.etaH[q] + p.implicDiv2DFlow * dEtaHdt * p.deltaTFreeSurf;
    if (f.dEtaHdt) f.dEtaHdt[q] = dEtaHdt;
  }
}

// Tile-sharded runs: gather (pack) / scatter (unpack) the halo-source points a peer
// needs, for every exchanged field and level: buf[(f*Nr + k)*n + h] <-> field at 2-D
// offset idx[h] (t*n2 + local) of level k.
__global__ void __launch_bounds__(256) k_halo_pack(Dims d, XFields x, const long *__restrict__ idx, long n,
                                                   double *__restrict__ buf, int unpack) {
  const long h = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int k = (int)blockIdx.y, fi = (int)blockIdx.z;
  if (h >= n || fi >= x.n || k >= x.nz[fi]) return;
  const long g = idx[h], t = g / d.n2, l = g % d.n2;
  double *a = x.p[fi] + t * d.n2 * x.nz[fi] + (long)k * d.n2 + l;
  double *b = buf + ((long)fi * d.Nr + k) * n + h;
  if (unpack) *a = *b;
  else *b = *a;
}

__global__ void k_bump_counter(int *c, int nIncr) {
  if (threadIdx.x == 0) { c[0] += nIncr; c[1] += 1; }
}

// ------------------------------------------------------------------ launchers
hipError_t launch_sfp_rhs(const Dims &d, const Params &p, const Fields &f, hipStream_t s) {
  const long ncol = (long)d.nx * d.ny * d.nT;
  // the k-march at BASELINE config 5's depth (round 5: LLC-90 45.5 against 63.4 us, step 1.419-1.420
  // against 1.438-1.443 ms, profiles/r05/sfp_march2/; the same march with a run-time loop kept one
  // level of loads in flight and took 138 us, profiles/r05/sfp_march/)
  if (!p.useCDscheme && d.Nr == 50) {
    hipLaunchKernelGGL(k_sfp_rhs_march<50>, dim3((unsigned)((ncol + 255) / 256)), dim3(256), 0, s, d, p, f);
    return hipGetLastError();
  }
  // mg_colf_nc's 16 columns (LLC-90: 63 us at 16, 69 at 32, 115 at 64; profiles/r04/sfpnc/,
  // where the correction pass's 32 is confirmed too)
  const int nc = mg_colf_nc(ncol, d.Nr, 4);
  MG_ALLOW_LDS(k_sfp_rhs);
  hipLaunchKernelGGL(k_sfp_rhs, dim3(mg_colf_blocks(ncol, nc)), dim3(256), mg_colf_lds(d.Nr, nc, 4), s, d, p, f, nc);
  return hipGetLastError();
}

int cg2d_block_ppt(int nPts) {
  for (int ppt = 1; ppt <= 8; ppt *= 2)
    if (nPts <= ppt * CG_THREADS) return ppt;
  return 0;
}
size_t cg2d_block_lds_bytes(int ppt) { return (size_t)(2 * (ppt * CG_THREADS + 1) + 4 * CG_WAVES) * sizeof(double); }
int cg2d_block_max_points() { return 8 * CG_THREADS; }  // LDS: 2*8193*8 B = 128 KiB

// cg2dRefOrder: the reference-order sums need NP + nTiles more doubles of LDS (PPT <= 4)
int cg2d_ref_max_points() { return 4 * CG_THREADS; }
static hipError_t launch_cg2d_ref(const Dims &d, const Params &p, const Fields &f, const unsigned *nbr, const int *gofs,
                                  int nPts, int maxIters, int nIterMin, SolveRecord *rec, int *stepCounter,
                                  hipStream_t s) {
  const int ppt = cg2d_block_ppt(nPts);
  if (!ppt || ppt > 4 || d.nTiles > nPts) return hipErrorInvalidValue;
  const size_t lds = cg2d_block_lds_bytes(ppt) + (size_t)(ppt * CG_THREADS + d.nTiles) * sizeof(double);
  const bool mr = nIterMin >= 0;
#define LAUNCH(PPT)                                                                                          \
  do {                                                                                                       \
    auto kern = mr ? k_cg2d_block<PPT, true, 0, true> : k_cg2d_block<PPT, false, 0, true>;                   \
    hipError_t e_ = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    if (e_ != hipSuccess) return e_;                                                                         \
    hipLaunchKernelGGL(kern, dim3(1), dim3(CG_THREADS), lds, s, d, p, f, nbr, gofs, nPts, maxIters, nIterMin, rec, \
                       stepCounter);                                                                         \
  } while (0)
  switch (ppt) {
    case 1: LAUNCH(1); break;
    case 2: LAUNCH(2); break;
    default: LAUNCH(4); break;
  }
#undef LAUNCH
  return hipGetLastError();
}

hipError_t launch_cg2d_block(const Dims &d, const Params &p, const Fields &f, const unsigned *nbr, const int *gofs,
                             int nPts, int maxIters, int nIterMin, SolveRecord *rec, int *stepCounter, hipStream_t s) {
  if (p.cg2dRefOrder)
    return launch_cg2d_ref(d, p, f, nbr, gofs, nPts, maxIters, nIterMin, rec, stepCounter, s);
  const int ppt = cg2d_block_ppt(nPts);
  if (!ppt) return hipErrorInvalidValue;
  const size_t lds = cg2d_block_lds_bytes(ppt);
  const bool mr = nIterMin >= 0;
#define LAUNCH(PPT)                                                                                        \
  do {                                                                                                     \
    constexpr int CR = (PPT <= 2) ? 2 : (PPT <= 4 ? 1 : 0);                                                                 \
    auto kern = mr ? k_cg2d_block<PPT, true, CR> : k_cg2d_block<PPT, false, CR>;                           \
    hipError_t e_ = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    if (e_ != hipSuccess) return e_;                                                                       \
    hipLaunchKernelGGL(kern, dim3(1), dim3(CG_THREADS), lds, s, d, p, f, nbr, gofs, nPts, maxIters, nIterMin, rec, \
                       stepCounter);                                                                       \
  } while (0)
  switch (ppt) {
    case 1: LAUNCH(1); break;
    case 2: LAUNCH(2); break;
    case 4: LAUNCH(4); break;
    default: LAUNCH(8); break;
  }
#undef LAUNCH
  return hipGetLastError();
}

// k_cg2d_bxy geometries (BX x BY points per thread, NT threads): variant v is chosen per
// grid at set-up (model.hip build_nbr: the global lat-lon index space must tile into
// BX x BY blocks, at most NT of them).  Fewer, fatter threads trade serial work per thread
// for cheaper reductions and barriers (fewer waves).
struct CgxGeom { int bx, by, nt; };
// measured on global_ocean.90x40x15 (profiles/r02/ocean90/cg2d_geometry.txt): fatter threads
// (3x4, 5x4, 3x8, 5x8) spill the per-point registers and run 1.5-8x slower per iteration
static const CgxGeom CGX[] = {{2, 4, 512}, {2, 2, 1024}};
constexpr int CGX_N = (int)(sizeof(CGX) / sizeof(CGX[0]));
int cg2d_bxy_variants() { return CGX_N; }
int cg2d_bxy_geometry(int v, int *bx, int *by, int *nt) {
  if (v < 0 || v >= CGX_N) return -1;
  *bx = CGX[v].bx; *by = CGX[v].by; *nt = CGX[v].nt;
  return 0;
}
template <int BX, int BY, int NT>
static hipError_t launch_bxy_t(const Dims &d, const Params &p, const Fields &f, const unsigned *nbx, const int *blkx,
                               int nBlk, int maxIters, int nIterMin, SolveRecord *rec, int *stepCounter, const int *slot2,
                               const long *srcOf, hipStream_t s) {
  if (nBlk > NT) return hipErrorInvalidValue;
  const bool mr = nIterMin >= 0, fm = p.cg2dUseFMA != 0, sr = p.useSRCGSolver != 0;
  const size_t lds = (2 * ((size_t)BX * BY * NT + 1) + 4 * 16) * sizeof(double);
  auto kern = sr   ? (mr ? (fm ? k_cg2d_bxy<BX, BY, NT, true, true, true> : k_cg2d_bxy<BX, BY, NT, true, false, true>)
                         : (fm ? k_cg2d_bxy<BX, BY, NT, false, true, true>
                               : k_cg2d_bxy<BX, BY, NT, false, false, true>))
              : (mr ? (fm ? k_cg2d_bxy<BX, BY, NT, true, true> : k_cg2d_bxy<BX, BY, NT, true, false>)
                         : (fm ? k_cg2d_bxy<BX, BY, NT, false, true> : k_cg2d_bxy<BX, BY, NT, false, false>));
  static bool attrSet[8] = {false, false, false, false, false, false, false, false};
  const int ai = 4 * sr + 2 * mr + fm;
  if (!attrSet[ai]) {
    hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attrSet[ai] = true;
  }
  hipLaunchKernelGGL(kern, dim3(1), dim3(NT), lds, s, d, p, f, nbx, blkx, nBlk, maxIters, nIterMin, rec, stepCounter, slot2,
                     srcOf);
  return hipGetLastError();
}
// slot2 (or nullptr): the 2-D point -> LDS slot map of the fused EXCH(cg2d_x) + etaN epilogue
hipError_t launch_cg2d_bxy(int v, const Dims &d, const Params &p, const Fields &f, const unsigned *nbx, const int *blkx,
                           int nBlk, int maxIters, int nIterMin, SolveRecord *rec, int *stepCounter, const int *slot2,
                           const long *srcOf, hipStream_t s) {
#define CGX_CASE(V, BX, BY, NT) \
  case V: return launch_bxy_t<BX, BY, NT>(d, p, f, nbx, blkx, nBlk, maxIters, nIterMin, rec, stepCounter, slot2, srcOf, s);
  switch (v) {
    CGX_CASE(0, 2, 4, 512)
    CGX_CASE(1, 2, 2, 1024)
  }
#undef CGX_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_cg2d_blk2(const Dims &d, const Params &p, const Fields &f, const unsigned *nb4, const int *blk,
                            int nBlk, int maxIters, int nIterMin, SolveRecord *rec, int *stepCounter, hipStream_t s) {
  if (nBlk > CG_THREADS) return hipErrorInvalidValue;
  const size_t lds = cg2d_block_lds_bytes(4) + 10 * CG_THREADS * sizeof(double);  // 146 KiB
  auto kern = nIterMin >= 0 ? k_cg2d_blk2<true> : k_cg2d_blk2<false>;
  static bool attrSet[2] = {false, false};   // once per instantiation (not a stream op; keeps graph capture clean)
  if (!attrSet[nIterMin >= 0]) {
    hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    attrSet[nIterMin >= 0] = true;
  }
  hipLaunchKernelGGL(kern, dim3(1), dim3(CG_THREADS), lds, s, d, p, f, nb4, blk, nBlk, maxIters, nIterMin, rec,
                     stepCounter);
  return hipGetLastError();
}

hipError_t launch_exchange(const Dims &d, double *a, const long *map, int nHalo, int nz, hipStream_t s) {
  if (nHalo <= 0) return hipSuccess;
  dim3 blk(256), grd((nHalo + 255) / 256, nz);
  hipLaunchKernelGGL(k_exchange, grd, blk, 0, s, d, a, map, nHalo, nz);
  return hipGetLastError();
}

hipError_t launch_correction(const Dims &d, const Params &p, const Fields &f, hipStream_t s) {
  const dim3 blk(MG_PLANE_THREADS), grd(mg_plane_blocks(d.nx - 1, d.ny - 1, d.nT));
  hipLaunchKernelGGL(k_correction, grd, blk, 0, s, d, p, f);
  return hipGetLastError();
}

hipError_t launch_exchange_multi(const Dims &d, const XFields &x, const long *map, int nHalo, int *ctr, hipStream_t s) {
  int nzMax = 1;
  for (int q = 0; q < x.n; q++) nzMax = x.nz[q] > nzMax ? x.nz[q] : nzMax;
  dim3 blk(256), grd((unsigned)((nHalo > 0 ? nHalo : 1) + 255) / 256, nzMax, x.n);
  hipLaunchKernelGGL(k_exchange_multi, grd, blk, 0, s, d, x, map, nHalo, ctr);
  return hipGetLastError();
}

hipError_t launch_exchange_mixed(const Dims &d, double *u, double *v, int nzUV, const long *uvMap, int nU, int nV,
                                 const XFields &x, const long *map, int nHalo, int *ctr, hipStream_t s) {
  int nzMax = nzUV;
  for (int q = 0; q < x.n; q++) nzMax = x.nz[q] > nzMax ? x.nz[q] : nzMax;
  const int nh = (nU + nV) > nHalo ? nU + nV : nHalo;
  dim3 blk(256), grd((unsigned)((nh > 0 ? nh : 1) + 255) / 256, nzMax, 1 + x.n);
  hipLaunchKernelGGL(k_exchange_mixed, grd, blk, 0, s, d, u, v, nzUV, uvMap, nU, nV, x, map, nHalo, ctr);
  return hipGetLastError();
}

hipError_t launch_exchange_uv(const Dims &d, double *u, double *v, const long *map, int nU, int nV, int nz,
                              hipStream_t s) {
  if (nU + nV <= 0) return hipSuccess;
  Dims dz = d;
  dz.n3 = d.n2 * nz;   // per-tile stride of an nz-level field
  hipLaunchKernelGGL(k_exchange_uv, dim3((unsigned)((nU + nV + 255) / 256), nz), dim3(256), 0, s, dz, u, v, map, nU,
                     nV);
  return hipGetLastError();
}

hipError_t launch_exchange_uv_pairs(const Dims &d, double *const *u, double *const *v, int n, const long *map, int nU,
                                   int nV, hipStream_t s) {
  if (nU + nV <= 0 || n <= 0) return hipSuccess;
  if (n > 3) return hipErrorInvalidValue;
  UVPairs pr{};
  for (int c = 0; c < n; c++) { pr.u[c] = u[c]; pr.v[c] = v[c]; }
  pr.n = n;
  hipLaunchKernelGGL(k_exchange_uv_pairs, dim3((unsigned)((nU + nV + 255) / 256), n), dim3(256), 0, s, d, pr, map, nU,
                     nV);
  return hipGetLastError();
}

hipError_t launch_exch_eta(const Dims &d, const Params &p, const Fields &f, const long *srcOf, bool etaH, int atInit,
                           hipStream_t s, int fromX) {
  const long n = d.n2 * d.nTiles;
  if (etaH) hipLaunchKernelGGL(k_exch_etaH, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, p, f, srcOf, atInit, fromX);
  else hipLaunchKernelGGL(k_exch_eta, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, f, srcOf);
  return hipGetLastError();
}

hipError_t launch_corr_cont(const Dims &d, const Params &p, const Fields &f, int atInit, hipStream_t s,
                            const long *etaSrc) {
  const long ncol = (long)d.sNx * d.sNy * d.nT;
  const int nArr = (p.nonlinFreeSurf > 0 && p.select_rStar != 0) ? 5 : 4;   // sH0 under r* only
  // deep grids: 32 columns per workgroup (LLC-90: 123 us against 140 at 16,
  // profiles/r03/colfnc/); shallow: 16 (config 2: 0.328-0.331 ms/step against 0.333 at 32,
  // profiles/r03/ab_trex_corrnc/)
  // the k-march at BASELINE config 5's depth (round 5: LLC-90 1.445 against 1.475-1.481 ms/step
  // for the frame, alternating on one box, profiles/r05/corr_march/)
  if (atInit == 0 && !(p.nonlinFreeSurf > 0 && p.select_rStar != 0) && d.Nr == 50) {
    // (levels one at a time: loading batches of 5 or 10 levels ahead measured slower, 103
    // against 87 us, profiles/r05/corr_sb/)
    hipLaunchKernelGGL(k_corr_cont_march<50>, dim3((unsigned)((ncol + 255) / 256)), dim3(256), 0, s, d, p, f, etaSrc);
    return hipGetLastError();
  }
  const int nc = d.Nr >= 30 ? 32 : 16;
  // (round 4: a two-column form with 16-byte loads was bit-identical but slower on LLC-90,
  // 151 against 137 us, profiles/r04/corr2/ -- the column frame is bound by its serial column
  // sums and LDS round trips, not by the width of its loads; removed in round 5)
  MG_ALLOW_LDS(k_corr_cont);
  hipLaunchKernelGGL(k_corr_cont, dim3(mg_colf_blocks(ncol, nc)), dim3(256), mg_colf_lds(d.Nr, nc, nArr), s, d, p, f,
                     atInit, nc, etaSrc);
  return hipGetLastError();
}

hipError_t launch_halo_pack(const Dims &d, const XFields &x, const long *idx, long n, double *buf, int unpack,
                            hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_halo_pack, dim3((unsigned)((n + 255) / 256), d.Nr, x.n), dim3(256), 0, s, d, x, idx, n, buf,
                     unpack);
  return hipGetLastError();
}

hipError_t launch_bump_counter(int *c, int nIncr, hipStream_t s) {
  hipLaunchKernelGGL(k_bump_counter, dim3(1), dim3(64), 0, s, c, nIncr);
  return hipGetLastError();
}

}  // namespace mgcm
