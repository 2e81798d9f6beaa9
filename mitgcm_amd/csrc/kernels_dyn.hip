// kernels_dyn.hip -- DYNAMICS on the MI355X: MOM_FLUXFORM + TIMESTEP + AB2 fused.
//
// Reference: model/src/dynamics.F:21-739 (k-loop :422-567),
//            pkg/mom_fluxform/mom_fluxform.F:42-1064,
//            model/src/timestep.F:10-429, model/src/adams_bashforth2.F:6-92.
//
// k_phi_hyd integrates CALC_PHI_HYD down each column (a k-scan, one thread per
// column) into phiHydC.  k_mom_step then runs one thread per (i,j,k) point: the
// vertical advective fluxes of both faces of the level (the fVerU/fVerV(kUp/kDown)
// ping-pong of dynamics.F:428-431) and every horizontal face flux that the
// reference keeps in 2-D scratch arrays (fZon, fMer, ...) are re-derived from the
// neighbours' state with the same expression and operand order, so each point is
// bit-identical to the loop-nest form (compiled with -ffp-contract=off).  The
// kernel is HBM/latency bound (about 1 flop/B): no MFMA.
#include <cstdlib>

#include "common.h"
#include "phys.h"
#include <cstring>
#include <cstdio>
#include <type_traits>

namespace mgcm {

// hFacZ (pkg/mom_common/mom_calc_hfacz.F:158-225, hZoption = 0)
__device__ __forceinline__ double hfacz(const Dims &d, const Fields &f, int i, int j, int k, int t) {
  if (i < 2 - d.OLx || j < 2 - d.OLy) return 0.0;
  double h = fmin(f.hFacW[MG_I3(d, i, j, k, t)], f.hFacW[MG_I3(d, i, j - 1, k, t)]);
  h = fmin(f.hFacS[MG_I3(d, i, j, k, t)], h);
  h = fmin(f.hFacS[MG_I3(d, i - 1, j, k, t)], h);
  return h;
}

// h0FacZ (mom_fluxform.F:290-307): from the rest-state h0FacW/S under the non-linear
// free surface with no-slip walls, else hFacZ
__device__ __forceinline__ double h0facz(const Dims &d, const Params &p, const Fields &f, int i, int j, int k, int t) {
  if (!(p.momViscosity && p.no_slip_sides && p.nonlinFreeSurf > 0)) return hfacz(d, f, i, j, k, t);
  if (i < 2 - d.OLx || j < 2 - d.OLy) return 0.0;
  return fmin(fmin(f.h0FacW[MG_I3(d, i, j, k, t)], f.h0FacW[MG_I3(d, i, j - 1, k, t)]),
              fmin(f.h0FacS[MG_I3(d, i, j, k, t)], f.h0FacS[MG_I3(d, i - 1, j, k, t)]));
}

// MOM_U_DEL2U / MOM_V_DEL2V (pkg/mom_fluxform/mom_u_del2u.F:59-117, mom_v_del2v.F:59-117,
// cosFac = 1, no OBCS) for one (i,j,k) of 2-OL..sN+OL-1 (0 elsewhere, as the zeroed v4F):
// the Laplacians of u and v the biharmonic viscous fluxes difference, with the no-slip
// side-wall term from the rest-state h0Fac (NONLIN_FRSURF).
__device__ __forceinline__ void del2uv_body(const Dims &d, const Params &p, const Fields &f, int lb) {
  MG_PLANE_LB(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, z, lb)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  const long q3 = MG_I3(d, i, j, k, t);
  if (i < 2 - d.OLx || i > d.sNx + d.OLx - 1 || j < 2 - d.OLy || j > d.sNy + d.OLy - 1) {
    f.del2u[q3] = 0.0;
    f.del2v[q3] = 0.0;
    return;
  }
  const double drF = f.drF[k - 1];
#define U(ii, jj) f.uVel[MG_I3(d, ii, jj, k, t)]
#define V(ii, jj) f.vVel[MG_I3(d, ii, jj, k, t)]
#define G2(a, ii, jj) f.a[MG_I2(d, ii, jj, t)]
#define G3(a, ii, jj) f.a[MG_I3(d, ii, jj, k, t)]
  {
    auto fz = [&](int ii) { return drF * G3(hFacC, ii, j) * G2(dyF, ii, j) * G2(recip_dxF, ii, j) * (U(ii + 1, j) - U(ii, j)) * 1.0; };
    auto fm = [&](int jj) {
      return drF * hfacz(d, f, i, jj, k, t) * G2(dxV, i, jj) * G2(recip_dyU, i, jj) * (U(i, jj) - U(i, jj - 1));
    };
    double v4 = f.recip_drF[k - 1] * G3(recip_hFacW, i, j) * G2(recip_rAw, i, j) *
                (fz(i) - fz(i - 1) + fm(j + 1) - fm(j)) * G3(maskW, i, j);
    if (p.no_slip_sides) {
      const double hS = G3(h0FacW, i, j) - h0facz(d, p, f, i, j, k, t);
      const double hN = G3(h0FacW, i, j) - h0facz(d, p, f, i, j + 1, k, t);
      v4 = v4 - G3(recip_hFacW, i, j) * G2(recip_rAw, i, j) *
                    (hS * G2(dxV, i, j) * G2(recip_dyU, i, j) + hN * G2(dxV, i, j + 1) * G2(recip_dyU, i, j + 1)) * U(i, j) *
                    p.sideDragFactor * G3(maskW, i, j);
    }
    f.del2u[q3] = v4;
  }
  {
    auto fz = [&](int ii) {
      return drF * hfacz(d, f, ii, j, k, t) * G2(dyU, ii, j) * G2(recip_dxV, ii, j) * (V(ii, j) - V(ii - 1, j)) * 1.0;
    };
    auto fm = [&](int jj) { return drF * G3(hFacC, i, jj) * G2(dxF, i, jj) * G2(recip_dyF, i, jj) * (V(i, jj + 1) - V(i, jj)); };
    double v4 = f.recip_drF[k - 1] * G3(recip_hFacS, i, j) * G2(recip_rAs, i, j) *
                (fz(i + 1) - fz(i) + fm(j) - fm(j - 1)) * G3(maskS, i, j);
    if (p.no_slip_sides) {
      const double hW = G3(h0FacS, i, j) - h0facz(d, p, f, i, j, k, t);
      const double hE = G3(h0FacS, i, j) - h0facz(d, p, f, i + 1, j, k, t);
      v4 = v4 - G3(recip_hFacS, i, j) * G2(recip_rAs, i, j) *
                    (hW * G2(dyU, i, j) * G2(recip_dxV, i, j) + hE * G2(dyU, i + 1, j) * G2(recip_dxV, i + 1, j)) * V(i, j) *
                    p.sideDragFactor * G3(maskS, i, j);
    }
    f.del2v[q3] = v4;
  }
#undef U
#undef V
#undef G2
#undef G3
}
__global__ void __launch_bounds__(256) k_del2uv(Dims d, Params p, Fields f) { del2uv_body(d, p, f, mg_xcd_block()); }

// CALC_PHI_HYD (calc_phi_hyd.F:175-327, OCEANIC, integr_GeoPot = 2, uniformFreeSurfLev,
// gravFac = 1) per column, as the other column kernels (MG_COLF): alphaRho = rhoInSitu
// plus MOM_QUASIHYDROSTATIC's 3-D Coriolis / NH-metric buoyancy (mom_quasihydrostatic.F:
// 76-147, angleCosC = 1, angleSinC = 0) and the two half-level increments are formed
// k-parallel into LDS, one thread per column runs the reference's sequential sum, and
// phiHydC, DIAGS_PHI_HYD's totPhiHyd (diags_phi_hyd.F:60-120, phi0surf = 0) and alphaRho
// (for CALC_GRAD_PHI_HYD's r* term) are stored k-parallel.  Under r* the same column pass
// runs MOM_CALC_RTRANS's dWtransC/U/V recurrences (mom_calc_rtrans.F:91-137) and keeps
// their value at every level for k_mom_step.  Columns cover -1..sNx+1 x -1..sNy+1 (the
// dynamics range 0..sNx+1 plus the west/south neighbours dWtransC is needed at); phi and
// totPhiHyd are stored on 0..sNx+1 only.
// PHYS: DO_OCEANIC_PHYS's per-point work (phys.h) done in the same column pass, whose frame
// then covers the whole halo range (the range DO_OCEANIC_PHYS fills); the rho each point
// computes feeds the phi_hyd sums directly and the phi_hyd stores keep to -1..sN+1 / 0..sN+1
// (k_phys_phi: DO_OCEANIC_PHYS and CALC_PHI_HYD in one launch where nothing between them
// reads DO_OCEANIC_PHYS's output at a neighbour -- no GM/Redi tensor -- and phi is not
// already fused with del2uv)
template <bool PHYS = false>
__device__ __forceinline__ void phi_hyd_body(const Dims &d, const Params &p, const Fields &f, int nc, int lb,
                                             const int *iterPtr = nullptr) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  MG_COLF_LB(PHYS ? 1 - d.OLx : -1, PHYS ? d.nx : d.sNx + 3, PHYS ? 1 - d.OLy : -1, PHYS ? d.ny : d.sNy + 3, nc, lb)
  const int Nr = d.Nr, NS = Nr * NC_;
  double *sM = lds, *sP = lds + NS, *sPh = lds + 2 * NS, *sC = lds + 3 * NS, *sU = lds + 4 * NS, *sV = lds + 5 * NS;
  const bool qh = p.quasiHydrostatic && (p.select3dCoriScheme >= 1 || p.useNHMTerms);
  const bool rstar = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
  const bool inPhi = !PHYS || (i >= -1 && i <= d.sNx + 1 && j >= -1 && j <= d.sNy + 1);
  const bool ring = inPhi && i >= 0 && j >= 0;
  const double recip_rhoConst = 1.0 / p.rhoConst;
  const long q2 = MG_I2(d, i, j, t);
  if (valid) MG_COLF_K(k) {
    const int me = (k - 1) * NC_ + cc;
    double dRlocM = 0.5 * f.drC[k - 1];
    if (k == 1) dRlocM = f.rF[0] - f.rC[0];
    const double dRlocP = (k == Nr) ? (f.rC[k - 1] - f.rF[k]) : 0.5 * f.drC[k];
    const long q3 = MG_I3(d, i, j, k, t);
    double a;
    if constexpr (PHYS) a = oceanic_phys_point(d, p, f, iterPtr, i, j, k, t);
    else a = f.rhoInSitu[q3];
    if (qh) {
      const double scalingFactor = p.rhoConst * p.gravitySign * (1.0 / p.gravity);
      const double u0 = f.uVel[q3], u1 = f.uVel[MG_I3(d, i + 1, j, k, t)];
      const double v0 = f.vVel[q3], v1 = f.vVel[MG_I3(d, i, j + 1, k, t)];
      double gW = 0.0;
      if (p.select3dCoriScheme >= 1) gW = f.fCoriCos[q2] * (1.0 * 0.5 * (u0 + u1) - 0.0 * 0.5 * (v0 + v1));
      if (p.useNHMTerms) gW = gW + ((u0 * u0 + u1 * u1) + (v0 * v0 + v1 * v1)) * 0.5 * p.recip_rSphere;
      a = a + scalingFactor * gW;
    }
    if (rstar && inPhi) f.alphaRho[q3] = a;
    sM[me] = dRlocM * p.gravity * a * recip_rhoConst;
    sP[me] = dRlocP * p.gravity * a * recip_rhoConst;
    if (rstar) {
      const double drF = f.drF[k - 1];
      sC[me] = f.rStarDhCDt[q2] * drF * f.h0FacC[q3] * f.rA[q2];
      if (ring) {
        sU[me] = f.rStarDhWDt[q2] * drF * f.h0FacW[q3] * f.rAw[q2];
        sV[me] = f.rStarDhSDt[q2] * drF * f.h0FacS[q3] * f.rAs[q2];
      }
    }
  }
  __syncthreads();
  if (valid && kk == 0) {
    double phF = 0.0;
    for (int k2 = 1; k2 <= Nr; k2++) {
      const int s2 = (k2 - 1) * NC_ + cc;
      const double phC = phF + sM[s2];
      phF = phC + sP[s2];
      sPh[s2] = phC;
    }
    if (rstar) {
      auto d0 = [&](long r) { return f.rStarDhCDt[r] * (f.Ro_surf[r] - f.R_low[r]) * f.rA[r]; };
      double c = d0(q2);
      double u = ring ? 0.5 * (d0(q2 - 1) + c) : 0.0, v = ring ? 0.5 * (d0(q2 - d.nx) + c) : 0.0;
      for (int k2 = 1; k2 <= Nr; k2++) {   // value seen by MOM_CALC_RTRANS(k2): levels 1..k2-1 removed
        const int s2 = (k2 - 1) * NC_ + cc;
        const double cc2 = sC[s2];
        sC[s2] = c;
        c = c - cc2;
        if (ring) {
          const double uu = sU[s2], vv = sV[s2];
          sU[s2] = u;
          sV[s2] = v;
          u = u - uu;
          v = v - vv;
        }
      }
    }
  }
  __syncthreads();
  if (valid) MG_COLF_K(k) {
    const int me = (k - 1) * NC_ + cc;
    const long q3 = MG_I3(d, i, j, k, t);
    if (rstar && inPhi) {
      f.dWtC[q3] = sC[me];
      if (ring) { f.dWtU[q3] = sU[me]; f.dWtV[q3] = sV[me]; }
    }
    if (ring) {
      const double phC = sPh[me];
      f.phiHydC[q3] = phC;
      if (p.storePhiHyd4Phys) {
        double tot;
        if (rstar && p.nonlinFreeSurf >= 4) {
          const double dPhiRef = (f.Ro_surf[q2] - f.rC[k - 1]) * p.gravity;
          tot = phC * f.rStarFacC[q2] + fmax(dPhiRef, 0.0) * (f.rStarFacC[q2] - 1.0) + 0.0;
        } else {
          tot = phC + f.Bo_surf[q2] * f.etaN[q2] + 0.0;
        }
        f.totPhiHyd[q3] = tot;
      }
    }
  }
}
__global__ void __launch_bounds__(256) k_phi_hyd(Dims d, Params p, Fields f, int nc) {
  phi_hyd_body(d, p, f, nc, mg_xcd_block());
}
// CALC_PHI_HYD as a flat per-column pass (phi_hyd_body's non-PHYS cases; RS = r*, QH = the
// quasi-hydrostatic buoyancy terms): one thread per column, consecutive threads along i,
// over phi_hyd_body's columns (-1..sN+1 under r*, whose dWtrans the west/south neighbours
// need; 0..sN+1 otherwise).  The column's operands are fetched PHI_CH levels at a time, every
// load of a chunk in flight before the chunk's sequential sums, and each level's results
// stored as the sums pass -- no LDS staging, no barrier, no thread idle while one thread per
// column sums.  The same expressions in the same order as phi_hyd_body: bit-identical.
constexpr int PHI_CH = 10;   // levels per chunk (5 with the r* / QH operands)
template <bool RS, bool QH, int NRC = 0>
__device__ __forceinline__ void phi_flat_body(const Dims &d, const Params &p, const Fields &f, int lb) {
  constexpr int o = RS ? 1 : 0;
  const int W = d.sNx + 2 + o, H = d.sNy + 2 + o;
  const long col = (long)lb * 256 + threadIdx.x, npl = (long)W * H;
  if (col >= npl * d.nT) return;
  const int t = d.t0 + (int)(col / npl), r = (int)(col % npl);
  const int i = r % W - o, j = r / W - o;
  const bool ring = i >= 0 && j >= 0;
  const int Nr = NRC > 0 ? NRC : d.Nr;   // NRC: the depth as a constant (the chunk loop unrolled)
  constexpr int CH = (RS || QH) ? 5 : PHI_CH;   // (8 operand arrays per level under r* + QH)
  const double recip_rhoConst = 1.0 / p.rhoConst;
  const double scalingFactor = p.rhoConst * p.gravitySign * (1.0 / p.gravity);
  const long q2 = MG_I2(d, i, j, t);
  // MOM_CALC_RTRANS's recurrences (phi_hyd_body: d0 and the k2 loop)
  double c = 0.0, u = 0.0, v = 0.0, dCdt = 0.0, dWdt = 0.0, dSdt = 0.0, rA = 0.0, rAw = 0.0, rAs = 0.0;
  if (RS) {
    auto d0 = [&](long rr) { return f.rStarDhCDt[rr] * (f.Ro_surf[rr] - f.R_low[rr]) * f.rA[rr]; };
    c = d0(q2);
    u = ring ? 0.5 * (d0(q2 - 1) + c) : 0.0;
    v = ring ? 0.5 * (d0(q2 - d.nx) + c) : 0.0;
    dCdt = f.rStarDhCDt[q2]; rA = f.rA[q2];
    if (ring) { dWdt = f.rStarDhWDt[q2]; dSdt = f.rStarDhSDt[q2]; rAw = f.rAw[q2]; rAs = f.rAs[q2]; }
  }
  const bool tot = p.storePhiHyd4Phys && ring;
  const bool totR = RS && p.nonlinFreeSurf >= 4;
  const double bEta = tot && !totR ? f.Bo_surf[q2] * f.etaN[q2] : 0.0;
  const double fac = tot && totR ? f.rStarFacC[q2] : 0.0, roS = tot && totR ? f.Ro_surf[q2] : 0.0;
  const double fCos = QH ? f.fCoriCos[q2] : 0.0;
  double phF = 0.0;
  auto chunk = [&](const int k0) {
    double a[CH], u0[CH], u1[CH], v0[CH], v1[CH], hC[CH], hW[CH], hS[CH], dM[CH], dP[CH];
#pragma unroll
    for (int cc = 0; cc < CH; cc++) {
      const int k = k0 + cc <= Nr ? k0 + cc : Nr;   // (clamped: the extra levels are not used)
      const long q3 = MG_I3(d, i, j, k, t);
      a[cc] = f.rhoInSitu[q3];
      if constexpr (NRC > 0) {
        // at a constant depth the level's half-cell thicknesses are fetched with the chunk's
        // operands: a 1-D load between the level's stores would wait for them (vmcnt counts
        // stores too)
        dM[cc] = (k == 1) ? f.rF[0] - f.rC[0] : 0.5 * f.drC[k - 1];
        dP[cc] = (k == Nr) ? (f.rC[k - 1] - f.rF[k]) : 0.5 * f.drC[k];
      }
      if (QH) {
        u0[cc] = f.uVel[q3]; u1[cc] = f.uVel[MG_I3(d, i + 1, j, k, t)];
        v0[cc] = f.vVel[q3]; v1[cc] = f.vVel[MG_I3(d, i, j + 1, k, t)];
      }
      if (RS) {
        hC[cc] = f.h0FacC[q3];
        if (ring) { hW[cc] = f.h0FacW[q3]; hS[cc] = f.h0FacS[q3]; }
      }
    }
#pragma unroll
    for (int cc = 0; cc < CH; cc++) {
      const int k = k0 + cc;
      if (k > Nr) continue;
      const long q3 = MG_I3(d, i, j, k, t);
      double dRlocM, dRlocP;
      if constexpr (NRC > 0) {
        dRlocM = dM[cc];
        dRlocP = dP[cc];
      } else {
        dRlocM = 0.5 * f.drC[k - 1];
        if (k == 1) dRlocM = f.rF[0] - f.rC[0];
        dRlocP = (k == Nr) ? (f.rC[k - 1] - f.rF[k]) : 0.5 * f.drC[k];
      }
      double al = a[cc];
      if (QH) {
        double gW = 0.0;
        if (p.select3dCoriScheme >= 1) gW = fCos * (1.0 * 0.5 * (u0[cc] + u1[cc]) - 0.0 * 0.5 * (v0[cc] + v1[cc]));
        if (p.useNHMTerms)
          gW = gW + ((u0[cc] * u0[cc] + u1[cc] * u1[cc]) + (v0[cc] * v0[cc] + v1[cc] * v1[cc])) * 0.5 * p.recip_rSphere;
        al = al + scalingFactor * gW;
      }
      if (RS) f.alphaRho[q3] = al;
      const double sM = dRlocM * p.gravity * al * recip_rhoConst;
      const double sP = dRlocP * p.gravity * al * recip_rhoConst;
      const double phC = phF + sM;
      phF = phC + sP;
      if (RS) {
        const double drF = f.drF[k - 1];
        const double cc2 = dCdt * drF * hC[cc] * rA;
        f.dWtC[q3] = c;
        c = c - cc2;
        if (ring) {
          const double uu = dWdt * drF * hW[cc] * rAw, vv = dSdt * drF * hS[cc] * rAs;
          f.dWtU[q3] = u;
          f.dWtV[q3] = v;
          u = u - uu;
          v = v - vv;
        }
      }
      if (ring) {
        f.phiHydC[q3] = phC;
        if (tot) {
          if (totR) {
            const double dPhiRef = (roS - f.rC[k - 1]) * p.gravity;
            f.totPhiHyd[q3] = phC * fac + fmax(dPhiRef, 0.0) * (fac - 1.0) + 0.0;
          } else {
            f.totPhiHyd[q3] = phC + bEta + 0.0;
          }
        }
      }
    }
  };
  if constexpr (NRC > 0) {
#pragma unroll
    for (int k0 = 1; k0 <= NRC; k0 += CH) chunk(k0);
  } else {
    for (int k0 = 1; k0 <= Nr; k0 += CH) chunk(k0);
  }
}
template <bool RS, bool QH, int NRC = 0>
__global__ void __launch_bounds__(256) k_phi_flat(Dims d, Params p, Fields f) {
  phi_flat_body<RS, QH, NRC>(d, p, f, mg_xcd_block());
}

// whether CALC_PHI_HYD runs the flat pass: by default where neither r* nor the QH terms add
// their per-level operands (LLC-90: 63 -> 30 us; with them, on the small r* grids, the one
// serial thread per column is slower than the column frame: config 2 0.319 against 0.309
// ms/step, config 3 0.414 against 0.411, profiles/r03/phiflat/).  MGCM_PHI_FLAT=0 never,
// 2 always (read per launch)
inline bool phi_flat_on(const Params &p) {
  const char *e = getenv("MGCM_PHI_FLAT");
  const int v = e ? atoi(e) : 1;
  if (v == 0 || v == 2) return v == 2;
  const bool rs = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
  const bool qh = p.quasiHydrostatic && (p.select3dCoriScheme >= 1 || p.useNHMTerms);
  return !rs && !qh;
}
inline int phi_flat_blocks(const Dims &d, const Params &p) {
  const int o = (p.nonlinFreeSurf > 0 && p.select_rStar > 0) ? 1 : 0;
  return (int)(((long)(d.sNx + 2 + o) * (d.sNy + 2 + o) * d.nT + 255) / 256);
}
__global__ void __launch_bounds__(256) k_phys_phi(Dims d, Params p, Fields f, int nc, const int *iterPtr) {
  phi_hyd_body<true>(d, p, f, nc, mg_xcd_block(), iterPtr);
}
// CALC_PHI_HYD and MOM_U_DEL2U / MOM_V_DEL2V in one grid (independent: each reads only the
// state DYNAMICS starts from): the first nbPhi logical blocks are k_phi_hyd's, the rest
// k_del2uv's; each body's barriers are block-uniform
__global__ void __launch_bounds__(256) k_phi_del2(Dims d, Params p, Fields f, int nc, int nbPhi) {
  const int lb = mg_xcd_block();
  if (lb < nbPhi) phi_hyd_body(d, p, f, nc, lb);
  else del2uv_body(d, p, f, lb - nbPhi);
}


// Values the VI helpers read outside the level's staged fields -- the tile's face and edge
// bits, the vertical grid's 1-D factors, the own point's rest-state thicknesses -- through
// these functions of the accessor: by default where they lie; k_mom_vi_m2's accessor
// (overloads after VIM2) hands them over from registers filled at the level's start, so no
// load of them waits behind the level's stores (vmcnt counts stores too).
template <class A> __device__ __forceinline__ int vi_tile_face(const A &, const Fields &f, int t) { return f.tileFace[t]; }
template <class A> __device__ __forceinline__ int vi_tile_edge(const A &, const Fields &f, int t) { return f.tileEdge[t]; }
template <class A> __device__ __forceinline__ double vi_rdrC(const A &, const Fields &f, int kk) { return f.recip_drC[kk - 1]; }
template <class A> __device__ __forceinline__ double vi_rdrF(const A &, const Fields &f, int kk) { return f.recip_drF[kk - 1]; }
template <class A> __device__ __forceinline__ double vi_drF(const A &, const Fields &f, int kk) { return f.drF[kk - 1]; }
template <class A> __device__ __forceinline__ double vi_h0W_own(const A &a, int i, int j, int k) { return a.h0FacW(i, j, k); }
template <class A> __device__ __forceinline__ double vi_h0S_own(const A &a, int i, int j, int k) { return a.h0FacS(i, j, k); }

// ---- MOM_VECINV's per-level intermediates as functions of an accessor A of the level's
// 3-D fields (uVel, vVel, hFacW, hFacS, recip_hFacC at (ii, jj, k)): VIGlobal reads them
// from HBM, VITile from the LDS-staged tile of k_mom_vi_tiled; the expression trees are
// shared, so both kernels produce the same bits.
// hFacZ (pkg/mom_common/mom_calc_hfacz.F:158-225, hZoption = 0)
template <class A>
__device__ __forceinline__ double vi_hfacz(const A &a, const Dims &d, int ii, int jj, int k) {
  if (ii < 2 - d.OLx || jj < 2 - d.OLy) return 0.0;
  double h = fmin(a.hFacW(ii, jj, k), a.hFacW(ii, jj - 1, k));
  h = fmin(a.hFacS(ii, jj, k), h);
  h = fmin(a.hFacS(ii - 1, jj, k), h);
  return h;
}
// h0FacZ (mom_fluxform.F:290-307 / mom_vecinv.F): rest-state h0FacW/S under the non-linear
// free surface with no-slip walls, else hFacZ
template <class A, class P>
__device__ __forceinline__ double vi_h0facz(const A &a, const Dims &d, const P &p, int ii, int jj, int k) {
  if (!(p.momViscosity && p.no_slip_sides && p.nonlinFreeSurf > 0)) return vi_hfacz(a, d, ii, jj, k);
  if (ii < 2 - d.OLx || jj < 2 - d.OLy) return 0.0;
  return fmin(fmin(a.h0FacW(ii, jj, k), a.h0FacW(ii, jj - 1, k)), fmin(a.h0FacS(ii, jj, k), a.h0FacS(ii - 1, jj, k)));
}
// MOM_CALC_KE (mom_calc_ke.F:66-150), computed on 1-OL..sN+OL-1
template <class A, class P>
__device__ __forceinline__ double vi_KE(const A &a, const Dims &d, const P &p, const Fields &f, int ii, int jj, int k, int t) {
  const int OLx = d.OLx, OLy = d.OLy, sNx = d.sNx, sNy = d.sNy;
  (void)OLx; (void)OLy; (void)sNx; (void)sNy;
#define U(ii, jj) a.uVel(ii, jj, k)
#define V(ii, jj) a.vVel(ii, jj, k)
#define G2(x, ii, jj) a.template g2<F2_##x>(ii, jj)
#define G3(x, ii, jj, kk) a.x(ii, jj, kk)

    if (ii < 1 - OLx || ii > sNx + OLx - 1 || jj < 1 - OLy || jj > sNy + OLy - 1) return 0.0;
    const double u0 = U(ii, jj), u1 = U(ii + 1, jj), v0 = V(ii, jj), v1 = V(ii, jj + 1);
    switch (p.selectKEscheme) {
      case 0: return 0.25 * ((u0 * u0 + u1 * u1) + (v0 * v0 + v1 * v1));
      case 1:
        return 0.25 * ((u0 * u0 * G2(rAw, ii, jj) + u1 * u1 * G2(rAw, ii + 1, jj)) +
                       (v0 * v0 * G2(rAs, ii, jj) + v1 * v1 * G2(rAs, ii, jj + 1))) * G2(recip_rA, ii, jj);
      case 2:
        return 0.25 * ((u0 * u0 * G3(hFacW, ii, jj, k) + u1 * u1 * G3(hFacW, ii + 1, jj, k)) +
                       (v0 * v0 * G3(hFacS, ii, jj, k) + v1 * v1 * G3(hFacS, ii, jj + 1, k))) *
               G3(recip_hFacC, ii, jj, k);
      default:
        return 0.25 * ((u0 * u0 * G3(hFacW, ii, jj, k) * G2(rAw, ii, jj) +
                        u1 * u1 * G3(hFacW, ii + 1, jj, k) * G2(rAw, ii + 1, jj)) +
                       (v0 * v0 * G3(hFacS, ii, jj, k) * G2(rAs, ii, jj) +
                        v1 * v1 * G3(hFacS, ii, jj + 1, k) * G2(rAs, ii, jj + 1))) *
               G3(recip_hFacC, ii, jj, k) * G2(recip_rA, ii, jj);
    }
  #undef U
#undef V
#undef G2
#undef G3
}
  // MOM_CALC_RELVORT3 (mom_calc_relvort3.F:72-233) on 2-OL..sN+OL, then 0 where hFacZ = 0
  // (mom_vecinv.F:395-403); 0 outside the computed range
  template <class A, class P>
__device__ __forceinline__ double vi_vort(const A &a, const Dims &d, const P &p, const Fields &f, int ii, int jj, int k, int t) {
  const int OLx = d.OLx, OLy = d.OLy, sNx = d.sNx, sNy = d.sNy;
  (void)OLx; (void)OLy; (void)sNx; (void)sNy;
#define U(ii, jj) a.uVel(ii, jj, k)
#define V(ii, jj) a.vVel(ii, jj, k)
#define G2(x, ii, jj) a.template g2<F2_##x>(ii, jj)
#define G3(x, ii, jj, kk) a.x(ii, jj, kk)

    if (ii < 2 - OLx || jj < 2 - OLy || ii > sNx + OLx || jj > sNy + OLy) return 0.0;
    if (vi_hfacz(a, d, ii, jj, k) == 0.0) return 0.0;
#define UC(a, b) (U(a, b) * G2(dxC, a, b))
#define VC(a, b) (V(a, b) * G2(dyC, a, b))
    const double rz = G2(recip_rAz, ii, jj);
    if (p.cubeCorners) {
      const int face = vi_tile_face(a, f, t), e = vi_tile_edge(a, f, t);
      const bool isN = e & 1, isS = e & 2, isE = e & 4, isW = e & 8;
      if (ii == 1 && jj == 1 && isW && isS) return rz * ((VC(ii, jj) - UC(ii, jj)) + UC(ii, jj - 1));
      if (ii == sNx + 1 && jj == 1 && isE && isS) {
        if (face == 2) return rz * ((-UC(ii, jj) - VC(ii - 1, jj)) + UC(ii, jj - 1));
        if (face == 4) return rz * ((-VC(ii - 1, jj) + UC(ii, jj - 1)) - UC(ii, jj));
        return rz * ((UC(ii, jj - 1) - UC(ii, jj)) - VC(ii - 1, jj));
      }
      if (ii == 1 && jj == sNy + 1 && isW && isN) {
        if (face == 1) return rz * ((UC(ii, jj - 1) + VC(ii, jj)) - UC(ii, jj));
        if (face == 3) return rz * ((-UC(ii, jj) + UC(ii, jj - 1)) + VC(ii, jj));
        return rz * ((VC(ii, jj) - UC(ii, jj)) + UC(ii, jj - 1));
      }
      if (ii == sNx + 1 && jj == sNy + 1 && isE && isN) {
        if (face % 2 == 1) return rz * ((-UC(ii, jj) - VC(ii - 1, jj)) + UC(ii, jj - 1));
        return rz * ((UC(ii, jj - 1) - UC(ii, jj)) - VC(ii - 1, jj));
      }
    }
    return rz * ((VC(ii, jj) - VC(ii - 1, jj)) - (UC(ii, jj) - UC(ii, jj - 1)));
#undef UC
#undef VC
  #undef U
#undef V
#undef G2
#undef G3
}
  // MOM_CALC_HDIV(hDivScheme = 2) (mom_calc_hdiv.F:76-89) on 1-OL..sN+OL-1
  template <class A, class P>
__device__ __forceinline__ double vi_hdiv(const A &a, const Dims &d, const P &p, const Fields &f, int ii, int jj, int k, int t) {
  const int OLx = d.OLx, OLy = d.OLy, sNx = d.sNx, sNy = d.sNy;
  (void)OLx; (void)OLy; (void)sNx; (void)sNy;
#define U(ii, jj) a.uVel(ii, jj, k)
#define V(ii, jj) a.vVel(ii, jj, k)
#define G2(x, ii, jj) a.template g2<F2_##x>(ii, jj)
#define G3(x, ii, jj, kk) a.x(ii, jj, kk)

    if (ii < 1 - OLx || ii > sNx + OLx - 1 || jj < 1 - OLy || jj > sNy + OLy - 1) return 0.0;
    return ((U(ii + 1, jj) * G2(dyG, ii + 1, jj) * G3(hFacW, ii + 1, jj, k) - U(ii, jj) * G2(dyG, ii, jj) * G3(hFacW, ii, jj, k)) +
            (V(ii, jj + 1) * G2(dxG, ii, jj + 1) * G3(hFacS, ii, jj + 1, k) - V(ii, jj) * G2(dxG, ii, jj) * G3(hFacS, ii, jj, k))) *
           G2(recip_rA, ii, jj) * G3(recip_hFacC, ii, jj, k);
  #undef U
#undef V
#undef G2
#undef G3
}

// Accessor of HBM (the per-point k_mom_step<true>): every value read where it lies.
struct VIGlobal {
  const Dims &d; const Params &p; const Fields &f; int k, t;
#define VIG(x) __device__ __forceinline__ double x(int ii, int jj, int kk) const { return AR3(x, MG_I3(d, ii, jj, kk, t)); }
  VIG(uVel) VIG(vVel) VIG(wVel) VIG(hFacW) VIG(hFacS) VIG(recip_hFacC) VIG(recip_hFacW) VIG(recip_hFacS) VIG(maskW)
  VIG(maskS) VIG(maskC) VIG(h0FacW) VIG(h0FacS)
#undef VIG
  template <int F> __device__ __forceinline__ double g2(int ii, int jj) const { return f.a2[(long)F * d.N2all + MG_I2(d, ii, jj, t)]; }
  __device__ __forceinline__ double hfz(int ii, int jj) const { return vi_hfacz(*this, d, ii, jj, k); }
  __device__ __forceinline__ double h0fz(int ii, int jj) const { return vi_h0facz(*this, d, p, ii, jj, k); }
  __device__ __forceinline__ double KE(int ii, int jj) const { return vi_KE(*this, d, p, f, ii, jj, k, t); }
  __device__ __forceinline__ double vort(int ii, int jj) const { return vi_vort(*this, d, p, f, ii, jj, k, t); }
  __device__ __forceinline__ double hDiv(int ii, int jj) const { return vi_hdiv(*this, d, p, f, ii, jj, k, t); }
};

// MOM_VECINV (pkg/mom_vecinv/mom_vecinv.F:42-1064) for one output point (i,j,k) of the
// DYNAMICS range 0..sN+1: every intermediate the reference keeps in 2-D scratch (KE,
// vort3, hFacZ, hDiv, the vertical viscous flux ping-pong) is re-derived at the
// neighbours it needs with the reference's expression and operand order, including
// MOM_CALC_RELVORT3's cube-corner circulations.  Subset (mgcm_init checks it): no
// useAbsVorticity / high-order / upwind vorticity, constant harmonic viscosity, explicit
// vertical viscosity, no biharmonic, no 3-D Coriolis / NH metric.  deepFac = rhoFac = 1.
template <class A, class P>
__device__ __forceinline__ void vecinv_tend(const A &a, const Dims &d, const P &p, const Fields &f, int i, int j, int k, int t, double &gU,
                            double &gV, double &guDiss, double &gvDiss) {
  const int Nr = d.Nr, OLx = d.OLx, OLy = d.OLy, sNx = d.sNx, sNy = d.sNy;
#define U(ii, jj) a.uVel(ii, jj, k)
#define V(ii, jj) a.vVel(ii, jj, k)
#define U3(ii, jj, kk) a.uVel(ii, jj, kk)
#define V3(ii, jj, kk) a.vVel(ii, jj, kk)
#define W3(ii, jj, kk) a.wVel(ii, jj, kk)
#define G2(x, ii, jj) a.template g2<F2_##x>(ii, jj)
#define G3(x, ii, jj, kk) a.x(ii, jj, kk)
  const double recip_drF = vi_rdrF(a, f, k), drF = vi_drF(a, f, k);
  auto rhz = [&](int ii, int jj) -> double {   // r_hFacZ
    const double h = a.hfz(ii, jj);
    return h == 0.0 ? 0.0 : 1.0 / h;
  };
  const double rhFacW = G3(recip_hFacW, i, j, k), rhFacS = G3(recip_hFacS, i, j, k);
  const double hZ = a.hfz(i, j), hZn = a.hfz(i, j + 1), hZe = a.hfz(i + 1, j);
  const double vz = a.vort(i, j), vzn = a.vort(i, j + 1), vze = a.vort(i + 1, j);
  guDiss = 0.0; gvDiss = 0.0;
  if (p.momViscosity) {
    // MOM_VI_HDISSIP (mom_vi_hdissip.F:105-131) on 2-OL..sN+OL-1, constant viscosity, cosFac = 1
    if (i >= 2 - OLx && i <= sNx + OLx - 1 && j >= 2 - OLy && j <= sNy + OLy - 1 &&
        (p.viscAhD != 0.0 || p.viscAhZ != 0.0)) {
      const double Dij = a.hDiv(i, j), Dim = a.hDiv(i, j - 1), Dmj = a.hDiv(i - 1, j);
      const double Zip = hZn * vzn, Zij = hZ * vz, Zpj = hZe * vze;
      const double uD2 = p.viscAhD * 1.0 * (Dij - Dmj) * G2(recip_dxC, i, j) -
                         p.viscAhZ * rhFacW * (Zip - Zij) * G2(recip_dyG, i, j);
      const double vD2 = p.viscAhZ * rhFacS * 1.0 * (Zpj - Zij) * G2(recip_dxG, i, j) +
                         p.viscAhD * (Dij - Dim) * G2(recip_dyC, i, j);
      guDiss = uD2 * G3(maskW, i, j, k);
      gvDiss = vD2 * G3(maskS, i, j, k);
    }
    // MOM_U/V_RVISCFLUX(k+1) into the fVerUkp ping-pong and its k-1 partner (mom_vecinv.F:546-563)
    auto rvU = [&](int kk) -> double {
      if (kk <= 1 || kk > Nr) return 0.0;
      return p.vfFacMom * 1.0 * (-p.viscAr * G2(rAw, i, j) * (U3(i, j, kk) - U3(i, j, kk - 1)) * p.rkSign *
                                 vi_rdrC(a, f, kk) * G3(maskW, i, j, kk) * G3(maskW, i, j, kk - 1));
    };
    auto rvV = [&](int kk) -> double {
      if (kk <= 1 || kk > Nr) return 0.0;
      return p.vfFacMom * 1.0 * (-p.viscAr * G2(rAs, i, j) * (V3(i, j, kk) - V3(i, j, kk - 1)) * p.rkSign *
                                 vi_rdrC(a, f, kk) * G3(maskS, i, j, kk) * G3(maskS, i, j, kk - 1));
    };
    // skipped with implicitViscosity (mom_vecinv.F:444): k_mom_impl solves it after the k loop
    if (!p.implicitViscosity) guDiss = guDiss - rhFacW * recip_drF * G2(recip_rAw, i, j) * (rvU(k + 1) - rvU(k)) * p.rkSign;
    if (p.no_slip_sides) {
      const double h0W = vi_h0W_own(a, i, j, k);
      const double hS = h0W - a.h0fz(i, j);
      const double hN = h0W - a.h0fz(i, j + 1);
      const double u0 = U(i, j);
      guDiss = guDiss + -rhFacW * recip_drF * G2(recip_rAw, i, j) *
                            (hS * G2(dxV, i, j) * G2(recip_dyU, i, j) * (p.viscAhZ * u0 - p.viscA4Z * 0.0) +
                             hN * G2(dxV, i, j + 1) * G2(recip_dyU, i, j + 1) * (p.viscAhZ * u0 - p.viscA4Z * 0.0)) *
                            drF * p.sideDragFactor;
    }
    if (p.no_slip_bottom) {
      const int kDn = (k + 1 < Nr) ? k + 1 : Nr, kLowF = k + 1;
      const double recDrC = (k == Nr) ? recip_drF : vi_rdrC(a, f, kLowF);
      double cD = 0.0 * 1.0;
      cD = cD + p.viscAr * recDrC * 2.0;
      cD = (k == Nr) ? cD * G3(maskW, i, j, k) : cD * G3(maskW, i, j, k) * (1.0 - G3(maskW, i, j, kDn));
      guDiss = guDiss + -cD * U(i, j) * rhFacW * recip_drF;
    }
    if (!p.implicitViscosity) gvDiss = gvDiss - rhFacS * recip_drF * G2(recip_rAs, i, j) * (rvV(k + 1) - rvV(k)) * p.rkSign;
    if (p.no_slip_sides) {
      const double h0S = vi_h0S_own(a, i, j, k);
      const double hW = h0S - a.h0fz(i, j);
      const double hE = h0S - a.h0fz(i + 1, j);
      const double v0 = V(i, j);
      gvDiss = gvDiss + -rhFacS * recip_drF * G2(recip_rAs, i, j) *
                            (hW * G2(dyU, i, j) * G2(recip_dxV, i, j) * (p.viscAhZ * v0 - p.viscA4Z * 0.0) +
                             hE * G2(dyU, i + 1, j) * G2(recip_dxV, i + 1, j) * (p.viscAhZ * v0 - p.viscA4Z * 0.0)) *
                            drF * p.sideDragFactor;
    }
    if (p.no_slip_bottom) {
      const int kDn = (k + 1 < Nr) ? k + 1 : Nr, kLowF = k + 1;
      const double recDrC = (k == Nr) ? recip_drF : vi_rdrC(a, f, kLowF);
      double cD = 0.0 * 1.0;
      cD = cD + p.viscAr * recDrC * 2.0;
      cD = (k == Nr) ? cD * G3(maskS, i, j, k) : cD * G3(maskS, i, j, k) * (1.0 - G3(maskS, i, j, kDn));
      gvDiss = gvDiss + -cD * V(i, j) * rhFacS * recip_drF;
    }
  }
#define VX(a, b) (V(a, b) * G2(dxG, a, b))
#define VXH(a, b) (V(a, b) * G2(dxG, a, b) * G3(hFacS, a, b, k))
#define UY(a, b) (U(a, b) * G2(dyG, a, b))
#define UYH(a, b) (U(a, b) * G2(dyG, a, b) * G3(hFacW, a, b, k))
  // MOM_VI_CORIOLIS (mom_vi_coriolis.F:60-190)
  gU = 0.0; gV = 0.0;
  if (p.useCoriolis) {
    const int cs = p.selectCoriScheme;
    const double epsil = 1.0e-9;
    double c;
    if (cs == 0) {
      const double vb = 0.25 * ((VX(i, j) + VX(i - 1, j)) + (VX(i, j + 1) + VX(i - 1, j + 1)));
      c = 0.5 * (G2(fCoriG, i, j) + G2(fCoriG, i, j + 1)) * vb * G2(recip_dxC, i, j) * G3(maskW, i, j, k);
    } else if (cs == 1) {
      const double vb = ((VXH(i, j) + VXH(i - 1, j)) + (VXH(i, j + 1) + VXH(i - 1, j + 1))) /
                        fmax(epsil, (G3(hFacS, i, j, k) + G3(hFacS, i - 1, j, k)) + (G3(hFacS, i, j + 1, k) + G3(hFacS, i - 1, j + 1, k)));
      c = 0.5 * (G2(fCoriG, i, j) + G2(fCoriG, i, j + 1)) * vb * G2(recip_dxC, i, j) * G3(maskW, i, j, k);
    } else if (cs == 2) {
      const double vb = 0.25 * ((VXH(i, j) + VXH(i - 1, j)) + (VXH(i, j + 1) + VXH(i - 1, j + 1)));
      c = 0.5 * (G2(fCoriG, i, j) + G2(fCoriG, i, j + 1)) * vb * G2(recip_dxC, i, j) * rhFacW;
    } else {
      const double vm = 0.5 * (VXH(i, j) + VXH(i - 1, j)), vp = 0.5 * (VXH(i, j + 1) + VXH(i - 1, j + 1));
      c = 0.5 * (vm * G2(fCoriG, i, j) + vp * G2(fCoriG, i, j + 1)) * G2(recip_dxC, i, j) * rhFacW;
    }
    gU = c;
    if (cs == 0) {
      const double ub = 0.25 * ((UY(i, j) + UY(i, j - 1)) + (UY(i + 1, j) + UY(i + 1, j - 1)));
      c = -0.5 * (G2(fCoriG, i, j) + G2(fCoriG, i + 1, j)) * ub * G2(recip_dyC, i, j) * G3(maskS, i, j, k);
    } else if (cs == 1) {
      const double ub = ((UYH(i, j) + UYH(i, j - 1)) + (UYH(i + 1, j) + UYH(i + 1, j - 1))) /
                        fmax(epsil, (G3(hFacW, i, j, k) + G3(hFacW, i, j - 1, k)) + (G3(hFacW, i + 1, j, k) + G3(hFacW, i + 1, j - 1, k)));
      c = -0.5 * (G2(fCoriG, i, j) + G2(fCoriG, i + 1, j)) * ub * G2(recip_dyC, i, j) * G3(maskS, i, j, k);
    } else if (cs == 2) {
      const double ub = 0.25 * ((UYH(i, j) + UYH(i, j - 1)) + (UYH(i + 1, j) + UYH(i + 1, j - 1)));
      c = -0.5 * (G2(fCoriG, i, j) + G2(fCoriG, i + 1, j)) * ub * G2(recip_dyC, i, j) * rhFacS;
    } else {
      const double um = 0.5 * (UYH(i, j) + UYH(i, j - 1)), up = 0.5 * (UYH(i + 1, j) + UYH(i + 1, j - 1));
      c = -0.5 * (um * G2(fCoriG, i, j) + up * G2(fCoriG, i + 1, j)) * G2(recip_dyC, i, j) * rhFacS;
    }
    gV = c;
  }
  if (p.momAdvection) {
    // MOM_VI_U/V_CORIOLIS with omega3 = vort3 (mom_vi_u_coriolis.F:70-190, mom_vi_v_coriolis.F)
    const int vs = p.selectVortScheme;
    const double epsil = 1.0e-9, oneThird = 1.0 / 3.0;
    double c;
    if (vs == 0) {
      const double vb = 0.25 * ((VXH(i, j) + VXH(i - 1, j)) + (VXH(i, j + 1) + VXH(i - 1, j + 1)));
      c = 0.5 * (vz * rhz(i, j) + vzn * rhz(i, j + 1)) * vb * G2(recip_dxC, i, j) * G3(maskW, i, j, k);
    } else if (vs == 1) {
      const double vb = 0.5 * ((VX(i, j) * hZ + VX(i - 1, j) * hZ) + (VX(i, j + 1) * hZn + VX(i - 1, j + 1) * hZn)) /
                        fmax(epsil, hZ + hZn);
      c = 0.5 * (vz + vzn) * vb * G2(recip_dxC, i, j) * G3(maskW, i, j, k);
    } else if (vs == 2) {
      const double vm = 0.5 * (VXH(i, j) + VXH(i - 1, j)), vp = 0.5 * (VXH(i, j + 1) + VXH(i - 1, j + 1));
      c = (vm * rhz(i, j) * vz + vp * rhz(i, j + 1) * vzn) * 0.5 * G2(recip_dxC, i, j) * G3(maskW, i, j, k);
    } else {
      c = 0.0;
      if (i <= sNx + OLx - 1) {
        const double rzw = rhz(i - 1, j) * a.vort(i - 1, j), rzwn = rhz(i - 1, j + 1) * a.vort(i - 1, j + 1);
        const double rze = rhz(i + 1, j) * vze, rzen = rhz(i + 1, j + 1) * a.vort(i + 1, j + 1);
        const double r0 = rhz(i, j) * vz, rn = rhz(i, j + 1) * vzn;
        const double mj = (r0 + (rn + rzw)) * oneThird * VXH(i - 1, j);
        const double ij = (r0 + (rn + rze)) * oneThird * VXH(i, j);
        const double mp = (rn + (r0 + rzwn)) * oneThird * VXH(i - 1, j + 1);
        const double ip = (rn + (r0 + rzen)) * oneThird * VXH(i, j + 1);
        c = ((mj + ij) + (mp + ip)) * 0.25 * G2(recip_dxC, i, j) * G3(maskW, i, j, k);
      }
    }
    gU = gU + c;
    if (vs == 0) {
      const double ub = 0.25 * ((UYH(i, j) + UYH(i, j - 1)) + (UYH(i + 1, j) + UYH(i + 1, j - 1)));
      c = -(0.5 * (vz * rhz(i, j) + vze * rhz(i + 1, j))) * ub * G2(recip_dyC, i, j) * G3(maskS, i, j, k);
    } else if (vs == 1) {
      const double ub = 0.5 * ((UY(i, j) * hZ + UY(i, j - 1) * hZ) + (UY(i + 1, j) * hZe + UY(i + 1, j - 1) * hZe)) /
                        fmax(epsil, hZ + hZe);
      c = -(0.5 * (vz + vze)) * ub * G2(recip_dyC, i, j) * G3(maskS, i, j, k);
    } else if (vs == 2) {
      const double um = 0.5 * (UYH(i, j) + UYH(i, j - 1)), up = 0.5 * (UYH(i + 1, j) + UYH(i + 1, j - 1));
      c = -((um * rhz(i, j) * vz + up * rhz(i + 1, j) * vze) * 0.5) * G2(recip_dyC, i, j) * G3(maskS, i, j, k);
    } else {
      c = 0.0;
      if (j <= sNy + OLy - 1) {
        const double r0 = rhz(i, j) * vz, re = rhz(i + 1, j) * vze;
        const double rs = rhz(i, j - 1) * a.vort(i, j - 1), rn = rhz(i, j + 1) * vzn;
        const double res = rhz(i + 1, j - 1) * a.vort(i + 1, j - 1), ren = rhz(i + 1, j + 1) * a.vort(i + 1, j + 1);
        const double im = (r0 + (re + rs)) * oneThird * UYH(i, j - 1);
        const double ij = (r0 + (re + rn)) * oneThird * UYH(i, j);
        const double pm = (re + (r0 + res)) * oneThird * UYH(i + 1, j - 1);
        const double pj = (re + (r0 + ren)) * oneThird * UYH(i + 1, j);
        c = -(((im + ij) + (pm + pj)) * 0.25) * G2(recip_dyC, i, j) * G3(maskS, i, j, k);
      }
    }
    gV = gV + c;
    // MOM_VI_U/V_VERTSHEAR (mom_vi_u_vertshear.F:60-110)
    {
      const int Kp1 = k + 1 < Nr ? k + 1 : Nr, Km1 = k - 1 > 1 ? k - 1 : 1;
      const double mKp1 = (k == Nr) ? 0.0 : 1.0, mKm1 = (k == 1) ? 0.0 : 1.0;
      const bool areaW = !(p.selectKEscheme == 1 || p.selectKEscheme == 3);
      double wm, wp;
      if (areaW) {
        wm = 0.5 * (W3(i, j, k) * G2(rA, i, j) * G3(maskC, i, j, Km1) + W3(i - 1, j, k) * G2(rA, i - 1, j) * G3(maskC, i - 1, j, Km1)) *
             mKm1 * G2(recip_rAw, i, j);
        wp = 0.5 * (W3(i, j, Kp1) * G2(rA, i, j) + W3(i - 1, j, Kp1) * G2(rA, i - 1, j)) * mKp1 * G2(recip_rAw, i, j);
      } else {
        wm = 0.5 * (W3(i, j, k) * G3(maskC, i, j, Km1) + W3(i - 1, j, k) * G3(maskC, i - 1, j, Km1)) * mKm1;
        wp = 0.5 * (W3(i, j, Kp1) + W3(i - 1, j, Kp1)) * mKp1;
      }
      double zm = (U3(i, j, k) - mKm1 * U3(i, j, Km1)) * p.rkSign;
      double zp = (mKp1 * U3(i, j, Kp1) - U3(i, j, k)) * p.rkSign;
      if (p.upwindShear) gU = gU + -0.5 * ((wp * zp + wm * zm) + (fabs(wp) * zp - fabs(wm) * zm)) * rhFacW * recip_drF;
      else gU = gU + -0.5 * (wp * zp + wm * zm) * rhFacW * recip_drF;
      if (areaW) {
        wm = 0.5 * (W3(i, j, k) * G2(rA, i, j) * G3(maskC, i, j, Km1) + W3(i, j - 1, k) * G2(rA, i, j - 1) * G3(maskC, i, j - 1, Km1)) *
             mKm1 * G2(recip_rAs, i, j);
        wp = 0.5 * (W3(i, j, Kp1) * G2(rA, i, j) + W3(i, j - 1, Kp1) * G2(rA, i, j - 1)) * mKp1 * G2(recip_rAs, i, j);
      } else {
        wm = 0.5 * (W3(i, j, k) * G3(maskC, i, j, Km1) + W3(i, j - 1, k) * G3(maskC, i, j - 1, Km1)) * mKm1;
        wp = 0.5 * (W3(i, j, Kp1) + W3(i, j - 1, Kp1)) * mKp1;
      }
      zm = (V3(i, j, k) - mKm1 * V3(i, j, Km1)) * p.rkSign;
      zp = (mKp1 * V3(i, j, Kp1) - V3(i, j, k)) * p.rkSign;
      if (p.upwindShear) gV = gV + -0.5 * ((wp * zp + wm * zm) + (fabs(wp) * zp - fabs(wm) * zm)) * rhFacS * recip_drF;
      else gV = gV + -0.5 * (wp * zp + wm * zm) * rhFacS * recip_drF;
    }
    // MOM_VI_U/V_GRAD_KE (mom_vi_u_grad_ke.F:49-55)
    const double ke = a.KE(i, j);
    gU = gU + -G2(recip_dxC, i, j) * (ke - a.KE(i - 1, j)) * G3(maskW, i, j, k);
    gV = gV + -G2(recip_dyC, i, j) * (ke - a.KE(i, j - 1)) * G3(maskS, i, j, k);
  }
#undef VX
#undef VXH
#undef UY
#undef UYH
  // mom_vecinv.F:1044-1051
  gU = gU * G3(maskW, i, j, k);
  gV = gV * G3(maskS, i, j, k);
#undef U
#undef V
#undef U3
#undef V3
#undef W3
#undef G2
#undef G3
}

// One point of DYNAMICS' momentum block.  COMP = 0 stores both components; 1 only the U
// outputs (gU, guNm1, cdU), 2 only the V outputs: the other component's arithmetic is then
// dead and compiled out, so k_mom_step_uv runs the two halves as separate, shorter threads.
// PART (flux form only, k_mom_ff4 / mom_ff4_body): 0 the whole point; 1 every term but the
// viscous ones, whose sum guDiss / gvDiss it takes from *sD after the workgroup barrier; 2 the
// viscous terms only, stored to *sD before that barrier (the other role's wave of the same
// points).  valid = false: no arithmetic, only the barrier (PART 1 / 2 reach it on every lane).
template <bool VI, int COMP, int PART = 0>
__device__ __forceinline__ void mom_step_ijz(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, int i,
                                             int j, int z, bool valid, double *sD) {
  static_assert(PART == 0 || (!VI && COMP != 0), "the viscous split is per component, flux form");
  valid = valid && !(i > d.sNx + d.OLx || j > d.sNy + d.OLy);
  if constexpr (PART == 0) {
    if (!valid) return;
  }
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  const int Nr = d.Nr;
  const int myIter = *iterPtr;
  // adams_bashforth2.F:61-65 (mom_StartAB = nIter0 for a cold start)
  const double abFac = (myIter == p.nIter0 && p.nIter0 == 0) ? 0.0 : 0.5 + p.abEps;
  const bool inner = (i >= 0 && i <= d.sNx + 1 && j >= 0 && j <= d.sNy + 1);
  const double mass2rUnit = 1.0 / p.rhoConst;
  const double uDudxFac = p.afFacMom, vDudyFac = p.afFacMom, rVelDudrFac = p.afFacMom;
  const double AhDudxFac = p.vfFacMom, AhDudyFac = p.vfFacMom;
  const double ArDudrFac = p.implicitViscosity ? 0.0 : p.vfFacMom;
  const double fuFac = p.cfFacMom, fvFac = p.cfFacMom;
  const long q2 = MG_I2(d, i, j, t);
  const bool rstar = p.nonlinFreeSurf > 0 && p.select_rStar > 0;

#define U(ii, jj, kk) AR3(uVel, MG_I3(d, ii, jj, kk, t))
#define V(ii, jj, kk) AR3(vVel, MG_I3(d, ii, jj, kk, t))
#define W(ii, jj, kk) AR3(wVel, MG_I3(d, ii, jj, kk, t))
#define G2(a, ii, jj) f.a[MG_I2(d, ii, jj, t)]
#define G3(a, ii, jj, kk) f.a[MG_I3(d, ii, jj, kk, t)]

  // vertical advective flux of momentum through the top of level kk (fVerU/V(kUp)):
  // MOM_CALC_RTRANS + MOM_U/V_ADV_WU/WV (mom_fluxform.F:384-424), select_rStar = 0
  // r*: MOM_CALC_RTRANS's dWtrans (mom_calc_rtrans.F:91-137): the column sums of the
  // level-thickness tendency above level kk, in the reference's sequential order
  auto fverU = [&](int kk) -> double {
    if (kk > Nr) return 0.0;
    double rTU = 0.5 * (W(i - 1, j, kk) * G2(rA, i - 1, j) + W(i, j, kk) * G2(rA, i, j));
    if (kk == 1) return rTU * U(i, j, 1);
    if (rstar) {   // dWtrans of this level from k_phi_hyd
      rTU = rTU - G3(dWtU, i, j, kk) + (G3(dWtC, i - 1, j, kk) + G3(dWtC, i, j, kk)) * 0.5;
      return rTU * (0.5 * (U(i, j, kk) + U(i, j, kk - 1)));
    }
    double fu_ = rTU * (0.5 * (U(i, j, kk) + U(i, j, kk - 1)));
    fu_ = fu_ + 0.25 * (W(i, j, kk) * G2(rA, i, j) * (G3(maskC, i, j, kk) - G3(maskC, i, j, kk - 1)) +
                        W(i - 1, j, kk) * G2(rA, i - 1, j) * (G3(maskC, i - 1, j, kk) - G3(maskC, i - 1, j, kk - 1))) *
                    U(i, j, kk);
    return fu_;
  };
  auto fverV = [&](int kk) -> double {
    if (kk > Nr) return 0.0;
    double rTV = 0.5 * (W(i, j - 1, kk) * G2(rA, i, j - 1) + W(i, j, kk) * G2(rA, i, j));
    if (kk == 1) return rTV * V(i, j, 1);
    if (rstar) {
      rTV = rTV - G3(dWtV, i, j, kk) + (G3(dWtC, i, j - 1, kk) + G3(dWtC, i, j, kk)) * 0.5;
      return rTV * (0.5 * (V(i, j, kk) + V(i, j, kk - 1)));
    }
    double fv_ = rTV * (0.5 * (V(i, j, kk) + V(i, j, kk - 1)));
    fv_ = fv_ + 0.25 * (W(i, j, kk) * G2(rA, i, j) * (G3(maskC, i, j, kk) - G3(maskC, i, j, kk - 1)) +
                        W(i, j - 1, kk) * G2(rA, i, j - 1) * (G3(maskC, i, j - 1, kk) - G3(maskC, i, j - 1, kk - 1))) *
                    V(i, j, kk);
    return fv_;
  };

  {
    const double drF = f.drF[k - 1], recip_drF = f.recip_drF[k - 1];
    double gU = 0.0, gV = 0.0, guDiss = 0.0, gvDiss = 0.0;
    double dPhiHydX = 0.0, dPhiHydY = 0.0;
    if (valid && inner && PART != 2) {
      // CALC_GRAD_PHI_HYD (calc_grad_phi_hyd.F:152-171), phi0surf = 0
      // r* (select_rStar >= 2, nonlinFreeSurf >= 4): varLoc = phiHydC*rStarFacC + phi0surf (:30-47)
      const bool rsc = rstar && p.select_rStar >= 2 && p.nonlinFreeSurf >= 4;
      auto varLoc = [&](int ii, int jj) {
        return rsc ? G3(phiHydC, ii, jj, k) * G2(rStarFacC, ii, jj) + 0.0 : G3(phiHydC, ii, jj, k) + 0.0;
      };
      const double vl = varLoc(i, j);
      if (i >= 1) dPhiHydX = G2(recip_dxC, i, j) * (vl - varLoc(i - 1, j));
      if (j >= 1) dPhiHydY = G2(recip_dyC, i, j) * (vl - varLoc(i, j - 1));
      if (rstar && p.select_rStar >= 2) {
        // calc_grad_phi_hyd.F:173-214 (fluidIsWater, z-coords, generalForm = F)
        const double factorP = p.gravity * (1.0 / p.rhoConst) * 0.5, rCk = f.rC[k - 1];
        auto vl2 = [&](int ii, int jj) { return G2(etaH, ii, jj) * (1.0 + rCk * G2(recip_Rcol, ii, jj)); };
        const double e0 = vl2(i, j), a0 = G3(alphaRho, i, j, k);
        if (i >= 1)
          dPhiHydX = dPhiHydX + factorP * (G3(alphaRho, i - 1, j, k) + a0) * (e0 - vl2(i - 1, j)) * G2(recip_dxC, i, j);
        if (j >= 1)
          dPhiHydY = dPhiHydY + factorP * (G3(alphaRho, i, j - 1, k) + a0) * (e0 - vl2(i, j - 1)) * G2(recip_dyC, i, j);
      }
    }
    if (valid && inner) {
      const double rhFacW = G3(recip_hFacW, i, j, k), rhFacS = G3(recip_hFacS, i, j, k);
      const double hZ = hfacz(d, f, i, j, k, t);
      if constexpr (VI) {
        vecinv_tend(VIGlobal{d, p, f, k, t}, d, p, f, i, j, k, t, gU, gV, guDiss, gvDiss);
      } else {
      // ---------------- advection (mom_u_adv_uu/vu/wu.F, mom_v_adv_uv/vv/wv.F)
      if (PART != 2 && p.momAdvection) {
        const double fVerUkm = fverU(k), fVerUkp = fverU(k + 1);
        const double fVerVkm = fverV(k), fVerVkp = fverV(k + 1);
        // uTrans / vTrans (mom_fluxform.F:287-327)
#define UTR(ii, jj) (U(ii, jj, k) * (G2(dyG, ii, jj) * drF * G3(hFacW, ii, jj, k)))
#define VTR(ii, jj) (V(ii, jj, k) * (G2(dxG, ii, jj) * drF * G3(hFacS, ii, jj, k)))
        const double fZi = 0.25 * (UTR(i, j) + UTR(i + 1, j)) * (U(i, j, k) + U(i + 1, j, k));
        const double fZm = 0.25 * (UTR(i - 1, j) + UTR(i, j)) * (U(i - 1, j, k) + U(i, j, k));
        const double fMp = 0.25 * (VTR(i, j + 1) + VTR(i - 1, j + 1)) * (U(i, j + 1, k) + U(i, j, k));
        const double fMi = 0.25 * (VTR(i, j) + VTR(i - 1, j)) * (U(i, j, k) + U(i, j - 1, k));
        gU = -rhFacW * recip_drF * G2(recip_rAw, i, j) *
             ((fZi - fZm) * uDudxFac + (fMp - fMi) * vDudyFac + (fVerUkp - fVerUkm) * p.rkSign * rVelDudrFac);
        const double gZp = 0.25 * (UTR(i + 1, j) + UTR(i + 1, j - 1)) * (V(i + 1, j, k) + V(i, j, k));
        const double gZi = 0.25 * (UTR(i, j) + UTR(i, j - 1)) * (V(i, j, k) + V(i - 1, j, k));
        const double gMi = 0.25 * (VTR(i, j) + VTR(i, j + 1)) * (V(i, j, k) + V(i, j + 1, k));
        const double gMm = 0.25 * (VTR(i, j - 1) + VTR(i, j)) * (V(i, j - 1, k) + V(i, j, k));
        gV = -rhFacS * recip_drF * G2(recip_rAs, i, j) *
             ((gZp - gZi) * uDudxFac + (gMi - gMm) * vDudyFac + (fVerVkp - fVerVkm) * p.rkSign * rVelDudrFac);
        if (rstar) {   // mom_fluxform.F:527-548, 787-808
          gU = gU - (G2(rStarExpW, i, j) - 1.0) / p.deltaTFreeSurf * U(i, j, k);
          gV = gV - (G2(rStarExpS, i, j) - 1.0) / p.deltaTFreeSurf * V(i, j, k);
        }
#undef UTR
#undef VTR
      }
      // ---------------- viscosity (mom_u/v_x/y/rviscflux.F, sidedrag, botdrag)
      if (PART != 1 && p.momViscosity) {
        // U: xviscflux at i and i-1, yviscflux at j+1 and j
        // v4F = del2u / del2v from k_del2uv (0 without biharmonic viscosity)
        const bool bh = p.viscA4D != 0.0 || p.viscA4Z != 0.0;
        auto D2U = [&](int ii, int jj) { return bh ? G3(del2u, ii, jj, k) : 0.0; };
        auto D2V = [&](int ii, int jj) { return bh ? G3(del2v, ii, jj, k) : 0.0; };
        const double d2u = D2U(i, j), d2v = D2V(i, j);
        const double fZi = G2(dyF, i, j) * drF * G3(hFacC, i, j, k) *
                           (-p.viscAhD * (U(i + 1, j, k) - U(i, j, k)) * 1.0 + p.viscA4D * (D2U(i + 1, j) - d2u) * 1.0) *
                           G2(recip_dxF, i, j);
        const double fZm = G2(dyF, i - 1, j) * drF * G3(hFacC, i - 1, j, k) *
                           (-p.viscAhD * (U(i, j, k) - U(i - 1, j, k)) * 1.0 + p.viscA4D * (d2u - D2U(i - 1, j)) * 1.0) *
                           G2(recip_dxF, i - 1, j);
        const double hZp = hfacz(d, f, i, j + 1, k, t);
        const double fMp = G2(dxV, i, j + 1) * drF * hZp *
                           (-p.viscAhZ * (U(i, j + 1, k) - U(i, j, k)) + p.viscA4Z * (D2U(i, j + 1) - d2u)) *
                           G2(recip_dyU, i, j + 1);
        const double fMi = G2(dxV, i, j) * drF * hZ * (-p.viscAhZ * (U(i, j, k) - U(i, j - 1, k)) + p.viscA4Z * (d2u - D2U(i, j - 1))) *
                           G2(recip_dyU, i, j);
        double fVrUp = 0.0, fVrDw = 0.0;
        if (k > 1)
          fVrUp = -p.viscAr * G2(rAw, i, j) * (U(i, j, k) - U(i, j, k - 1)) * p.rkSign * f.recip_drC[k - 1] *
                  G3(maskW, i, j, k) * G3(maskW, i, j, k - 1);
        if (k + 1 <= Nr)
          fVrDw = -p.viscAr * G2(rAw, i, j) * (U(i, j, k + 1) - U(i, j, k)) * p.rkSign * f.recip_drC[k] *
                  G3(maskW, i, j, k + 1) * G3(maskW, i, j, k);
        guDiss = -rhFacW * recip_drF * G2(recip_rAw, i, j) *
                 ((fZi - fZm) * AhDudxFac + (fMp - fMi) * AhDudyFac + (fVrDw - fVrUp) * p.rkSign * ArDudrFac);
        if (p.no_slip_sides) {
          // MOM_U_SIDEDRAG with NONLIN_FRSURF: h0FacW - h0FacZ (h0Fac = hFac at rest)
          const double hS = G3(h0FacW, i, j, k) - h0facz(d, p, f, i, j, k, t);
          const double hN = G3(h0FacW, i, j, k) - h0facz(d, p, f, i, j + 1, k, t);
          const double u0 = U(i, j, k);
          const double vF = -rhFacW * recip_drF * G2(recip_rAw, i, j) *
                            (hS * G2(dxV, i, j) * G2(recip_dyU, i, j) * (p.viscAhZ * u0 - p.viscA4Z * d2u) +
                             hN * G2(dxV, i, j + 1) * G2(recip_dyU, i, j + 1) * (p.viscAhZ * u0 - p.viscA4Z * d2u)) *
                            drF * p.sideDragFactor;
          guDiss = guDiss + vF;
        }
        if (p.no_slip_bottom) {
          const int kDn = (k + 1 < Nr) ? k + 1 : Nr, kLowF = k + 1;
          const double recDrC = (k == Nr) ? recip_drF : f.recip_drC[kLowF - 1];
          double cD = 0.0 * 1.0;
          cD = cD + p.viscAr * recDrC * 2.0;
          cD = (k == Nr) ? cD * G3(maskW, i, j, k) : cD * G3(maskW, i, j, k) * (1.0 - G3(maskW, i, j, kDn));
          guDiss = guDiss - cD * U(i, j, k) * rhFacW * recip_drF;
        }
        // V: xviscflux at i+1 and i, yviscflux at j and j-1
        const double hZe = hfacz(d, f, i + 1, j, k, t);
        const double gZp = G2(dyU, i + 1, j) * drF * hZe *
                           (-p.viscAhZ * (V(i + 1, j, k) - V(i, j, k)) * 1.0 + p.viscA4Z * (D2V(i + 1, j) - d2v) * 1.0) *
                           G2(recip_dxV, i + 1, j);
        const double gZi = G2(dyU, i, j) * drF * hZ *
                           (-p.viscAhZ * (V(i, j, k) - V(i - 1, j, k)) * 1.0 + p.viscA4Z * (d2v - D2V(i - 1, j)) * 1.0) *
                           G2(recip_dxV, i, j);
        const double gMi = G2(dxF, i, j) * drF * G3(hFacC, i, j, k) *
                           (-p.viscAhD * (V(i, j + 1, k) - V(i, j, k)) + p.viscA4D * (D2V(i, j + 1) - d2v)) * G2(recip_dyF, i, j);
        const double gMm = G2(dxF, i, j - 1) * drF * G3(hFacC, i, j - 1, k) *
                           (-p.viscAhD * (V(i, j, k) - V(i, j - 1, k)) + p.viscA4D * (d2v - D2V(i, j - 1))) *
                           G2(recip_dyF, i, j - 1);
        double gVrUp = 0.0, gVrDw = 0.0;
        if (k > 1)
          gVrUp = -p.viscAr * G2(rAs, i, j) * (V(i, j, k) - V(i, j, k - 1)) * p.rkSign * f.recip_drC[k - 1] *
                  G3(maskS, i, j, k) * G3(maskS, i, j, k - 1);
        if (k + 1 <= Nr)
          gVrDw = -p.viscAr * G2(rAs, i, j) * (V(i, j, k + 1) - V(i, j, k)) * p.rkSign * f.recip_drC[k] *
                  G3(maskS, i, j, k + 1) * G3(maskS, i, j, k);
        gvDiss = -rhFacS * recip_drF * G2(recip_rAs, i, j) *
                 ((gZp - gZi) * AhDudxFac + (gMi - gMm) * AhDudyFac + (gVrDw - gVrUp) * p.rkSign * ArDudrFac);
        if (p.no_slip_sides) {
          const double hW = G3(h0FacS, i, j, k) - h0facz(d, p, f, i, j, k, t);
          const double hE = G3(h0FacS, i, j, k) - h0facz(d, p, f, i + 1, j, k, t);
          const double v0 = V(i, j, k);
          const double vF = -rhFacS * recip_drF * G2(recip_rAs, i, j) *
                            (hW * G2(dyU, i, j) * G2(recip_dxV, i, j) * (p.viscAhZ * v0 - p.viscA4Z * d2v) +
                             hE * G2(dyU, i + 1, j) * G2(recip_dxV, i + 1, j) * (p.viscAhZ * v0 - p.viscA4Z * d2v)) *
                            drF * p.sideDragFactor;
          gvDiss = gvDiss + vF;
        }
        if (p.no_slip_bottom) {
          const int kDn = (k + 1 < Nr) ? k + 1 : Nr, kLowF = k + 1;
          const double recDrC = (k == Nr) ? recip_drF : f.recip_drC[kLowF - 1];
          double cD = 0.0 * 1.0;
          cD = cD + p.viscAr * recDrC * 2.0;
          cD = (k == Nr) ? cD * G3(maskS, i, j, k) : cD * G3(maskS, i, j, k) * (1.0 - G3(maskS, i, j, kDn));
          gvDiss = gvDiss - cD * V(i, j, k) * rhFacS * recip_drF;
        }
      }
      // ---------------- spherical metric terms (mom_u/v_metric_sphere.F, mom_fluxform.F:714-721, 973-980)
      if (PART != 2 && p.useNHMTerms) {
        // MOM_U/V_METRIC_NH (pkg/mom_common/mom_u_metric_nh.F:56-68, mom_v_metric_nh.F), mtNHFac = 1
        const int kp1 = k + 1 < Nr ? k + 1 : Nr;
        const double ov = (k == Nr) ? 0.0 : 1.0;
        gU = gU + 1.0 * (U(i, j, k) * p.recip_rSphere * 0.25 *
                         ((W(i - 1, j, kp1) + W(i, j, kp1)) * ov + (W(i - 1, j, k) + W(i, j, k))) * p.gravitySign);
        gV = gV + 1.0 * (V(i, j, k) * p.recip_rSphere * 0.25 *
                         ((W(i, j - 1, kp1) + W(i, j, kp1)) * ov + (W(i, j - 1, k) + W(i, j, k))) * p.gravitySign);
      }
      if (PART != 2 && p.metricSphere) {
        const double mTu = U(i, j, k) * p.recip_rSphere * 0.25 *
                           (V(i, j, k) + V(i - 1, j, k) + V(i, j + 1, k) + V(i - 1, j + 1, k)) * G2(tanPhiAtU, i, j);
        gU = gU + p.mtFacMom * mTu;
        const double ub = U(i, j, k) + U(i + 1, j, k) + U(i, j - 1, k) + U(i + 1, j - 1, k);
        const double mTv = -(p.recip_rSphere * 0.25 * ub * 0.25 * ub * G2(tanPhiAtV, i, j));
        gV = gV + p.mtFacMom * mTv;
      }
      // ---------------- Coriolis (mom_u_coriolis.F, mom_v_coriolis.F); with the CD scheme
      // it is applied in TIMESTEP instead (mom_fluxform.F:995, k_cd_scheme)
      if (PART != 2 && p.useCoriolis && !p.useCDscheme) {
        const int sc = p.selectCoriScheme;
        double c;
        if (sc >= 2)
          c = 0.5 * (G2(fCori, i, j) * 0.5 * (V(i, j, k) + V(i, j + 1, k)) +
                     G2(fCori, i - 1, j) * 0.5 * (V(i - 1, j, k) + V(i - 1, j + 1, k)));
        else
          c = 0.5 * (G2(fCori, i, j) + G2(fCori, i - 1, j)) * 0.25 *
              (V(i, j, k) + V(i, j + 1, k) + V(i - 1, j, k) + V(i - 1, j + 1, k));
        if (sc == 1 || sc == 3)
          c = c * 4.0 / fmax(1.0, G3(maskS, i, j, k) + G3(maskS, i, j + 1, k) + G3(maskS, i - 1, j, k) + G3(maskS, i - 1, j + 1, k));
        gU = gU + fuFac * c;
        if (sc >= 2)
          c = -0.5 * (G2(fCori, i, j) * 0.5 * (U(i, j, k) + U(i + 1, j, k)) +
                      G2(fCori, i, j - 1) * 0.5 * (U(i, j - 1, k) + U(i + 1, j - 1, k)));
        else
          c = -0.5 * (G2(fCori, i, j) + G2(fCori, i, j - 1)) * 0.25 *
              (U(i, j, k) + U(i + 1, j, k) + U(i, j - 1, k) + U(i + 1, j - 1, k));
        if (sc == 1 || sc == 3)
          c = c * 4.0 / fmax(1.0, G3(maskW, i, j, k) + G3(maskW, i + 1, j, k) + G3(maskW, i, j - 1, k) + G3(maskW, i + 1, j - 1, k));
        gV = gV + fvFac * c;
      }
      if (PART != 2 && p.select3dCoriScheme >= 1) {
        // MOM_U_CORIOLIS_NH (pkg/mom_common/mom_u_coriolis_nh.F:60-76), angleCosC = 1; the V
        // component only on curvilinear / rotated grids (mom_fluxform.F:1025-1040)
        const int kp1 = k + 1 < Nr ? k + 1 : Nr;
        const double wMsk = (k == Nr) ? 0.0 : 1.0;
        const double c = 0.5 * (G2(fCoriCos, i, j) * 1.0 * 0.5 * (W(i, j, k) + W(i, j, kp1) * wMsk) +
                                G2(fCoriCos, i - 1, j) * 1.0 * 0.5 * (W(i - 1, j, k) + W(i - 1, j, kp1) * wMsk)) *
                         p.gravitySign;
        gU = gU + fuFac * c;
      }
      // mom_fluxform.F:1044-1051
      gU = gU * G3(maskW, i, j, k);
      guDiss = guDiss * G3(maskW, i, j, k);
      gV = gV * G3(maskS, i, j, k);
      gvDiss = gvDiss * G3(maskS, i, j, k);
      }   // vectorInvariantMomentum
    }
    if constexpr (PART == 2) {   // hand the viscous sum to the PART 1 wave of the same point
      *sD = COMP == 1 ? guDiss : gvDiss;
      __syncthreads();
      return;
    }
    if constexpr (PART == 1) {
      __syncthreads();
      if (COMP == 1) guDiss = *sD;
      else gvDiss = *sD;
      if (!valid) return;
    }
    // ---------------- TIMESTEP (timestep.F:104-388)
    double guExt = 0.0, gvExt = 0.0;
    if (p.momForcing && k == 1) {
      // APPLY_FORCING_U/V (apply_forcing.F:81-88) on j=0..sNy+1,i=1..sNx+1 (U) / i=0..sNx+1,j=1..sNy+1 (V)
      if (j >= 0 && j <= d.sNy + 1 && i >= 1 && i <= d.sNx + 1)
        guExt = guExt + p.foFacMom * (AR2(fu, q2) * mass2rUnit) * recip_drF * G3(recip_hFacW, i, j, k);
      if (j >= 1 && j <= d.sNy + 1 && i >= 0 && i <= d.sNx + 1)
        gvExt = gvExt + p.foFacMom * (AR2(fv, q2) * mass2rUnit) * recip_drF * G3(recip_hFacS, i, j, k);
    }
    if (inner) {
      // timestep.F:116-126 synchronous time step: gU -= phFac*dPhiHydX
      gU = gU - p.pfFacMom * dPhiHydX;
      gV = gV - p.pfFacMom * dPhiHydY;
      if (p.momViscosity && p.momDissip_In_AB) { gU = gU + guDiss; gV = gV + gvDiss; }
      if (p.momForcing && p.momForcingOutAB != 1) { gU = gU + guExt; gV = gV + gvExt; }
    }
    // ADAMS_BASHFORTH2 over the whole halo-inclusive slab (adams_bashforth2.F:81-88)
    const long q3 = MG_I3(d, i, j, k, t);
    {
      const double gUo = COMP != 2 ? AR3(guNm1, q3) : 0.0, gVo = COMP != 1 ? AR3(gvNm1, q3) : 0.0;
      double a = abFac * (gU - gUo);
      if (COMP != 2) AR3(guNm1, q3) = gU;
      gU = gU + a;
      a = abFac * (gV - gVo);
      if (COMP != 1) AR3(gvNm1, q3) = gV;
      gV = gV + a;
    }
    double gUtmp = 0.0, gVtmp = 0.0;   // timestep.F local arrays: 0 outside iMin..iMax, jMin..jMax
    if (inner) {
      gUtmp = gU; gVtmp = gV;
      if (p.momForcing && p.momForcingOutAB == 1) { gUtmp = gUtmp + guExt; gVtmp = gVtmp + gvExt; }
      if (p.momViscosity && !p.momDissip_In_AB) { gUtmp = gUtmp + guDiss; gVtmp = gVtmp + gvDiss; }
      if (!p.useCDscheme) {
        if (rstar && p.nonlinFreeSurf > 1) {   // timestep.F:274-284
          gUtmp = gUtmp / G2(rStarExpW, i, j);
          gVtmp = gVtmp / G2(rStarExpS, i, j);
        }
        // u* = u + dt*(gUtmp + gUdPx)*maskW  (timestep.F:373-388), gUdPx = 0 for implicSurfPress = 1
        gU = U(i, j, k) + p.deltaTMom * (gUtmp + 0.0) * G3(maskW, i, j, k);
        gV = V(i, j, k) + p.deltaTMom * (gVtmp + 0.0) * G3(maskS, i, j, k);
      }
    }
    if (p.useCDscheme) {   // k_cd_scheme finishes u*
      if (COMP != 2) AR3(cdU, q3) = gUtmp;
      if (COMP != 1) AR3(cdV, q3) = gVtmp;
    }
    if (COMP != 2) AR3(gU, q3) = gU;
    if (COMP != 1) AR3(gV, q3) = gV;
  }
#undef U
#undef V
#undef W
#undef G2
#undef G3
}
template <bool VI, int COMP>
__device__ __forceinline__ void mom_step_point(const Dims &d, const Params &p, const Fields &f, const int *iterPtr,
                                               int lblock) {
  MG_PLANE_LB(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, z, lblock)
  mom_step_ijz<VI, COMP>(d, p, f, iterPtr, i, j, z, true, nullptr);
}
// MOM_FLUXFORM + TIMESTEP + AB2 with four threads per point: wave 0 the U component's
// advective / metric / Coriolis / pressure terms, wave 1 its viscous terms, waves 2, 3 the
// same for V -- 64 points per workgroup, the viscous sums handed over through LDS; each
// thread's dependency chain is about half of k_mom_step_uv's.  The same expressions, summed in
// the same order: bit-identical.
__host__ __device__ __forceinline__ int mom_ff4_blocks(const Dims &d) { return (d.nx * d.ny + 63) / 64 * d.Nr * d.nT; }
// whether the flux-form momentum runs four threads per point (MGCM_MOM_FF4=0 never, 1 default,
// 2 also inside config 2's fused grid; read per launch).  Measured (profiles/r03/ff4/): config
// 4 0.1438 against 0.1458 ms/step with the U/V halves; inside k_dt_l2 beside the tracer
// right-hand sides (config 2) 0.3215 against 0.3092 -- there the U/V halves stay
inline bool mom_ff4_on(bool fused = false) {
  const char *e = getenv("MGCM_MOM_FF4");
  const int v = e ? atoi(e) : 1;
  return fused ? v == 2 : v != 0;
}
__device__ __forceinline__ void mom_ff4_body(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, int lb) {
  __shared__ double sD[128];
  const int np = d.nx * d.ny, nbp = (np + 63) / 64;
  const int z = lb / nbp, lane = (int)threadIdx.x & 63, w = (int)threadIdx.x >> 6;
  const int q = (lb % nbp) * 64 + lane;
  const bool valid = q < np;
  const int i = 1 - d.OLx + (valid ? q % d.nx : 0), j = 1 - d.OLy + (valid ? q / d.nx : 0);
  double *slot = sD + (w >> 1) * 64 + lane;
  switch (w) {
    case 0: mom_step_ijz<false, 1, 1>(d, p, f, iterPtr, i, j, z, valid, slot); break;
    case 1: mom_step_ijz<false, 1, 2>(d, p, f, iterPtr, i, j, z, valid, slot); break;
    case 2: mom_step_ijz<false, 2, 1>(d, p, f, iterPtr, i, j, z, valid, slot); break;
    default: mom_step_ijz<false, 2, 2>(d, p, f, iterPtr, i, j, z, valid, slot); break;
  }
}
__global__ void __launch_bounds__(256) k_mom_ff4(Dims d, Params p, Fields f, const int *iterPtr) {
  mom_ff4_body(d, p, f, iterPtr, mg_xcd_block());
}

template <bool VI>
__global__ void __launch_bounds__(256) k_mom_step(Dims d, Params p, Fields f, const int *iterPtr) {
  mom_step_point<VI, 0>(d, p, f, iterPtr, mg_xcd_block());
}
// the U and V halves as separate threads: even logical blocks U, odd V of the same plane
// range (neighbouring blocks, so both halves of a region share an XCD's L2)
template <bool VI>
__global__ void __launch_bounds__(256) k_mom_step_uv(Dims d, Params p, Fields f, const int *iterPtr) {
  const int lb = mg_xcd_block();
  if (lb & 1) mom_step_point<VI, 2>(d, p, f, iterPtr, lb >> 1);
  else mom_step_point<VI, 1>(d, p, f, iterPtr, lb >> 1);
}

// CD_CODE_SCHEME (pkg/cd_code/cd_code_scheme.F:85-236, called from timestep.F:228-270;
// staggerTimeStep = F so phxFac = phyFac = 0) for one (i,j,k) of 2-OL..sN+OL-1:
// the D-grid velocities uVelD/vVelD are stepped and relaxed, the Coriolis terms
// guCor/gvCor added to gUtmp/gVtmp (cdU/cdV from k_mom_step), and u* formed on the
// TIMESTEP range 0..sN+1.  uNM1/vNM1 = u, v is done by k_sfp_rhs (after this kernel,
// whose neighbours still read the old values).
__device__ __forceinline__ void cd_scheme_body(const Dims &d, const Params &p, const Fields &f, const int *iterPtr,
                                               int lb) {
  MG_PLANE_LB(2 - d.OLx, d.nx - 2, 2 - d.OLy, d.ny - 2, z, lb)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  const int myIter = *iterPtr;
  const double ab15 = myIter == 0 ? 1.0 : 1.5 + p.epsAB_CD;
  const double ab05 = myIter == 0 ? -0.0 : -0.5 - p.epsAB_CD;
#define G2(a_, ii, jj) f.a_[MG_I2(d, ii, jj, t)]
#define G3(a_, ii, jj, kk) f.a_[MG_I3(d, ii, jj, kk, t)]
  auto pf = [&](int ii, int jj) { return G2(Bo_surf, ii, jj) * (ab15 * G2(etaN, ii, jj) + ab05 * G2(etaNm1, ii, jj)); };
  auto afV = [&](int ii, int jj) {
    return (G3(cdV, ii, jj, k) - (G2(recip_dyC, ii, jj) * (pf(ii, jj) - pf(ii, jj - 1)) + 0.0)) * G3(maskS, ii, jj, k);
  };
  auto afU = [&](int ii, int jj) {
    return (G3(cdU, ii, jj, k) - (G2(recip_dxC, ii, jj) * (pf(ii, jj) - pf(ii - 1, jj)) + 0.0)) * G3(maskW, ii, jj, k);
  };
  const long q3 = MG_I3(d, i, j, k, t);
  // vVelD at this U point
  double vf = ((afV(i, j) + afV(i - 1, j + 1)) + (afV(i - 1, j) + afV(i, j + 1))) * 0.25 * G3(maskW, i, j, k) -
              (G2(fCori, i, j) + G2(fCori, i - 1, j)) * 0.5 * (ab15 * G3(uVel, i, j, k) + ab05 * G3(uNM1, i, j, k));
  double vD = AR3(vVelD, q3) + p.deltaTMom * vf;
  vD = (p.rCD * vD +
        (1.0 - p.rCD) *
            (ab15 * ((G3(vVel, i, j, k) + G3(vVel, i - 1, j + 1, k)) + (G3(vVel, i - 1, j, k) + G3(vVel, i, j + 1, k))) * 0.25 +
             ab05 * ((G3(vNM1, i, j, k) + G3(vNM1, i - 1, j + 1, k)) + (G3(vNM1, i - 1, j, k) + G3(vNM1, i, j + 1, k))) * 0.25)) *
       G3(maskW, i, j, k);
  AR3(vVelD, q3) = vD;
  const double guCor = (G2(fCori, i, j) + G2(fCori, i - 1, j)) * 0.5 * vD * p.cfFacMom;
  // uVelD at this V point
  vf = ((afU(i, j) + afU(i + 1, j - 1)) + (afU(i + 1, j) + afU(i, j - 1))) * 0.25 * G3(maskS, i, j, k) +
       (G2(fCori, i, j) + G2(fCori, i, j - 1)) * 0.5 * (ab15 * G3(vVel, i, j, k) + ab05 * G3(vNM1, i, j, k));
  double uD = AR3(uVelD, q3) + p.deltaTMom * vf;
  uD = (p.rCD * uD +
        (1.0 - p.rCD) *
            (ab15 * ((G3(uVel, i, j, k) + G3(uVel, i + 1, j - 1, k)) + (G3(uVel, i, j - 1, k) + G3(uVel, i + 1, j, k))) * 0.25 +
             ab05 * ((G3(uNM1, i, j, k) + G3(uNM1, i + 1, j - 1, k)) + (G3(uNM1, i, j - 1, k) + G3(uNM1, i + 1, j, k))) * 0.25)) *
       G3(maskS, i, j, k);
  AR3(uVelD, q3) = uD;
  const double gvCor = -(G2(fCori, i, j) + G2(fCori, i, j - 1)) * 0.5 * uD * p.cfFacMom;
  if (i >= 0 && i <= d.sNx + 1 && j >= 0 && j <= d.sNy + 1) {
    double gUtmp = AR3(cdU, q3) + guCor, gVtmp = AR3(cdV, q3) + gvCor;
    if (p.nonlinFreeSurf > 1 && p.select_rStar > 0) {   // timestep.F:274-284
      gUtmp = gUtmp / G2(rStarExpW, i, j);
      gVtmp = gVtmp / G2(rStarExpS, i, j);
    }
    AR3(gU, q3) = G3(uVel, i, j, k) + p.deltaTMom * (gUtmp + 0.0) * G3(maskW, i, j, k);
    AR3(gV, q3) = G3(vVel, i, j, k) + p.deltaTMom * (gVtmp + 0.0) * G3(maskS, i, j, k);
  }
#undef G2
#undef G3
}
__global__ void __launch_bounds__(256) k_cd_scheme(Dims d, Params p, Fields f, const int *iterPtr) {
  cd_scheme_body(d, p, f, iterPtr, mg_xcd_block());
}

// ---------------------------------------------------------------------------------------
// MOM_VECINV + CALC_GRAD_PHI_HYD + TIMESTEP + ADAMS_BASHFORTH2 as a 2.5-D tiled sweep: one
// workgroup owns a BX x BY block of the DYNAMICS range 0..sN+1 of one tile and marches
// k = 1..Nr.  The level fields the stencils reach (u, v, w, hFacW, hFacS, hFacC on the
// block plus one ring) are staged in LDS once per level: u, v, hFac in three rotating
// slots (levels k-1, k, k+1: the vertical shear and the vertical viscous fluxes), w in
// two; level k+1 is loaded while level k's intermediates are formed.  KE, vort3, hFacZ,
// h0FacZ and hDiv are formed once per point of the block's (BX+1) x (BY+1) grid into LDS
// instead of being re-derived by every neighbour.  Masks and reciprocal hFacs come from
// the staged hFac (maskW = hFacW != 0, recip_hFacW = 1/hFacW: ini_masks_etc.F and
// update_r_star.F define them so).  vecinv_tend is the same template as the per-point
// kernel's (accessor VITile), so the two kernels agree bit for bit.
constexpr int VT_NT = 256, VT_EMAX = 352, VT_IMAX = 304;

struct VITile {
  const Dims &d; const Params &p; const Fields &f; int k, t, i0, j0, EW, IW;
  const double *sU, *sV, *sW, *sHW, *sHS, *sHC;   // [3][EMAX] / w [2][EMAX]
  const double *sKE, *sVort, *sHfz, *sH0fz, *sHDiv;   // [IMAX]
  __device__ __forceinline__ int e(int ii, int jj) const { return (jj - j0 + 1) * EW + (ii - i0 + 1); }
  template <int F> __device__ __forceinline__ double g2(int ii, int jj) const { return f.a2[(long)F * d.N2all + MG_I2(d, ii, jj, t)]; }
  __device__ __forceinline__ int sl(int kk) const { return (kk % 3) * VT_EMAX; }
  __device__ __forceinline__ double uVel(int ii, int jj, int kk) const { return sU[sl(kk) + e(ii, jj)]; }
  __device__ __forceinline__ double vVel(int ii, int jj, int kk) const { return sV[sl(kk) + e(ii, jj)]; }
  __device__ __forceinline__ double wVel(int ii, int jj, int kk) const { return sW[(kk & 1) * VT_EMAX + e(ii, jj)]; }
  __device__ __forceinline__ double hFacW(int ii, int jj, int kk) const { return sHW[sl(kk) + e(ii, jj)]; }
  __device__ __forceinline__ double hFacS(int ii, int jj, int kk) const { return sHS[sl(kk) + e(ii, jj)]; }
  __device__ __forceinline__ double hFacC(int ii, int jj, int kk) const { return sHC[sl(kk) + e(ii, jj)]; }
  __device__ __forceinline__ double maskW(int ii, int jj, int kk) const { return hFacW(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double maskS(int ii, int jj, int kk) const { return hFacS(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double maskC(int ii, int jj, int kk) const { return hFacC(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double recip_hFacW(int ii, int jj, int kk) const {
    const double h = hFacW(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double recip_hFacS(int ii, int jj, int kk) const {
    const double h = hFacS(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double recip_hFacC(int ii, int jj, int kk) const {
    const double h = hFacC(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double h0FacW(int ii, int jj, int kk) const { return AR3(h0FacW, MG_I3(d, ii, jj, kk, t)); }
  __device__ __forceinline__ double h0FacS(int ii, int jj, int kk) const { return AR3(h0FacS, MG_I3(d, ii, jj, kk, t)); }
  __device__ __forceinline__ int iv(int ii, int jj) const { return (jj - j0) * IW + (ii - i0); }       // vort grid
  __device__ __forceinline__ int id(int ii, int jj) const { return (jj - j0 + 1) * IW + (ii - i0 + 1); } // hDiv grid
  __device__ __forceinline__ double hfz(int ii, int jj) const { return sHfz[iv(ii, jj)]; }
  __device__ __forceinline__ double h0fz(int ii, int jj) const { return sH0fz[iv(ii, jj)]; }
  __device__ __forceinline__ double vort(int ii, int jj) const { return sVort[iv(ii, jj)]; }
  __device__ __forceinline__ double KE(int ii, int jj) const { return sKE[id(ii, jj)]; }
  __device__ __forceinline__ double hDiv(int ii, int jj) const { return sHDiv[id(ii, jj)]; }
};

__global__ void __launch_bounds__(VT_NT) k_mom_vi_tiled(Dims d, Params p, Fields f, const int *iterPtr, int BX, int BY,
                                                         int nbx, int nby, int KC, int nkc) {
  __shared__ double sU[3 * VT_EMAX], sV[3 * VT_EMAX], sHW[3 * VT_EMAX], sHS[3 * VT_EMAX], sHC[3 * VT_EMAX];
  __shared__ double sW[2 * VT_EMAX];
  __shared__ double sKE[VT_IMAX], sVort[VT_IMAX], sHfz[VT_IMAX], sH0fz[VT_IMAX], sHDiv[VT_IMAX];
  // block id: (i,j) block fastest, then the chunk of KC levels, then the tile
  const int nb = nbx * nby, lb = mg_xcd_block();
  const int t = d.t0 + lb / (nb * nkc), bxy = lb % nb, kb = 1 + ((lb / nb) % nkc) * KC;
  const int ke = kb + KC - 1 < d.Nr ? kb + KC - 1 : d.Nr;
  const int i0 = (bxy % nbx) * BX, j0 = (bxy / nbx) * BY;
  const int tid = threadIdx.x;
  const int EW = BX + 2, EN = (BX + 2) * (BY + 2), IW = BX + 1, IN = (BX + 1) * (BY + 1);
  const int Nr = d.Nr;
  const int i = i0 + tid % BX, j = j0 + tid / BX;
  const bool act = tid < BX * BY && i <= d.sNx + 1 && j <= d.sNy + 1;
  const int myIter = *iterPtr;
  const double abFac = (myIter == p.nIter0 && p.nIter0 == 0) ? 0.0 : 0.5 + p.abEps;   // adams_bashforth2.F:61-65
  const double mass2rUnit = 1.0 / p.rhoConst;
  const bool rstar = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
  const long q2 = MG_I2(d, i, j, t);
  VITile a{d, p, f, 1, t, i0, j0, EW, IW, sU, sV, sW, sHW, sHS, sHC, sKE, sVort, sHfz, sH0fz, sHDiv};
  // the block's extent: i0-1..i0+BX, j0-1..j0+BY, clipped to the array (points past it are
  // read by no active thread)
  auto ext_q3 = [&](int ee, int kk, bool &in) -> long {
    const int ii = i0 - 1 + ee % EW, jj = j0 - 1 + ee / EW;
    in = ii <= d.sNx + d.OLx && jj <= d.sNy + d.OLy;
    return MG_I3(d, in ? ii : 1, in ? jj : 1, kk, t);
  };
  double nU[2], nV[2], nW[2], nHW[2], nHS[2], nHC[2];
  auto fetch = [&](int kk) {
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int ee = tid + r * VT_NT;
      bool in = false;
      if (ee < EN) {
        const long q = ext_q3(ee, kk, in);
        nU[r] = in ? AR3(uVel, q) : 0.0; nV[r] = in ? AR3(vVel, q) : 0.0; nW[r] = in ? AR3(wVel, q) : 0.0;
        nHW[r] = in ? AR3(hFacW, q) : 0.0; nHS[r] = in ? AR3(hFacS, q) : 0.0; nHC[r] = in ? AR3(hFacC, q) : 0.0;
      }
    }
  };
  auto stash = [&](int kk) {
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int ee = tid + r * VT_NT;
      if (ee < EN) {
        const int o = (kk % 3) * VT_EMAX + ee;
        sU[o] = nU[r]; sV[o] = nV[r]; sHW[o] = nHW[r]; sHS[o] = nHS[r]; sHC[o] = nHC[r];
        sW[(kk & 1) * VT_EMAX + ee] = nW[r];
      }
    }
  };
  // levels kb-1 (the vertical shear / viscous flux partner above) and kb
  if (kb > 1) { fetch(kb - 1); stash(kb - 1); }
  fetch(kb);
  stash(kb);
  __syncthreads();
  for (int k = kb; k <= ke; k++) {
    a.k = k;
    if (k < Nr) fetch(k + 1);   // in flight while level k's intermediates are formed
    // per-level intermediates on the (BX+1) x (BY+1) grids
    for (int q = tid; q < IN; q += VT_NT) {
      const int ii = i0 + q % IW, jj = j0 + q / IW;          // vort / hFacZ grid: i0..i0+BX
      const bool ok = ii <= d.sNx + d.OLx && jj <= d.sNy + d.OLy;
      sHfz[q] = ok ? vi_hfacz(a, d, ii, jj, k) : 0.0;
      sH0fz[q] = ok ? vi_h0facz(a, d, p, ii, jj, k) : 0.0;
      sVort[q] = ok ? vi_vort(a, d, p, f, ii, jj, k, t) : 0.0;
      const int ih = ii - 1, jh = jj - 1;                     // KE / hDiv grid: i0-1..i0+BX-1
      sKE[q] = vi_KE(a, d, p, f, ih, jh, k, t);
      sHDiv[q] = vi_hdiv(a, d, p, f, ih, jh, k, t);
    }
    if (k < Nr) stash(k + 1);
    __syncthreads();
    if (act) {
      const long q3 = MG_I3(d, i, j, k, t);
      const double recip_drF = f.recip_drF[k - 1];
      double gU = 0.0, gV = 0.0, guDiss = 0.0, gvDiss = 0.0, dPhiHydX = 0.0, dPhiHydY = 0.0;
      {  // CALC_GRAD_PHI_HYD (calc_grad_phi_hyd.F:152-214), as k_mom_step
        const bool rsc = rstar && p.select_rStar >= 2 && p.nonlinFreeSurf >= 4;
        auto varLoc = [&](int ii, int jj) {
          return rsc ? AR3(phiHydC, MG_I3(d, ii, jj, k, t)) * AR2(rStarFacC, MG_I2(d, ii, jj, t)) + 0.0
                     : AR3(phiHydC, MG_I3(d, ii, jj, k, t)) + 0.0;
        };
        const double vl = varLoc(i, j);
        if (i >= 1) dPhiHydX = AR2(recip_dxC, q2) * (vl - varLoc(i - 1, j));
        if (j >= 1) dPhiHydY = AR2(recip_dyC, q2) * (vl - varLoc(i, j - 1));
        if (rstar && p.select_rStar >= 2) {
          const double factorP = p.gravity * (1.0 / p.rhoConst) * 0.5, rCk = f.rC[k - 1];
          auto vl2 = [&](int ii, int jj) { return AR2(etaH, MG_I2(d, ii, jj, t)) * (1.0 + rCk * AR2(recip_Rcol, MG_I2(d, ii, jj, t))); };
          const double e0 = vl2(i, j), a0 = AR3(alphaRho, q3);
          if (i >= 1)
            dPhiHydX = dPhiHydX + factorP * (AR3(alphaRho, MG_I3(d, i - 1, j, k, t)) + a0) * (e0 - vl2(i - 1, j)) * AR2(recip_dxC, q2);
          if (j >= 1)
            dPhiHydY = dPhiHydY + factorP * (AR3(alphaRho, MG_I3(d, i, j - 1, k, t)) + a0) * (e0 - vl2(i, j - 1)) * AR2(recip_dyC, q2);
        }
      }
      vecinv_tend(a, d, p, f, i, j, k, t, gU, gV, guDiss, gvDiss);
      // TIMESTEP (timestep.F:104-388), as k_mom_step
      double guExt = 0.0, gvExt = 0.0;
      if (p.momForcing && k == 1) {
        if (j >= 0 && j <= d.sNy + 1 && i >= 1 && i <= d.sNx + 1)
          guExt = guExt + p.foFacMom * (AR2(fu, q2) * mass2rUnit) * recip_drF * a.recip_hFacW(i, j, k);
        if (j >= 1 && j <= d.sNy + 1 && i >= 0 && i <= d.sNx + 1)
          gvExt = gvExt + p.foFacMom * (AR2(fv, q2) * mass2rUnit) * recip_drF * a.recip_hFacS(i, j, k);
      }
      gU = gU - p.pfFacMom * dPhiHydX;
      gV = gV - p.pfFacMom * dPhiHydY;
      if (p.momViscosity && p.momDissip_In_AB) { gU = gU + guDiss; gV = gV + gvDiss; }
      if (p.momForcing && p.momForcingOutAB != 1) { gU = gU + guExt; gV = gV + gvExt; }
      {  // ADAMS_BASHFORTH2 (adams_bashforth2.F:81-88)
        const double gUo = AR3(guNm1, q3), gVo = AR3(gvNm1, q3);
        double ab = abFac * (gU - gUo);
        AR3(guNm1, q3) = gU;
        gU = gU + ab;
        ab = abFac * (gV - gVo);
        AR3(gvNm1, q3) = gV;
        gV = gV + ab;
      }
      double gUtmp = gU, gVtmp = gV;
      if (p.momForcing && p.momForcingOutAB == 1) { gUtmp = gUtmp + guExt; gVtmp = gVtmp + gvExt; }
      if (p.momViscosity && !p.momDissip_In_AB) { gUtmp = gUtmp + guDiss; gVtmp = gVtmp + gvDiss; }
      if (rstar && p.nonlinFreeSurf > 1) {
        gUtmp = gUtmp / AR2(rStarExpW, q2);
        gVtmp = gVtmp / AR2(rStarExpS, q2);
      }
      AR3(gU, q3) = a.uVel(i, j, k) + p.deltaTMom * (gUtmp + 0.0) * a.maskW(i, j, k);
      AR3(gV, q3) = a.vVel(i, j, k) + p.deltaTMom * (gVtmp + 0.0) * a.maskS(i, j, k);
    }
    __syncthreads();
  }
}

// One level per workgroup: level k of the block plus one ring staged in LDS (u, v, w,
// hFacW, hFacS, hFacC), the intermediates formed once per point into LDS; the other
// levels' values (vertical shear, vertical viscous fluxes, masks at k-1 / k+1, w(k+1))
// are read where they lie.  No level march: many small workgroups, modest registers.
struct VILevel {
  const Dims &d; const Params &p; const Fields &f; int k, t, i0, j0, EW, IW;
  const double *sU, *sV, *sW, *sHW, *sHS, *sHC;   // level k on the extent
  const double *sKE, *sVort, *sHfz, *sH0fz, *sHDiv;
  __device__ __forceinline__ int e(int ii, int jj) const { return (jj - j0 + 1) * EW + (ii - i0 + 1); }
  __device__ __forceinline__ long g(int ii, int jj, int kk) const { return MG_I3(d, ii, jj, kk, t); }
  template <int F> __device__ __forceinline__ double g2(int ii, int jj) const { return f.a2[(long)F * d.N2all + MG_I2(d, ii, jj, t)]; }
  __device__ __forceinline__ double uVel(int ii, int jj, int kk) const { return kk == k ? sU[e(ii, jj)] : AR3(uVel, g(ii, jj, kk)); }
  __device__ __forceinline__ double vVel(int ii, int jj, int kk) const { return kk == k ? sV[e(ii, jj)] : AR3(vVel, g(ii, jj, kk)); }
  __device__ __forceinline__ double wVel(int ii, int jj, int kk) const { return kk == k ? sW[e(ii, jj)] : AR3(wVel, g(ii, jj, kk)); }
  __device__ __forceinline__ double hFacW(int ii, int jj, int kk) const { return kk == k ? sHW[e(ii, jj)] : AR3(hFacW, g(ii, jj, kk)); }
  __device__ __forceinline__ double hFacS(int ii, int jj, int kk) const { return kk == k ? sHS[e(ii, jj)] : AR3(hFacS, g(ii, jj, kk)); }
  __device__ __forceinline__ double hFacC(int ii, int jj, int kk) const { return kk == k ? sHC[e(ii, jj)] : AR3(hFacC, g(ii, jj, kk)); }
  __device__ __forceinline__ double maskW(int ii, int jj, int kk) const { return hFacW(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double maskS(int ii, int jj, int kk) const { return hFacS(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double maskC(int ii, int jj, int kk) const { return hFacC(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double recip_hFacW(int ii, int jj, int kk) const {
    const double h = hFacW(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double recip_hFacS(int ii, int jj, int kk) const {
    const double h = hFacS(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double recip_hFacC(int ii, int jj, int kk) const {
    const double h = hFacC(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double h0FacW(int ii, int jj, int kk) const { return AR3(h0FacW, g(ii, jj, kk)); }
  __device__ __forceinline__ double h0FacS(int ii, int jj, int kk) const { return AR3(h0FacS, g(ii, jj, kk)); }
  __device__ __forceinline__ int iv(int ii, int jj) const { return (jj - j0) * IW + (ii - i0); }
  __device__ __forceinline__ int id(int ii, int jj) const { return (jj - j0 + 1) * IW + (ii - i0 + 1); }
  __device__ __forceinline__ double hfz(int ii, int jj) const { return sHfz[iv(ii, jj)]; }
  __device__ __forceinline__ double h0fz(int ii, int jj) const { return sH0fz[iv(ii, jj)]; }
  __device__ __forceinline__ double vort(int ii, int jj) const { return sVort[iv(ii, jj)]; }
  __device__ __forceinline__ double KE(int ii, int jj) const { return sKE[id(ii, jj)]; }
  __device__ __forceinline__ double hDiv(int ii, int jj) const { return sHDiv[id(ii, jj)]; }
};

__global__ void __launch_bounds__(VT_NT) k_mom_vi_level(Dims d, Params p, Fields f, const int *iterPtr, int BX, int BY,
                                                         int nbx, int nby) {
  __shared__ double sU[VT_EMAX], sV[VT_EMAX], sW[VT_EMAX], sHW[VT_EMAX], sHS[VT_EMAX], sHC[VT_EMAX];
  __shared__ double sKE[VT_IMAX], sVort[VT_IMAX], sHfz[VT_IMAX], sH0fz[VT_IMAX], sHDiv[VT_IMAX];
  // block id: (i,j) block fastest, then the level, then the tile
  const int nb = nbx * nby, lb = mg_xcd_block();
  const int t = d.t0 + lb / (nb * d.Nr), bxy = lb % nb, k = 1 + (lb / nb) % d.Nr;
  const int i0 = (bxy % nbx) * BX, j0 = (bxy / nbx) * BY;
  const int tid = threadIdx.x;
  const int EW = BX + 2, EN = (BX + 2) * (BY + 2), IW = BX + 1, IN = (BX + 1) * (BY + 1);
  const int i = i0 + tid % BX, j = j0 + tid / BX;
  const bool act = tid < BX * BY && i <= d.sNx + 1 && j <= d.sNy + 1;
  VILevel a{d, p, f, k, t, i0, j0, EW, IW, sU, sV, sW, sHW, sHS, sHC, sKE, sVort, sHfz, sH0fz, sHDiv};
  for (int ee = tid; ee < EN; ee += VT_NT) {
    const int ii = i0 - 1 + ee % EW, jj = j0 - 1 + ee / EW;
    const bool in = ii <= d.sNx + d.OLx && jj <= d.sNy + d.OLy;
    const long q = MG_I3(d, in ? ii : 1, in ? jj : 1, k, t);
    sU[ee] = in ? AR3(uVel, q) : 0.0; sV[ee] = in ? AR3(vVel, q) : 0.0; sW[ee] = in ? AR3(wVel, q) : 0.0;
    sHW[ee] = in ? AR3(hFacW, q) : 0.0; sHS[ee] = in ? AR3(hFacS, q) : 0.0; sHC[ee] = in ? AR3(hFacC, q) : 0.0;
  }
  __syncthreads();
  for (int q = tid; q < IN; q += VT_NT) {
    const int ii = i0 + q % IW, jj = j0 + q / IW;
    const bool ok = ii <= d.sNx + d.OLx && jj <= d.sNy + d.OLy;
    sHfz[q] = ok ? vi_hfacz(a, d, ii, jj, k) : 0.0;
    sH0fz[q] = ok ? vi_h0facz(a, d, p, ii, jj, k) : 0.0;
    sVort[q] = ok ? vi_vort(a, d, p, f, ii, jj, k, t) : 0.0;
    sKE[q] = vi_KE(a, d, p, f, ii - 1, jj - 1, k, t);
    sHDiv[q] = vi_hdiv(a, d, p, f, ii - 1, jj - 1, k, t);
  }
  __syncthreads();
  if (!act) return;
  const int myIter = *iterPtr;
  const double abFac = (myIter == p.nIter0 && p.nIter0 == 0) ? 0.0 : 0.5 + p.abEps;   // adams_bashforth2.F:61-65
  const double mass2rUnit = 1.0 / p.rhoConst;
  const bool rstar = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
  const long q2 = MG_I2(d, i, j, t), q3 = MG_I3(d, i, j, k, t);
  const double recip_drF = f.recip_drF[k - 1];
  double gU = 0.0, gV = 0.0, guDiss = 0.0, gvDiss = 0.0, dPhiHydX = 0.0, dPhiHydY = 0.0;
  {  // CALC_GRAD_PHI_HYD (calc_grad_phi_hyd.F:152-214), as k_mom_step
    const bool rsc = rstar && p.select_rStar >= 2 && p.nonlinFreeSurf >= 4;
    auto varLoc = [&](int ii, int jj) {
      return rsc ? AR3(phiHydC, MG_I3(d, ii, jj, k, t)) * AR2(rStarFacC, MG_I2(d, ii, jj, t)) + 0.0
                 : AR3(phiHydC, MG_I3(d, ii, jj, k, t)) + 0.0;
    };
    const double vl = varLoc(i, j);
    if (i >= 1) dPhiHydX = AR2(recip_dxC, q2) * (vl - varLoc(i - 1, j));
    if (j >= 1) dPhiHydY = AR2(recip_dyC, q2) * (vl - varLoc(i, j - 1));
    if (rstar && p.select_rStar >= 2) {
      const double factorP = p.gravity * (1.0 / p.rhoConst) * 0.5, rCk = f.rC[k - 1];
      auto vl2 = [&](int ii, int jj) { return AR2(etaH, MG_I2(d, ii, jj, t)) * (1.0 + rCk * AR2(recip_Rcol, MG_I2(d, ii, jj, t))); };
      const double e0 = vl2(i, j), a0 = AR3(alphaRho, q3);
      if (i >= 1)
        dPhiHydX = dPhiHydX + factorP * (AR3(alphaRho, MG_I3(d, i - 1, j, k, t)) + a0) * (e0 - vl2(i - 1, j)) * AR2(recip_dxC, q2);
      if (j >= 1)
        dPhiHydY = dPhiHydY + factorP * (AR3(alphaRho, MG_I3(d, i, j - 1, k, t)) + a0) * (e0 - vl2(i, j - 1)) * AR2(recip_dyC, q2);
    }
  }
  vecinv_tend(a, d, p, f, i, j, k, t, gU, gV, guDiss, gvDiss);
  double guExt = 0.0, gvExt = 0.0;
  if (p.momForcing && k == 1) {
    if (j >= 0 && j <= d.sNy + 1 && i >= 1 && i <= d.sNx + 1)
      guExt = guExt + p.foFacMom * (AR2(fu, q2) * mass2rUnit) * recip_drF * a.recip_hFacW(i, j, k);
    if (j >= 1 && j <= d.sNy + 1 && i >= 0 && i <= d.sNx + 1)
      gvExt = gvExt + p.foFacMom * (AR2(fv, q2) * mass2rUnit) * recip_drF * a.recip_hFacS(i, j, k);
  }
  gU = gU - p.pfFacMom * dPhiHydX;
  gV = gV - p.pfFacMom * dPhiHydY;
  if (p.momViscosity && p.momDissip_In_AB) { gU = gU + guDiss; gV = gV + gvDiss; }
  if (p.momForcing && p.momForcingOutAB != 1) { gU = gU + guExt; gV = gV + gvExt; }
  {
    const double gUo = AR3(guNm1, q3), gVo = AR3(gvNm1, q3);
    double ab = abFac * (gU - gUo);
    AR3(guNm1, q3) = gU;
    gU = gU + ab;
    ab = abFac * (gV - gVo);
    AR3(gvNm1, q3) = gV;
    gV = gV + ab;
  }
  double gUtmp = gU, gVtmp = gV;
  if (p.momForcing && p.momForcingOutAB == 1) { gUtmp = gUtmp + guExt; gVtmp = gVtmp + gvExt; }
  if (p.momViscosity && !p.momDissip_In_AB) { gUtmp = gUtmp + guDiss; gVtmp = gVtmp + gvDiss; }
  if (rstar && p.nonlinFreeSurf > 1) {
    gUtmp = gUtmp / AR2(rStarExpW, q2);
    gVtmp = gVtmp / AR2(rStarExpS, q2);
  }
  AR3(gU, q3) = a.uVel(i, j, k) + p.deltaTMom * (gUtmp + 0.0) * a.maskW(i, j, k);
  AR3(gV, q3) = a.vVel(i, j, k) + p.deltaTMom * (gVtmp + 0.0) * a.maskS(i, j, k);
}

// ---------------------------------------------------------------------------------------
// MOM_VECINV + CALC_GRAD_PHI_HYD + TIMESTEP + ADAMS_BASHFORTH2 as a register-pipelined
// k-march (default for VI): a workgroup owns a BX x BY block of the DYNAMICS range of one
// tile and marches KC levels.  What stays constant down the column is fetched once: the
// 2-D metrics the ring-point intermediates and the Coriolis averages reach (dxC, dyC,
// recAz, dxG, dyG, recip_rA) are staged in LDS over the block extent, the output point's
// own metrics (reciprocal spacings, areas, side-drag lengths, f at the three corners, rA
// of the three w points) live in registers.  Per level only the level itself is staged:
// u, v, hFacW, hFacS over the extent, hFacC in a 2-slot ring (maskC at k-1) and w in a
// 2-slot ring (w at k+1); the vertical neighbours the output point needs (u, v, hFacW,
// hFacS at k-1 and k+1) are its own column's values, carried in registers.  Level k+1
// (and w at k+2) is fetched into registers while level k is computed, every load
// unconditional with clamped indices, so a level's loads issue together.  The expression
// trees are vecinv_tend's (accessor VIMarch), so the result is bit-identical to the
// per-point and per-level kernels.
struct VIMarchRegs {   // the output point's own 2-D values (i,j); n = (i,j+1), e = (i+1,j), w = (i-1,j), s = (i,j-1)
  double recip_dxC, recip_dyC, recip_dxG, recip_dyG, rAw, rAs, recip_rAw, recip_rAs;
  double dxV, dxVn, recip_dyU, recip_dyUn, dyU, dyUe, recip_dxV, recip_dxVe;
  double fCoriG, fCoriGn, fCoriGe, rA, rAw_w, rA_s;
};
constexpr int VM_S2 = 6;   // LDS-staged 2-D fields: dxC, dyC, recip_rAz, dxG, dyG, recip_rA
struct VIMarch {
  const Dims &d; const Params &p; const Fields &f; int k, t, i0, j0, EW, IW, i, j;
  const double *sU, *sV, *sHW, *sHS, *sHC, *sW, *s2;
  const double *sKE, *sVort, *sHfz, *sH0fz, *sHDiv;
  const VIMarchRegs &c;
  double uM, uP, vM, vP, hwM, hwP, hsM, hsP;   // own column at k-1 and k+1
  __device__ __forceinline__ int e(int ii, int jj) const { return (jj - j0 + 1) * EW + (ii - i0 + 1); }
  __device__ __forceinline__ long g(int ii, int jj, int kk) const { return MG_I3(d, ii, jj, kk, t); }
  __device__ __forceinline__ bool own(int ii, int jj) const { return ii == i && jj == j; }
  // u, v, hFacW, hFacS: level k anywhere on the extent (LDS), other levels at the own point
  // only (k-1 / k+1 registers) -- the only places MOM_VECINV reaches them; hFacC at k-1, k
  // and w at k, k+1 from the 2-slot rings.  Selects, not branches: no fallback loads.
  __device__ __forceinline__ double lvl(const double *sl, double m_, double p_, int ii, int jj, int kk) const {
    if (!own(ii, jj)) return sl[e(ii, jj)];
    return kk == k ? sl[e(ii, jj)] : (kk < k ? m_ : p_);
  }
  __device__ __forceinline__ double uVel(int ii, int jj, int kk) const { return lvl(sU, uM, uP, ii, jj, kk); }
  __device__ __forceinline__ double vVel(int ii, int jj, int kk) const { return lvl(sV, vM, vP, ii, jj, kk); }
  __device__ __forceinline__ double hFacW(int ii, int jj, int kk) const { return lvl(sHW, hwM, hwP, ii, jj, kk); }
  __device__ __forceinline__ double hFacS(int ii, int jj, int kk) const { return lvl(sHS, hsM, hsP, ii, jj, kk); }
  __device__ __forceinline__ double hFacC(int ii, int jj, int kk) const { return sHC[(kk & 1) * VT_EMAX + e(ii, jj)]; }
  __device__ __forceinline__ double wVel(int ii, int jj, int kk) const { return sW[(kk & 1) * VT_EMAX + e(ii, jj)]; }
  __device__ __forceinline__ double maskW(int ii, int jj, int kk) const { return hFacW(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double maskS(int ii, int jj, int kk) const { return hFacS(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double maskC(int ii, int jj, int kk) const { return hFacC(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double recip_hFacW(int ii, int jj, int kk) const {
    const double h = hFacW(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double recip_hFacS(int ii, int jj, int kk) const {
    const double h = hFacS(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double recip_hFacC(int ii, int jj, int kk) const {
    const double h = hFacC(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double h0FacW(int ii, int jj, int kk) const { return AR3(h0FacW, g(ii, jj, kk)); }
  __device__ __forceinline__ double h0FacS(int ii, int jj, int kk) const { return AR3(h0FacS, g(ii, jj, kk)); }
  template <int F> __device__ __forceinline__ double g2(int ii, int jj) const {
    const int di = ii - i, dj = jj - j;
    if constexpr (F == F2_dxC) return s2[0 * VT_EMAX + e(ii, jj)];
    else if constexpr (F == F2_dyC) return s2[1 * VT_EMAX + e(ii, jj)];
    else if constexpr (F == F2_recip_rAz) return s2[2 * VT_EMAX + e(ii, jj)];
    else if constexpr (F == F2_dxG) return s2[3 * VT_EMAX + e(ii, jj)];
    else if constexpr (F == F2_dyG) return s2[4 * VT_EMAX + e(ii, jj)];
    else if constexpr (F == F2_recip_rA) return s2[5 * VT_EMAX + e(ii, jj)];
    else {
#define VM_R(name, DI, DJ, reg) if constexpr (F == F2_##name) { if (di == (DI) && dj == (DJ)) return c.reg; }
      VM_R(recip_dxC, 0, 0, recip_dxC) VM_R(recip_dyC, 0, 0, recip_dyC) VM_R(recip_dxG, 0, 0, recip_dxG)
      VM_R(recip_dyG, 0, 0, recip_dyG) VM_R(rAw, 0, 0, rAw) VM_R(rAs, 0, 0, rAs) VM_R(recip_rAw, 0, 0, recip_rAw)
      VM_R(recip_rAs, 0, 0, recip_rAs) VM_R(dxV, 0, 0, dxV) VM_R(dxV, 0, 1, dxVn) VM_R(recip_dyU, 0, 0, recip_dyU)
      VM_R(recip_dyU, 0, 1, recip_dyUn) VM_R(dyU, 0, 0, dyU) VM_R(dyU, 1, 0, dyUe) VM_R(recip_dxV, 0, 0, recip_dxV)
      VM_R(recip_dxV, 1, 0, recip_dxVe) VM_R(fCoriG, 0, 0, fCoriG) VM_R(fCoriG, 0, 1, fCoriGn)
      VM_R(fCoriG, 1, 0, fCoriGe) VM_R(rA, 0, 0, rA) VM_R(rA, -1, 0, rAw_w) VM_R(rA, 0, -1, rA_s)
#undef VM_R
      return f.a2[(long)F * d.N2all + MG_I2(d, ii, jj, t)];   // anything else: where it lies
    }
  }
  __device__ __forceinline__ int iv(int ii, int jj) const { return (jj - j0) * IW + (ii - i0); }
  __device__ __forceinline__ int id(int ii, int jj) const { return (jj - j0 + 1) * IW + (ii - i0 + 1); }
  __device__ __forceinline__ double hfz(int ii, int jj) const { return sHfz[iv(ii, jj)]; }
  __device__ __forceinline__ double h0fz(int ii, int jj) const { return sH0fz[iv(ii, jj)]; }
  __device__ __forceinline__ double vort(int ii, int jj) const { return sVort[iv(ii, jj)]; }
  __device__ __forceinline__ double KE(int ii, int jj) const { return sKE[id(ii, jj)]; }
  __device__ __forceinline__ double hDiv(int ii, int jj) const { return sHDiv[id(ii, jj)]; }
};

// PF: fetch level k+1 into registers during level k (else after it); CREG: the output
// point's metrics held in registers across the march (else re-read every level)
template <bool PF, bool CREG>
__global__ void __launch_bounds__(VT_NT) k_mom_vi_march(Dims d, Params p, Fields f, const int *iterPtr, int BX, int BY,
                                                         int nbx, int nby, int KC, int nkc) {
  __shared__ double sU[VT_EMAX], sV[VT_EMAX], sHW[VT_EMAX], sHS[VT_EMAX], sHC[2 * VT_EMAX], sW[2 * VT_EMAX];
  __shared__ double s2[VM_S2 * VT_EMAX];
  __shared__ double sKE[VT_IMAX], sVort[VT_IMAX], sHfz[VT_IMAX], sH0fz[VT_IMAX], sHDiv[VT_IMAX];
  // block id: (i,j) block fastest, then the chunk of KC levels, then the tile
  const int nb = nbx * nby, lb = mg_xcd_block();
  const int t = d.t0 + lb / (nb * nkc), bxy = lb % nb, kb = 1 + ((lb / nb) % nkc) * KC;
  const int Nr = d.Nr, ke = kb + KC - 1 < Nr ? kb + KC - 1 : Nr;
  const int i0 = (bxy % nbx) * BX, j0 = (bxy / nbx) * BY;
  const int tid = threadIdx.x;
  const int EW = BX + 2, EN = (BX + 2) * (BY + 2), IW = BX + 1, IN = (BX + 1) * (BY + 1);
  const int i = i0 + tid % BX, j = j0 + tid / BX;
  const bool act = tid < BX * BY && i <= d.sNx + 1 && j <= d.sNy + 1;
  const int ic = act ? i : 1, jc = act ? j : 1;   // in-range stand-in for idle threads' loads
  const long q2 = MG_I2(d, ic, jc, t);
  // the extent i0-1..i0+BX x j0-1..j0+BY, clipped to the array (points past it are read by
  // no active thread): element r of this thread, its flat 2-D offset and whether it exists
  long eq[2];
  bool ein[2];
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int ee = tid + r * VT_NT;
    const int ii = i0 - 1 + ee % EW, jj = j0 - 1 + ee / EW;
    ein[r] = ee < EN && ii <= d.sNx + d.OLx && jj <= d.sNy + d.OLy;
    eq[r] = MG_I2(d, ein[r] ? ii : 1, ein[r] ? jj : 1, t);
  }
  // 2-D staging (once per workgroup)
  {
    const int ids[VM_S2] = {F2_dxC, F2_dyC, F2_recip_rAz, F2_dxG, F2_dyG, F2_recip_rA};
#pragma unroll
    for (int n = 0; n < VM_S2; n++)
#pragma unroll
      for (int r = 0; r < 2; r++) {
        const int ee = tid + r * VT_NT;
        const double v = f.a2[(long)ids[n] * d.N2all + eq[r]];
        if (ee < EN) s2[n * VT_EMAX + ee] = ein[r] ? v : 0.0;
      }
  }
  auto load_c = [&](VIMarchRegs &c, const long q2) {
    const long qn = q2 + d.nx, qe = q2 + 1, qw = q2 - 1, qs = q2 - d.nx;
    c.recip_dxC = AR2(recip_dxC, q2); c.recip_dyC = AR2(recip_dyC, q2);
    c.recip_dxG = AR2(recip_dxG, q2); c.recip_dyG = AR2(recip_dyG, q2);
    c.rAw = AR2(rAw, q2); c.rAs = AR2(rAs, q2); c.recip_rAw = AR2(recip_rAw, q2); c.recip_rAs = AR2(recip_rAs, q2);
    c.dxV = AR2(dxV, q2); c.dxVn = AR2(dxV, qn); c.recip_dyU = AR2(recip_dyU, q2); c.recip_dyUn = AR2(recip_dyU, qn);
    c.dyU = AR2(dyU, q2); c.dyUe = AR2(dyU, qe); c.recip_dxV = AR2(recip_dxV, q2); c.recip_dxVe = AR2(recip_dxV, qe);
    c.fCoriG = AR2(fCoriG, q2); c.fCoriGn = AR2(fCoriG, qn); c.fCoriGe = AR2(fCoriG, qe);
    c.rA = AR2(rA, q2); c.rAw_w = AR2(rA, qw); c.rA_s = AR2(rA, qs);
  };
  VIMarchRegs c0;   // CREG: loaded once, live in registers across the march
  if constexpr (CREG) load_c(c0, q2);
  // level fetches into registers (unconditional loads, masked where the element is absent),
  // addressed as uniform field base + 32-bit byte offset (the global_load saddr form)
  const long t3 = (long)t * (d.n3 - d.n2);   // MG_I3 = MG_I2 + (k-1)*n2 + t*(n3-n2)
  const unsigned lvB = (unsigned)(d.n2 * 8);
  unsigned eb[2];
#pragma unroll
  for (int r = 0; r < 2; r++) eb[r] = (unsigned)((eq[r] + t3) * 8);
  const unsigned ob = (unsigned)((q2 + t3) * 8);
  const char *bU = (const char *)(f.a3 + (long)F3_uVel * d.N3all), *bV = (const char *)(f.a3 + (long)F3_vVel * d.N3all);
  const char *bHW = (const char *)(f.a3 + (long)F3_hFacW * d.N3all), *bHS = (const char *)(f.a3 + (long)F3_hFacS * d.N3all);
  const char *bHC = (const char *)(f.a3 + (long)F3_hFacC * d.N3all), *bW = (const char *)(f.a3 + (long)F3_wVel * d.N3all);
  auto ld = [](const char *b, unsigned off) { return *(const double *)(b + off); };
  double nU[2], nV[2], nHW[2], nHS[2], nHC[2], nW[2], oU, oV, oHW, oHS;
  auto fetch = [&](int kk) {   // level kk over the extent + the own column's u, v, hFacW, hFacS
    const unsigned lo = (unsigned)(kk - 1) * lvB;
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const unsigned o = eb[r] + lo;
      nU[r] = ld(bU, o); nV[r] = ld(bV, o); nHW[r] = ld(bHW, o); nHS[r] = ld(bHS, o); nHC[r] = ld(bHC, o);
    }
    const unsigned o = ob + lo;
    oU = ld(bU, o); oV = ld(bV, o); oHW = ld(bHW, o); oHS = ld(bHS, o);
  };
  auto fetchW = [&](int kk) {
    const unsigned lo = (unsigned)(kk - 1) * lvB;
#pragma unroll
    for (int r = 0; r < 2; r++) nW[r] = ld(bW, eb[r] + lo);
  };
  auto stash = [&](int kk) {
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int ee = tid + r * VT_NT;
      if (ee < EN) {
        sU[ee] = ein[r] ? nU[r] : 0.0; sV[ee] = ein[r] ? nV[r] : 0.0;
        sHW[ee] = ein[r] ? nHW[r] : 0.0; sHS[ee] = ein[r] ? nHS[r] : 0.0;
        sHC[(kk & 1) * VT_EMAX + ee] = ein[r] ? nHC[r] : 0.0;
      }
    }
  };
  auto stashW = [&](int kk) {
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int ee = tid + r * VT_NT;
      if (ee < EN) sW[(kk & 1) * VT_EMAX + ee] = (ein[r] && kk <= Nr) ? nW[r] : 0.0;
    }
  };
  // prologue: own column at kb-1; hFacC at kb-1; level kb; w at kb and kb+1
  double uM = 0.0, vM = 0.0, hwM = 0.0, hsM = 0.0;
  if (kb > 1) {
    fetch(kb - 1);
    uM = oU; vM = oV; hwM = oHW; hsM = oHS;
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int ee = tid + r * VT_NT;
      if (ee < EN) sHC[((kb - 1) & 1) * VT_EMAX + ee] = ein[r] ? nHC[r] : 0.0;
    }
  }
  fetchW(kb);
  stashW(kb);
  fetchW(kb + 1 <= Nr ? kb + 1 : Nr);
  stashW(kb + 1);
  fetch(kb);
  stash(kb);
  const int myIter = *iterPtr;
  const double abFac = (myIter == p.nIter0 && p.nIter0 == 0) ? 0.0 : 0.5 + p.abEps;   // adams_bashforth2.F:61-65
  const double mass2rUnit = 1.0 / p.rhoConst;
  const bool rstar = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
  __syncthreads();
  for (int k = kb; k <= ke; k++) {
    // the thread's coordinates re-materialised each level (an empty asm the compiler cannot
    // see through): the addresses derived from them are recomputed per level instead of
    // hoisted out of the march and held in registers across it
    int iL = i, jL = j;
    long q2L = q2;
    asm volatile("" : "+v"(iL), "+v"(jL), "+v"(q2L));
    [&](const int i, const int j, const long q2) {
    VIMarchRegs c1;   // !CREG: re-read every level (cache hits) instead of held across the march
    if constexpr (!CREG) load_c(c1, q2);
    const VIMarchRegs &c = CREG ? c0 : c1;
    const int kn = k + 1 <= Nr ? k + 1 : Nr, kw = k + 2 <= Nr ? k + 2 : Nr;
    if constexpr (PF) {
      fetch(kn);    // level k+1 and the own column at k+1, in flight during level k
      fetchW(kw);
    } else {   // own column at k+1 only; the level itself is fetched after the output
      const unsigned o = ob + (unsigned)(kn - 1) * lvB;
      oU = ld(bU, o); oV = ld(bV, o); oHW = ld(bHW, o); oHS = ld(bHS, o);
    }
    // the output point's accessor, and one for the ring-point intermediates whose own point
    // matches nothing (they read level k only; an idle thread's registers hold (1,1)'s values)
    VIMarch a{d, p, f, k, t, i0, j0, EW, IW, i, j, sU, sV, sHW, sHS, sHC, sW, s2, sKE, sVort, sHfz, sH0fz, sHDiv, c,
              uM, k < Nr ? oU : 0.0, vM, k < Nr ? oV : 0.0, hwM, k < Nr ? oHW : 0.0, hsM, k < Nr ? oHS : 0.0};
    VIMarch ai{d, p, f, k, t, i0, j0, EW, IW, -1000000, -1000000, sU, sV, sHW, sHS, sHC, sW, s2, sKE, sVort, sHfz, sH0fz,
               sHDiv, c, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int q = tid; q < IN; q += VT_NT) {
      const int ii = i0 + q % IW, jj = j0 + q / IW;          // vort / hFacZ grid: i0..i0+BX
      const bool ok = ii <= d.sNx + d.OLx && jj <= d.sNy + d.OLy;
      sHfz[q] = ok ? vi_hfacz(ai, d, ii, jj, k) : 0.0;
      sH0fz[q] = ok ? vi_h0facz(ai, d, p, ii, jj, k) : 0.0;
      sVort[q] = ok ? vi_vort(ai, d, p, f, ii, jj, k, t) : 0.0;
      sKE[q] = vi_KE(ai, d, p, f, ii - 1, jj - 1, k, t);     // KE / hDiv grid: i0-1..i0+BX-1
      sHDiv[q] = vi_hdiv(ai, d, p, f, ii - 1, jj - 1, k, t);
    }
    __syncthreads();
    if (act) {
      auto q3of = [&](long qq2, int kk) { return qq2 + (long)(kk - 1) * d.n2 + t3; };
      const long q3 = q3of(q2, k);
      const double recip_drF = f.recip_drF[k - 1];
      double gU = 0.0, gV = 0.0, guDiss = 0.0, gvDiss = 0.0, dPhiHydX = 0.0, dPhiHydY = 0.0;
      {  // CALC_GRAD_PHI_HYD (calc_grad_phi_hyd.F:152-214), as k_mom_step
        const bool rsc = rstar && p.select_rStar >= 2 && p.nonlinFreeSurf >= 4;
        auto varLoc = [&](long qq2) {
          return rsc ? AR3(phiHydC, q3of(qq2, k)) * AR2(rStarFacC, qq2) + 0.0 : AR3(phiHydC, q3of(qq2, k)) + 0.0;
        };
        const double vl = varLoc(q2);
        if (i >= 1) dPhiHydX = c.recip_dxC * (vl - varLoc(q2 - 1));
        if (j >= 1) dPhiHydY = c.recip_dyC * (vl - varLoc(q2 - d.nx));
        if (rstar && p.select_rStar >= 2) {
          const double factorP = p.gravity * (1.0 / p.rhoConst) * 0.5, rCk = f.rC[k - 1];
          auto vl2 = [&](long qq2) { return AR2(etaH, qq2) * (1.0 + rCk * AR2(recip_Rcol, qq2)); };
          const double e0 = vl2(q2), a0 = AR3(alphaRho, q3);
          if (i >= 1) dPhiHydX = dPhiHydX + factorP * (AR3(alphaRho, q3 - 1) + a0) * (e0 - vl2(q2 - 1)) * c.recip_dxC;
          if (j >= 1) dPhiHydY = dPhiHydY + factorP * (AR3(alphaRho, q3 - d.nx) + a0) * (e0 - vl2(q2 - d.nx)) * c.recip_dyC;
        }
      }
      vecinv_tend(a, d, p, f, i, j, k, t, gU, gV, guDiss, gvDiss);
      double guExt = 0.0, gvExt = 0.0;
      if (p.momForcing && k == 1) {
        if (j >= 0 && j <= d.sNy + 1 && i >= 1 && i <= d.sNx + 1)
          guExt = guExt + p.foFacMom * (AR2(fu, q2) * mass2rUnit) * recip_drF * a.recip_hFacW(i, j, k);
        if (j >= 1 && j <= d.sNy + 1 && i >= 0 && i <= d.sNx + 1)
          gvExt = gvExt + p.foFacMom * (AR2(fv, q2) * mass2rUnit) * recip_drF * a.recip_hFacS(i, j, k);
      }
      gU = gU - p.pfFacMom * dPhiHydX;
      gV = gV - p.pfFacMom * dPhiHydY;
      if (p.momViscosity && p.momDissip_In_AB) { gU = gU + guDiss; gV = gV + gvDiss; }
      if (p.momForcing && p.momForcingOutAB != 1) { gU = gU + guExt; gV = gV + gvExt; }
      {  // ADAMS_BASHFORTH2 (adams_bashforth2.F:81-88)
        const double gUo = AR3(guNm1, q3), gVo = AR3(gvNm1, q3);
        double ab = abFac * (gU - gUo);
        AR3(guNm1, q3) = gU;
        gU = gU + ab;
        ab = abFac * (gV - gVo);
        AR3(gvNm1, q3) = gV;
        gV = gV + ab;
      }
      double gUtmp = gU, gVtmp = gV;
      if (p.momForcing && p.momForcingOutAB == 1) { gUtmp = gUtmp + guExt; gVtmp = gVtmp + gvExt; }
      if (p.momViscosity && !p.momDissip_In_AB) { gUtmp = gUtmp + guDiss; gVtmp = gVtmp + gvDiss; }
      if (rstar && p.nonlinFreeSurf > 1) {
        gUtmp = gUtmp / AR2(rStarExpW, q2);
        gVtmp = gVtmp / AR2(rStarExpS, q2);
      }
      AR3(gU, q3) = a.uVel(i, j, k) + p.deltaTMom * (gUtmp + 0.0) * a.maskW(i, j, k);
      AR3(gV, q3) = a.vVel(i, j, k) + p.deltaTMom * (gVtmp + 0.0) * a.maskS(i, j, k);
    }
    }(iL, jL, q2L);
    if (k == ke) break;
    // the own column moves down: level k becomes k-1 (read before level k+1 overwrites it)
    if (act) { const int eo = (j - j0 + 1) * EW + (i - i0 + 1); uM = sU[eo]; vM = sV[eo]; hwM = sHW[eo]; hsM = sHS[eo]; }
    if constexpr (!PF) {
      fetch(k + 1 <= Nr ? k + 1 : Nr);
      fetchW(k + 2 <= Nr ? k + 2 : Nr);
    }
    __syncthreads();
    stash(k + 1);
    stashW(k + 2);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// The k-march specialised at compile time (k_mom_vi_m2): the block shape BX x BY and
// MOM_VECINV's option switches (VIP<C>, C = vi_opt_code of the run's Params) are template
// constants, so the LDS neighbour offsets fold into ds_read immediates, untaken scheme
// branches vanish and the run-time parameters left are the dozen coefficients VIP carries
// (the generic k_mom_vi_march keeps the whole Params live in scalar registers and spills
// them to VGPR lanes inside the march: ~300 v_readlane per level body).  vecinv_tend and the
// vi_* intermediates are the same templates reading p.x, so the expression trees -- and the
// bits -- are those of every other MOM_VECINV kernel.  Used when the run's option code and
// block shape have an instantiation (vi_m2_kernel), else the generic march.
template <unsigned C>
struct VIP {
  static constexpr int selectVortScheme = C & 3, selectCoriScheme = (C >> 2) & 3, selectKEscheme = (C >> 4) & 3;
  static constexpr int momViscosity = (C >> 6) & 1, no_slip_sides = (C >> 7) & 1, no_slip_bottom = (C >> 8) & 1;
  static constexpr int implicitViscosity = (C >> 9) & 1, useCoriolis = (C >> 10) & 1, momAdvection = (C >> 11) & 1;
  static constexpr int upwindShear = (C >> 12) & 1, cubeCorners = (C >> 13) & 1, momForcing = (C >> 14) & 1;
  static constexpr int momDissip_In_AB = (C >> 15) & 1, momForcingOutAB = (C >> 16) & 1;
  static constexpr int nonlinFreeSurf = (C >> 17) & 7, select_rStar = (C >> 20) & 3;
  double rkSign, sideDragFactor, vfFacMom, viscA4Z, viscAhD, viscAhZ, viscAr;
  double abEps, deltaTMom, foFacMom, gravity, pfFacMom, rhoConst;
  int nIter0;
};
// the option code of a run: every switch the VI kernels branch on, clamped to the values
// those branches distinguish (nonlinFreeSurf: > 0, > 1, >= 4; select_rStar: > 0, >= 2;
// momForcingOutAB: == 1)
static unsigned vi_opt_code(const Params &p) {
  auto cl = [](int v, int hi) { return (unsigned)(v < 0 ? 0 : v > hi ? hi : v); };
  auto b = [](int v) { return v != 0 ? 1u : 0u; };
  return cl(p.selectVortScheme, 3) | cl(p.selectCoriScheme, 3) << 2 | cl(p.selectKEscheme, 3) << 4 |
         b(p.momViscosity) << 6 | b(p.no_slip_sides) << 7 | b(p.no_slip_bottom) << 8 | b(p.implicitViscosity) << 9 |
         b(p.useCoriolis) << 10 | b(p.momAdvection) << 11 | b(p.upwindShear) << 12 | b(p.cubeCorners) << 13 |
         b(p.momForcing) << 14 | b(p.momDissip_In_AB) << 15 | (p.momForcingOutAB == 1 ? 1u : 0u) << 16 |
         cl(p.nonlinFreeSurf, 7) << 17 | cl(p.select_rStar, 3) << 20;
}
template <unsigned C>
static VIP<C> vi_params(const Params &p) {
  VIP<C> v;
  v.rkSign = p.rkSign; v.sideDragFactor = p.sideDragFactor; v.vfFacMom = p.vfFacMom; v.viscA4Z = p.viscA4Z;
  v.viscAhD = p.viscAhD; v.viscAhZ = p.viscAhZ; v.viscAr = p.viscAr; v.abEps = p.abEps; v.deltaTMom = p.deltaTMom;
  v.foFacMom = p.foFacMom; v.gravity = p.gravity; v.pfFacMom = p.pfFacMom; v.rhoConst = p.rhoConst;
  v.nIter0 = p.nIter0;
  return v;
}

// Accessor of k_mom_vi_m2.  OWN: the output point (i,j), whose column's k-1 / k+1 values of
// u, v, hFacW, hFacS sit in registers and whose own 2-D metrics in VIMarchRegs; !OWN: the
// ring-point intermediates, which read level k only (no own-point selects at all).
template <int BX, int BY, class P, bool OWN, int HR = 2>
struct VIM2 {   // HR: slots of the hFacC / wVel level rings (level kk in slot kk % HR)
  static constexpr int EW = BX + 2, IW = BX + 1;
  const Dims &d; const P &p; const Fields &f; int k, t, i0, j0, i, j;
  const double *sU, *sV, *sHW, *sHS, *sHC, *sW, *s2;
  const double *sKE, *sVort, *sHfz, *sH0fz, *sHDiv;
  const VIMarchRegs &c;
  double uM, uP, vM, vP, hwM, hwP, hsM, hsP;
  // filled at the level's start (vi_tile_face ... overloads below): the tile's face / edge
  // bits, recip_drC(k), recip_drC(k+1), recip_drF(k), drF(k), the own point's h0FacW / h0FacS
  int face = 0, edge = 0;
  double rdrCk = 0.0, rdrCk1 = 0.0, rdrFk = 0.0, drFk = 0.0, h0W = 0.0, h0S = 0.0;
  __device__ __forceinline__ int e(int ii, int jj) const { return (jj - j0 + 1) * EW + (ii - i0 + 1); }
  __device__ __forceinline__ long g(int ii, int jj, int kk) const { return MG_I3(d, ii, jj, kk, t); }
  __device__ __forceinline__ double lvl(const double *sl, double m_, double p_, int ii, int jj, int kk) const {
    if constexpr (OWN) {
      if (ii == i && jj == j && kk != k) return kk < k ? m_ : p_;
    }
    return sl[e(ii, jj)];
  }
  __device__ __forceinline__ double uVel(int ii, int jj, int kk) const { return lvl(sU, uM, uP, ii, jj, kk); }
  __device__ __forceinline__ double vVel(int ii, int jj, int kk) const { return lvl(sV, vM, vP, ii, jj, kk); }
  __device__ __forceinline__ double hFacW(int ii, int jj, int kk) const { return lvl(sHW, hwM, hwP, ii, jj, kk); }
  __device__ __forceinline__ double hFacS(int ii, int jj, int kk) const { return lvl(sHS, hsM, hsP, ii, jj, kk); }
  __device__ __forceinline__ double hFacC(int ii, int jj, int kk) const { return sHC[(kk % HR) * (EW * (BY + 2)) + e(ii, jj)]; }
  __device__ __forceinline__ double wVel(int ii, int jj, int kk) const { return sW[(kk % HR) * (EW * (BY + 2)) + e(ii, jj)]; }
  __device__ __forceinline__ double maskW(int ii, int jj, int kk) const { return hFacW(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double maskS(int ii, int jj, int kk) const { return hFacS(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double maskC(int ii, int jj, int kk) const { return hFacC(ii, jj, kk) != 0.0 ? 1.0 : 0.0; }
  __device__ __forceinline__ double recip_hFacW(int ii, int jj, int kk) const {
    const double h = hFacW(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double recip_hFacS(int ii, int jj, int kk) const {
    const double h = hFacS(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double recip_hFacC(int ii, int jj, int kk) const {
    const double h = hFacC(ii, jj, kk); return h != 0.0 ? 1.0 / h : 0.0; }
  __device__ __forceinline__ double h0FacW(int ii, int jj, int kk) const { return AR3(h0FacW, g(ii, jj, kk)); }
  __device__ __forceinline__ double h0FacS(int ii, int jj, int kk) const { return AR3(h0FacS, g(ii, jj, kk)); }
  template <int F> __device__ __forceinline__ double g2(int ii, int jj) const {
    constexpr int EN = EW * (BY + 2);
    if constexpr (F == F2_dxC) return s2[0 * EN + e(ii, jj)];
    else if constexpr (F == F2_dyC) return s2[1 * EN + e(ii, jj)];
    else if constexpr (F == F2_recip_rAz) return s2[2 * EN + e(ii, jj)];
    else if constexpr (F == F2_dxG) return s2[3 * EN + e(ii, jj)];
    else if constexpr (F == F2_dyG) return s2[4 * EN + e(ii, jj)];
    else if constexpr (F == F2_recip_rA) return s2[5 * EN + e(ii, jj)];
    else {
      if constexpr (OWN) {
        const int di = ii - i, dj = jj - j;
#define VM_R(name, DI, DJ, reg) if constexpr (F == F2_##name) { if (di == (DI) && dj == (DJ)) return c.reg; }
        VM_R(recip_dxC, 0, 0, recip_dxC) VM_R(recip_dyC, 0, 0, recip_dyC) VM_R(recip_dxG, 0, 0, recip_dxG)
        VM_R(recip_dyG, 0, 0, recip_dyG) VM_R(rAw, 0, 0, rAw) VM_R(rAs, 0, 0, rAs) VM_R(recip_rAw, 0, 0, recip_rAw)
        VM_R(recip_rAs, 0, 0, recip_rAs) VM_R(dxV, 0, 0, dxV) VM_R(dxV, 0, 1, dxVn) VM_R(recip_dyU, 0, 0, recip_dyU)
        VM_R(recip_dyU, 0, 1, recip_dyUn) VM_R(dyU, 0, 0, dyU) VM_R(dyU, 1, 0, dyUe) VM_R(recip_dxV, 0, 0, recip_dxV)
        VM_R(recip_dxV, 1, 0, recip_dxVe) VM_R(fCoriG, 0, 0, fCoriG) VM_R(fCoriG, 0, 1, fCoriGn)
        VM_R(fCoriG, 1, 0, fCoriGe) VM_R(rA, 0, 0, rA) VM_R(rA, -1, 0, rAw_w) VM_R(rA, 0, -1, rA_s)
#undef VM_R
      }
      return f.a2[(long)F * d.N2all + MG_I2(d, ii, jj, t)];   // anything else: where it lies
    }
  }
  __device__ __forceinline__ int iv(int ii, int jj) const { return (jj - j0) * IW + (ii - i0); }
  __device__ __forceinline__ int id(int ii, int jj) const { return (jj - j0 + 1) * IW + (ii - i0 + 1); }
  __device__ __forceinline__ double hfz(int ii, int jj) const { return sHfz[iv(ii, jj)]; }
  __device__ __forceinline__ double h0fz(int ii, int jj) const { return sH0fz[iv(ii, jj)]; }
  __device__ __forceinline__ double vort(int ii, int jj) const { return sVort[iv(ii, jj)]; }
  __device__ __forceinline__ double KE(int ii, int jj) const { return sKE[id(ii, jj)]; }
  __device__ __forceinline__ double hDiv(int ii, int jj) const { return sHDiv[id(ii, jj)]; }
};
template <int BX, int BY, class P, bool OWN, int HR>
__device__ __forceinline__ int vi_tile_face(const VIM2<BX, BY, P, OWN, HR> &a, const Fields &, int) { return a.face; }
template <int BX, int BY, class P, bool OWN, int HR>
__device__ __forceinline__ int vi_tile_edge(const VIM2<BX, BY, P, OWN, HR> &a, const Fields &, int) { return a.edge; }
template <int BX, int BY, class P, bool OWN, int HR>   // (called at kk = k and k + 1 only)
__device__ __forceinline__ double vi_rdrC(const VIM2<BX, BY, P, OWN, HR> &a, const Fields &, int kk) {
  return kk == a.k ? a.rdrCk : a.rdrCk1;
}
template <int BX, int BY, class P, bool OWN, int HR>
__device__ __forceinline__ double vi_rdrF(const VIM2<BX, BY, P, OWN, HR> &a, const Fields &, int) { return a.rdrFk; }
template <int BX, int BY, class P, bool OWN, int HR>
__device__ __forceinline__ double vi_drF(const VIM2<BX, BY, P, OWN, HR> &a, const Fields &, int) { return a.drFk; }
template <int BX, int BY, class P, bool OWN, int HR>
__device__ __forceinline__ double vi_h0W_own(const VIM2<BX, BY, P, OWN, HR> &a, int, int, int) { return a.h0W; }
template <int BX, int BY, class P, bool OWN, int HR>
__device__ __forceinline__ double vi_h0S_own(const VIM2<BX, BY, P, OWN, HR> &a, int, int, int) { return a.h0S; }

// The k-march of k_mom_vi_march<PF, CREG> (same phases, same staging), on VIM2 / VIP<C>.
// EARLY: the output point's own HBM reads of level k (phi_hyd at the three points of the
// pressure gradient, guNm1, gvNm1) issued at the start of the level, in flight during the
// ring-point intermediates, instead of after their barrier.  LBW: minimum waves per SIMD
// the register allocation must allow (__launch_bounds__).
#ifdef MGCM_VI_STAMPS   // diagnostic build only: per-phase shader-cycle totals of sampled workgroups
#define VI_STAMP(n)                                                          \
  do {                                                                       \
    __builtin_amdgcn_sched_barrier(0);                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();              \
    __builtin_amdgcn_sched_barrier(0);                                       \
    if ((n) > 0) viAcc[(n) - 1] += t_ - viPrev;                              \
    viPrev = t_;                                                             \
  } while (0)
#else
#define VI_STAMP(n) \
  do {              \
  } while (0)
#endif
template <int BX, int BY, unsigned C, bool PF, bool CREG, bool EARLY, int LBW>
__global__ void __launch_bounds__(VT_NT, LBW) k_mom_vi_m2(Dims d, VIP<C> p, Fields f, const int *iterPtr, int nbx, int nby,
                                                      int KC, int nkc) {
  using P = VIP<C>;
  constexpr int EW = BX + 2, EN = (BX + 2) * (BY + 2), IW = BX + 1, IN = (BX + 1) * (BY + 1);
  constexpr int NR = (EN + VT_NT - 1) / VT_NT;   // extent elements per thread
  static_assert(BX * BY <= VT_NT && EN <= 2 * VT_NT, "block shape");
  __shared__ double sU[EN], sV[EN], sHW[EN], sHS[EN], sHC[2 * EN], sW[2 * EN];
  __shared__ double s2[VM_S2 * EN];
  __shared__ double sKE[IN], sVort[IN], sHfz[IN], sH0fz[IN], sHDiv[IN];
  const int nb = nbx * nby, lb = mg_xcd_block();
  const int t = d.t0 + lb / (nb * nkc), bxy = lb % nb, kb = 1 + ((lb / nb) % nkc) * KC;
  const int Nr = d.Nr, ke = kb + KC - 1 < Nr ? kb + KC - 1 : Nr;
  const int i0 = (bxy % nbx) * BX, j0 = (bxy / nbx) * BY;
  const int tid = threadIdx.x;
  const int i = i0 + tid % BX, j = j0 + tid / BX;
  const bool act = tid < BX * BY && i <= d.sNx + 1 && j <= d.sNy + 1;
  const int ic = act ? i : 1, jc = act ? j : 1;
  const long q2 = MG_I2(d, ic, jc, t);
  long eq[NR];
  bool ein[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int ee = tid + r * VT_NT;
    const int ii = i0 - 1 + ee % EW, jj = j0 - 1 + ee / EW;
    ein[r] = ee < EN && ii <= d.sNx + d.OLx && jj <= d.sNy + d.OLy;
    eq[r] = MG_I2(d, ein[r] ? ii : 1, ein[r] ? jj : 1, t);
  }
  // the prologue's HBM reads are all issued before any of its LDS stores: a store behind the
  // `ee < EN` branch ends the basic block, and a load placed after it waited for every earlier
  // one (vmcnt(0)) -- about fifteen serial memory round trips per workgroup before the march
  double v2[VM_S2][NR];
  {
    const int ids[VM_S2] = {F2_dxC, F2_dyC, F2_recip_rAz, F2_dxG, F2_dyG, F2_recip_rA};
#pragma unroll
    for (int n = 0; n < VM_S2; n++)
#pragma unroll
      for (int r = 0; r < NR; r++) v2[n][r] = f.a2[(long)ids[n] * d.N2all + eq[r]];
  }
  auto load_c = [&](VIMarchRegs &c, const long q2) {
    const long qn = q2 + d.nx, qe = q2 + 1, qw = q2 - 1, qs = q2 - d.nx;
    c.recip_dxC = AR2(recip_dxC, q2); c.recip_dyC = AR2(recip_dyC, q2);
    c.recip_dxG = AR2(recip_dxG, q2); c.recip_dyG = AR2(recip_dyG, q2);
    c.rAw = AR2(rAw, q2); c.rAs = AR2(rAs, q2); c.recip_rAw = AR2(recip_rAw, q2); c.recip_rAs = AR2(recip_rAs, q2);
    c.dxV = AR2(dxV, q2); c.dxVn = AR2(dxV, qn); c.recip_dyU = AR2(recip_dyU, q2); c.recip_dyUn = AR2(recip_dyU, qn);
    c.dyU = AR2(dyU, q2); c.dyUe = AR2(dyU, qe); c.recip_dxV = AR2(recip_dxV, q2); c.recip_dxVe = AR2(recip_dxV, qe);
    c.fCoriG = AR2(fCoriG, q2); c.fCoriGn = AR2(fCoriG, qn); c.fCoriGe = AR2(fCoriG, qe);
    c.rA = AR2(rA, q2); c.rAw_w = AR2(rA, qw); c.rA_s = AR2(rA, qs);
  };
  VIMarchRegs c0;
  if constexpr (CREG) load_c(c0, q2);
  const int tFace = P::cubeCorners ? f.tileFace[t] : 0, tEdge = P::cubeCorners ? f.tileEdge[t] : 0;
  const long t3 = (long)t * (d.n3 - d.n2);
  const unsigned lvB = (unsigned)(d.n2 * 8);
  unsigned eb[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) eb[r] = (unsigned)((eq[r] + t3) * 8);
  const unsigned ob = (unsigned)((q2 + t3) * 8);
  const char *bU = (const char *)(f.a3 + (long)F3_uVel * d.N3all), *bV = (const char *)(f.a3 + (long)F3_vVel * d.N3all);
  const char *bHW = (const char *)(f.a3 + (long)F3_hFacW * d.N3all), *bHS = (const char *)(f.a3 + (long)F3_hFacS * d.N3all);
  const char *bHC = (const char *)(f.a3 + (long)F3_hFacC * d.N3all), *bW = (const char *)(f.a3 + (long)F3_wVel * d.N3all);
  auto ld = [](const char *b, unsigned off) { return *(const double *)(b + off); };
  double nU[NR], nV[NR], nHW[NR], nHS[NR], nHC[NR], nW[NR], oU, oV, oHW, oHS;
  auto fetch = [&](int kk) {
    const unsigned lo = (unsigned)(kk - 1) * lvB;
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const unsigned o = eb[r] + lo;
      nU[r] = ld(bU, o); nV[r] = ld(bV, o); nHW[r] = ld(bHW, o); nHS[r] = ld(bHS, o); nHC[r] = ld(bHC, o);
    }
    const unsigned o = ob + lo;
    oU = ld(bU, o); oV = ld(bV, o); oHW = ld(bHW, o); oHS = ld(bHS, o);
  };
  auto fetchW = [&](int kk) {
    const unsigned lo = (unsigned)(kk - 1) * lvB;
#pragma unroll
    for (int r = 0; r < NR; r++) nW[r] = ld(bW, eb[r] + lo);
  };
  auto stash = [&](int kk) {
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const int ee = tid + r * VT_NT;
      if (ee < EN) {
        sU[ee] = ein[r] ? nU[r] : 0.0; sV[ee] = ein[r] ? nV[r] : 0.0;
        sHW[ee] = ein[r] ? nHW[r] : 0.0; sHS[ee] = ein[r] ? nHS[r] : 0.0;
        sHC[(kk & 1) * EN + ee] = ein[r] ? nHC[r] : 0.0;
      }
    }
  };
  auto stashW = [&](int kk) {
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const int ee = tid + r * VT_NT;
      if (ee < EN) sW[(kk & 1) * EN + ee] = (ein[r] && kk <= Nr) ? nW[r] : 0.0;
    }
  };
  double uM = 0.0, vM = 0.0, hwM = 0.0, hsM = 0.0, hcM[NR];
  if (kb > 1) {
    fetch(kb - 1);
    uM = oU; vM = oV; hwM = oHW; hsM = oHS;
#pragma unroll
    for (int r = 0; r < NR; r++) hcM[r] = nHC[r];
  }
  fetchW(kb);
  double w0[NR];
#pragma unroll
  for (int r = 0; r < NR; r++) w0[r] = nW[r];
  fetchW(kb + 1 <= Nr ? kb + 1 : Nr);
  fetch(kb);
#pragma unroll
  for (int n = 0; n < VM_S2; n++)
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const int ee = tid + r * VT_NT;
      if (ee < EN) s2[n * EN + ee] = ein[r] ? v2[n][r] : 0.0;
    }
#pragma unroll
  for (int r = 0; r < NR; r++) {
    const int ee = tid + r * VT_NT;
    if (ee < EN) sW[(kb & 1) * EN + ee] = (ein[r] && kb <= Nr) ? w0[r] : 0.0;
  }
  if (kb > 1) {
#pragma unroll
    for (int r = 0; r < NR; r++) {
      const int ee = tid + r * VT_NT;
      if (ee < EN) sHC[((kb - 1) & 1) * EN + ee] = ein[r] ? hcM[r] : 0.0;
    }
  }
  stashW(kb + 1);
  stash(kb);
  const int myIter = *iterPtr;
  const double abFac = (myIter == p.nIter0 && p.nIter0 == 0) ? 0.0 : 0.5 + p.abEps;   // adams_bashforth2.F:61-65
  const double mass2rUnit = 1.0 / p.rhoConst;
  constexpr bool rstar = P::nonlinFreeSurf > 0 && P::select_rStar > 0;
  __syncthreads();
#ifdef MGCM_VI_STAMPS
  unsigned long long viAcc[6] = {0, 0, 0, 0, 0, 0}, viPrev = 0;
  const unsigned long long viT0 = __builtin_amdgcn_s_memtime();
#endif
  for (int k = kb; k <= ke; k++) {
    VI_STAMP(0);
    int iL = i, jL = j;
    long q2L = q2;
    asm volatile("" : "+v"(iL), "+v"(jL), "+v"(q2L));
    [&](const int i, const int j, const long q2) {
    // the arena bases and strides re-materialised per level too: every field address derived
    // from them is then formed where it is used instead of hoisted out of the march and held
    // in scalar registers (which spill to VGPR lanes)
    Fields fl = f;
    Dims dl = d;
    asm volatile("" : "+s"(fl.a2), "+s"(fl.a3), "+s"(dl.N2all), "+s"(dl.N3all));
    const Fields &f = fl;
    const Dims &d = dl;
    VIMarchRegs c1;
    if constexpr (!CREG) load_c(c1, q2);
    const VIMarchRegs &c = CREG ? c0 : c1;
    const int kn = k + 1 <= Nr ? k + 1 : Nr, kw = k + 2 <= Nr ? k + 2 : Nr;
    if constexpr (PF) {
      fetch(kn);
      fetchW(kw);
    } else {
      const unsigned o = ob + (unsigned)(kn - 1) * lvB;
      oU = ld(bU, o); oV = ld(bV, o); oHW = ld(bHW, o); oHS = ld(bHS, o);
    }
    // EARLY: the level's own-point HBM reads, before the intermediates' barrier (the
    // pressure-gradient phi_hyd values of the linear free surface / non-rsc r* case only)
    constexpr bool rscE = rstar && P::select_rStar >= 2 && P::nonlinFreeSurf >= 4;
    double ePhi0 = 0.0, ePhiX = 0.0, ePhiY = 0.0, eGuo = 0.0, eGvo = 0.0;
    if constexpr (EARLY) {
      const long q3e = q2 + (long)(k - 1) * d.n2 + t3;
      eGuo = AR3(guNm1, q3e); eGvo = AR3(gvNm1, q3e);
      if constexpr (!rscE) { ePhi0 = AR3(phiHydC, q3e); ePhiX = AR3(phiHydC, q3e - 1); ePhiY = AR3(phiHydC, q3e - d.nx); }
    }
    VIM2<BX, BY, P, true> a{d, p, f, k, t, i0, j0, i, j, sU, sV, sHW, sHS, sHC, sW, s2, sKE, sVort, sHfz, sH0fz, sHDiv, c,
                            uM, k < Nr ? oU : 0.0, vM, k < Nr ? oV : 0.0, hwM, k < Nr ? oHW : 0.0, hsM, k < Nr ? oHS : 0.0};
    VIM2<BX, BY, P, false> ai{d, p, f, k, t, i0, j0, 0, 0, sU, sV, sHW, sHS, sHC, sW, s2, sKE, sVort, sHfz, sH0fz, sHDiv, c,
                              0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    // the level's 1-D factors and the own point's rest-state thicknesses, fetched here with
    // the level's other reads (vi_rdrC ... overloads)
    a.face = ai.face = tFace;
    a.edge = ai.edge = tEdge;
    a.rdrCk = f.recip_drC[k - 1];
    a.rdrCk1 = k < Nr ? f.recip_drC[k] : 0.0;
    a.rdrFk = f.recip_drF[k - 1];
    a.drFk = f.drF[k - 1];
    if constexpr (P::momViscosity && P::no_slip_sides) {
      const long q3h = q2 + (long)(k - 1) * d.n2 + t3;
      a.h0W = AR3(h0FacW, q3h);
      a.h0S = AR3(h0FacS, q3h);
    }
    for (int q = tid; q < IN; q += VT_NT) {
      const int ii = i0 + q % IW, jj = j0 + q / IW;          // vort / hFacZ grid: i0..i0+BX
      const bool ok = ii <= d.sNx + d.OLx && jj <= d.sNy + d.OLy;
      sHfz[q] = ok ? vi_hfacz(ai, d, ii, jj, k) : 0.0;
      sH0fz[q] = ok ? vi_h0facz(ai, d, p, ii, jj, k) : 0.0;
      sVort[q] = ok ? vi_vort(ai, d, p, f, ii, jj, k, t) : 0.0;
      sKE[q] = vi_KE(ai, d, p, f, ii - 1, jj - 1, k, t);     // KE / hDiv grid: i0-1..i0+BX-1
      sHDiv[q] = vi_hdiv(ai, d, p, f, ii - 1, jj - 1, k, t);
    }
    VI_STAMP(1);
    __syncthreads();
    VI_STAMP(2);
    if (act) {
      auto q3of = [&](long qq2, int kk) { return qq2 + (long)(kk - 1) * d.n2 + t3; };
      const long q3 = q3of(q2, k);
      const double recip_drF = a.rdrFk;
      // one component at a time (CC 1: U, 2: V): tendency, AB2, store, each from its own
      // vecinv_tend call whose other outputs are dead (the compiler drops their arithmetic;
      // the common reads are shared), a scheduling barrier between the two so the halves' live
      // values do not overlap: 215 against 247 VGPRs at 2 waves per SIMD, LLC-90's VI 319-320
      // against 323.7-323.8 us with both chains interleaved (round 6, profiles/r06/ab_hr_vi/);
      // capped for 3 waves per SIMD the split form still spills 43 VGPRs (605 us)
      auto comp = [&](auto tagC) {
        constexpr int CC = decltype(tagC)::value;   // 1: U, 2: V
        double gU = 0.0, gV = 0.0, guDiss = 0.0, gvDiss = 0.0, dPhiHydX = 0.0, dPhiHydY = 0.0;
        {  // CALC_GRAD_PHI_HYD (calc_grad_phi_hyd.F:152-214), as k_mom_step
          constexpr bool rsc = rstar && P::select_rStar >= 2 && P::nonlinFreeSurf >= 4;
          auto varLoc = [&](long qq2) {
            if constexpr (rsc) return AR3(phiHydC, q3of(qq2, k)) * AR2(rStarFacC, qq2) + 0.0;
            else return AR3(phiHydC, q3of(qq2, k)) + 0.0;
          };
          if constexpr (EARLY && !rsc) {
            const double vl = ePhi0 + 0.0;
            if (CC == 1 && i >= 1) dPhiHydX = c.recip_dxC * (vl - (ePhiX + 0.0));
            if (CC == 2 && j >= 1) dPhiHydY = c.recip_dyC * (vl - (ePhiY + 0.0));
          } else {
            const double vl = varLoc(q2);
            if (CC == 1 && i >= 1) dPhiHydX = c.recip_dxC * (vl - varLoc(q2 - 1));
            if (CC == 2 && j >= 1) dPhiHydY = c.recip_dyC * (vl - varLoc(q2 - d.nx));
          }
          if constexpr (rstar && P::select_rStar >= 2) {
            const double factorP = p.gravity * (1.0 / p.rhoConst) * 0.5, rCk = f.rC[k - 1];
            auto vl2 = [&](long qq2) { return AR2(etaH, qq2) * (1.0 + rCk * AR2(recip_Rcol, qq2)); };
            const double e0 = vl2(q2), a0 = AR3(alphaRho, q3);
            if (CC == 1 && i >= 1) dPhiHydX = dPhiHydX + factorP * (AR3(alphaRho, q3 - 1) + a0) * (e0 - vl2(q2 - 1)) * c.recip_dxC;
            if (CC == 2 && j >= 1) dPhiHydY = dPhiHydY + factorP * (AR3(alphaRho, q3 - d.nx) + a0) * (e0 - vl2(q2 - d.nx)) * c.recip_dyC;
          }
        }
        vecinv_tend(a, d, p, f, i, j, k, t, gU, gV, guDiss, gvDiss);
        double guExt = 0.0, gvExt = 0.0;
        if (P::momForcing && k == 1) {
          if (CC == 1 && j >= 0 && j <= d.sNy + 1 && i >= 1 && i <= d.sNx + 1)
            guExt = guExt + p.foFacMom * (AR2(fu, q2) * mass2rUnit) * recip_drF * a.recip_hFacW(i, j, k);
          if (CC == 2 && j >= 1 && j <= d.sNy + 1 && i >= 0 && i <= d.sNx + 1)
            gvExt = gvExt + p.foFacMom * (AR2(fv, q2) * mass2rUnit) * recip_drF * a.recip_hFacS(i, j, k);
        }
        double g = CC == 1 ? gU - p.pfFacMom * dPhiHydX : gV - p.pfFacMom * dPhiHydY;
        const double gDiss = CC == 1 ? guDiss : gvDiss, gExt = CC == 1 ? guExt : gvExt;
        if (P::momViscosity && P::momDissip_In_AB) g = g + gDiss;
        if (P::momForcing && P::momForcingOutAB != 1) g = g + gExt;
        {  // ADAMS_BASHFORTH2 (adams_bashforth2.F:81-88)
          const double go = CC == 1 ? (EARLY ? eGuo : AR3(guNm1, q3)) : (EARLY ? eGvo : AR3(gvNm1, q3));
          const double ab = abFac * (g - go);
          if (CC == 1) AR3(guNm1, q3) = g; else AR3(gvNm1, q3) = g;
          g = g + ab;
        }
        double gtmp = g;
        if (P::momForcing && P::momForcingOutAB == 1) gtmp = gtmp + gExt;
        if (P::momViscosity && !P::momDissip_In_AB) gtmp = gtmp + gDiss;
        if constexpr (rstar && P::nonlinFreeSurf > 1) gtmp = gtmp / (CC == 1 ? AR2(rStarExpW, q2) : AR2(rStarExpS, q2));
        if (CC == 1) AR3(gU, q3) = a.uVel(i, j, k) + p.deltaTMom * (gtmp + 0.0) * a.maskW(i, j, k);
        else AR3(gV, q3) = a.vVel(i, j, k) + p.deltaTMom * (gtmp + 0.0) * a.maskS(i, j, k);
      };
      comp(std::integral_constant<int, 1>{});
      __builtin_amdgcn_sched_barrier(0);   // U's chain before V's
      comp(std::integral_constant<int, 2>{});
    }
    VI_STAMP(3);
    }(iL, jL, q2L);
    if (k == ke) break;
    if (act) { const int eo = (j - j0 + 1) * EW + (i - i0 + 1); uM = sU[eo]; vM = sV[eo]; hwM = sHW[eo]; hsM = sHS[eo]; }
    if constexpr (!PF) {
      fetch(k + 1 <= Nr ? k + 1 : Nr);
      fetchW(k + 2 <= Nr ? k + 2 : Nr);
    }
    __syncthreads();
    VI_STAMP(4);
    stash(k + 1);
    stashW(k + 2);
    VI_STAMP(5);
    __syncthreads();
    VI_STAMP(6);
  }
#ifdef MGCM_VI_STAMPS
  if (threadIdx.x == 0 && (blockIdx.x % 97) == 0)
    printf("VISTAMP blk %d levels %d total %llu | phaseA %llu bar1 %llu phaseB %llu fetch+bar2 %llu stash %llu bar3 %llu\n",
           (int)blockIdx.x, ke - kb + 1, __builtin_amdgcn_s_memtime() - viT0, viAcc[0], viAcc[1], viAcc[2], viAcc[3],
           viAcc[4], viAcc[5]);
#endif
}

// The halo ring outside the DYNAMICS range (i or j outside 0..sN+1): no tendency, but
// ADAMS_BASHFORTH2 runs over the whole slab (gU = abFac*(0 - guNm1), guNm1 = 0), as
// k_mom_step does there.
// One thread per ring point (blockIdx.y = level, blockIdx.z = tile): the OLy-1 full rows
// below and above, then the OLx-1 columns left and right of the rows 0..sNy+1.
static int mom_halo_ring_count_host(const Dims &d) { return 2 * (d.OLy - 1) * d.nx + (d.sNy + 2) * 2 * (d.OLx - 1); }
__device__ __forceinline__ int mom_halo_ring_count(const Dims &d) {
  return 2 * (d.OLy - 1) * d.nx + (d.sNy + 2) * 2 * (d.OLx - 1);
}
__device__ __forceinline__ void mom_halo_ab_at(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, int r,
                                               int k, int t) {
  if (r >= mom_halo_ring_count(d)) return;
  const int nb = (d.OLy - 1) * d.nx, cw = 2 * (d.OLx - 1);
  int i, j;
  if (r < 2 * nb) {
    const int r2 = r < nb ? r : r - nb;
    j = (r < nb ? 1 - d.OLy : d.sNy + 2) + r2 / d.nx;
    i = 1 - d.OLx + r2 % d.nx;
  } else {
    const int r2 = r - 2 * nb, c = r2 % cw;
    j = r2 / cw;
    i = c < d.OLx - 1 ? 1 - d.OLx + c : d.sNx + 2 + (c - (d.OLx - 1));
  }
  const int myIter = *iterPtr;
  const double abFac = (myIter == p.nIter0 && p.nIter0 == 0) ? 0.0 : 0.5 + p.abEps;
  const long q3 = MG_I3(d, i, j, k, t);
  double gU = 0.0, gV = 0.0;
  const double gUo = AR3(guNm1, q3), gVo = AR3(gvNm1, q3);
  double ab = abFac * (gU - gUo);
  AR3(guNm1, q3) = gU;
  gU = gU + ab;
  ab = abFac * (gV - gVo);
  AR3(gvNm1, q3) = gV;
  gV = gV + ab;
  AR3(gU, q3) = gU;
  AR3(gV, q3) = gV;
}
__global__ void __launch_bounds__(256) k_mom_halo_ab(Dims d, Params p, Fields f, const int *iterPtr) {
  mom_halo_ab_at(d, p, f, iterPtr, (int)(blockIdx.x * blockDim.x + threadIdx.x), (int)blockIdx.y + 1,
                 d.t0 + (int)blockIdx.z);
}
// DO_OCEANIC_PHYS's per-point pass (k_oceanic_phys) with the halo ring's AB2 in extra
// workgroups of the same grid (nbRing per level and tile, after the nbPhys of the pass): the
// ring's gU/gV/guNm1/gvNm1 are read and written by nothing else of the step (launch_mom_ring),
// so its launch may be any of the step's -- one fewer launch on the staggered cube
// (one_step, MG_FUSE_RINGP)
__global__ void __launch_bounds__(256) k_phys_ring(Dims d, Params p, Fields f, const int *iterPtr, int nbPhys, int nbRing) {
  const int lb = mg_xcd_block();
  if (lb >= nbPhys) {
    const int l = lb - nbPhys, z = l / nbRing;
    mom_halo_ab_at(d, p, f, iterPtr, (l % nbRing) * (int)blockDim.x + (int)threadIdx.x, z % d.Nr + 1, d.t0 + z / d.Nr);
    return;
  }
  MG_PLANE_LB(1 - d.OLx, d.nx, 1 - d.OLy, d.ny, z, lb)
  const int t = d.t0 + z / d.Nr, k = z % d.Nr + 1;
  oceanic_phys_point(d, p, f, iterPtr, i, j, k, t);
}
hipError_t launch_phys_ring(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s) {
  const unsigned nbPhys = mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr);
  const int nbRing = (mom_halo_ring_count_host(d) + 255) / 256;
  hipLaunchKernelGGL(k_phys_ring, dim3(nbPhys + (unsigned)(nbRing * d.Nr * d.nT)), dim3(256), 0, s, d, p, f, iterPtr,
                     (int)nbPhys, nbRing);
  return hipGetLastError();
}

// k_mom_vi_m2's instantiations: (BX, BY, option code) of the workloads that run the k-march
// -- the LLC-90 synthetic (BASELINE config 5: 92-wide DYNAMICS range -> 31 x 8 blocks) and
// its LLC-30 shrink (32 x 8) with the same namelist.  Anything else runs k_mom_vi_march.
constexpr unsigned vi_code(int vs, int cs, int ks, int visc, int nss, int nsb, int impl, int cor, int adv, int upw,
                           int cube, int forc, int dissAB, int outAB1, int nlfs, int rstar) {
  return (unsigned)vs | (unsigned)cs << 2 | (unsigned)ks << 4 | (unsigned)visc << 6 | (unsigned)nss << 7 |
         (unsigned)nsb << 8 | (unsigned)impl << 9 | (unsigned)cor << 10 | (unsigned)adv << 11 | (unsigned)upw << 12 |
         (unsigned)cube << 13 | (unsigned)forc << 14 | (unsigned)dissAB << 15 | (unsigned)outAB1 << 16 |
         (unsigned)nlfs << 17 | (unsigned)rstar << 20;
}
constexpr unsigned VI_CODE_LLC = vi_code(1, 0, 0, 1, 1, 1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 0);
template <int BX, int BY, unsigned C, int V>
static void vi_m2_one(const Dims &d, const VIP<C> &vp, const Fields &f, const int *iterPtr, int nbx, int nby, int KC,
                      int nkc, hipStream_t s) {
  hipLaunchKernelGGL((k_mom_vi_m2<BX, BY, C, (V & 1) != 0, (V & 2) != 0, (V & 4) != 0, (V & 8) ? 2 : 1>),
                     dim3((unsigned)(nbx * nby * d.nT * nkc)), dim3(VT_NT), 0, s, d, vp, f, iterPtr, nbx, nby, KC, nkc);
}
// k_mom_vi_m2 as launched: the output point's metrics held in registers across the march
// (CREG), its own HBM reads of a level issued at the level's start (EARLY), registers capped
// for 2 waves per SIMD, level k+1 fetched after level k (LLC-90: 456-459 us; CREG alone 487,
// neither 534, the generic march 527; prefetching level k+1 into registers 513-740 (1 wave per
// SIMD or spills); a U/V-split 512-thread form 492, the same with a double-buffered prefetch
// 501, a two-pass form (intermediates through HBM, per-point tendencies) 585:
// profiles/r03/vi_m2/; the ring-point intermediates of the 31 x 8 block's second pass dealt
// out by quantity over the four waves 459 -> 518 us, profiles/r04/llc_ab/).  false where the
// run's option code or block shape has no instantiation (the generic march runs then).
static bool vi_m2_launch(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, int BX, int BY, int nbx,
                         int nby, int KC, int nkc, hipStream_t s) {
  const unsigned code = vi_opt_code(p);
  if (code == VI_CODE_LLC && BX == 31 && BY == 8) {
    vi_m2_one<31, 8, VI_CODE_LLC, 14>(d, vi_params<VI_CODE_LLC>(p), f, iterPtr, nbx, nby, KC, nkc, s);
    return true;
  }
  if (code == VI_CODE_LLC && BX == 32 && BY == 8) {
    vi_m2_one<32, 8, VI_CODE_LLC, 14>(d, vi_params<VI_CODE_LLC>(p), f, iterPtr, nbx, nby, KC, nkc, s);
    return true;
  }
  return false;
}

// block shape of k_mom_vi_tiled: BX along i (a whole output row when it is short), BY rows
static void vi_tile_shape(const Dims &d, int &BX, int &BY) {
  const int W = d.sNx + 2, H = d.sNy + 2;
  const int nbx = (W + 31) / 32;
  BX = (W + nbx - 1) / nbx;                 // 92 -> 31, 34 -> 17 (two blocks), <= 32
  BY = VT_NT / BX;
  while (BY > 1 && ((BX + 2) * (BY + 2) > VT_EMAX || (BX + 1) * (BY + 1) > VT_IMAX)) BY--;
  // (7 rows keep a 31-wide block's (BX+1)(BY+1) intermediate points within one pass of the
  // 256 threads, but the specialised k-march at 31 x 7 (more blocks, more spills) measured
  // slower on LLC-90: 1.58-1.60 against 1.54-1.56 ms/step, profiles/r04/viby/)
  const int nby = (H + BY - 1) / BY;
  BY = (H + nby - 1) / nby;                 // balance the rows over the blocks
}

// MOM_U_IMPLICIT_R / MOM_V_IMPLICIT_R (pkg/mom_common/mom_u_implicit_r.F:118-160,
// mom_v_implicit_r.F) with implicitViscosity only (momImplVertAdv = F, selectImplicitDrag
// = 0), after the DYNAMICS k loop (dynamics.F:568-580): the tri-diagonal system of the
// vertical viscosity on u* (V = false: i = 1..sNx+1, j = 1..sNy) or v* (V = true:
// i = 1..sNx, j = 1..sNy+1), solved in place with SOLVE_TRIDIAGONAL's default recurrence
// (solve_tridiagonal.F:224-297); outside that range the system is the identity.  Column
// frame as k_tracer_impl: k-parallel coefficients into LDS, one thread per column sweeps.
template <bool V>
__global__ void __launch_bounds__(256) k_mom_impl(Dims d, Params p, Fields f, int nc) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  MG_COLF(1, V ? d.sNx : d.sNx + 1, 1, V ? d.sNy + 1 : d.sNy, nc)
  const int Nr = d.Nr, NS = Nr * NC_;
  double *sSub = lds, *sSup = lds + NS, *sY = lds + 2 * NS;
  double *g = V ? f.a3 + (long)F3_gV * d.N3all : f.a3 + (long)F3_gU * d.N3all;
  const double *msk = V ? f.a3 + (long)F3_maskS * d.N3all : f.a3 + (long)F3_maskW * d.N3all;
  const double *rh = V ? f.a3 + (long)F3_recip_hFacS * d.N3all : f.a3 + (long)F3_recip_hFacW * d.N3all;
  if (valid) {
    MG_COLF_K(k) {
      const int me = (k - 1) * NC_ + cc;
      const long q3 = MG_I3(d, i, j, k, t);
      double sub = 0.0, sup = 0.0;   // kappaRU = kappaRV = viscArNr(k) (calc_viscosity.F)
      if (k >= 2 && msk[MG_I3(d, i, j, k - 1, t)] == 1.0)
        sub = -(p.deltaTMom * rh[q3] * f.recip_drF[k - 1] * p.viscAr * f.recip_drC[k - 1]);
      if (k <= Nr - 1 && msk[MG_I3(d, i, j, k + 1, t)] == 1.0)
        sup = -(p.deltaTMom * rh[q3] * f.recip_drF[k - 1] * p.viscAr * f.recip_drC[k]);
      sSub[me] = sub;
      sSup[me] = sup;
      sY[me] = g[q3];
    }
  }
  __syncthreads();
  if (valid && kk == 0) {
    double cpPrev = 0.0, ypPrev = 0.0;
    for (int k2 = 1; k2 <= Nr; k2++) {
      const int s2 = (k2 - 1) * NC_ + cc;
      const double sub = sSub[s2], sup = sSup[s2];
      const double diag = 1.0 - (sub + sup);
      const double y = sY[s2];
      double cp, yp;
      if (k2 == 1) {
        if (diag != 0.0) { const double rec = 1.0 / diag; cp = sup * rec; yp = y * rec; }
        else { cp = 0.0; yp = 0.0; }
      } else {
        const double tmp = diag - sub * cpPrev;
        if (tmp != 0.0) { const double rec = 1.0 / tmp; cp = sup * rec; yp = (y - sub * ypPrev) * rec; }
        else { cp = 0.0; yp = 0.0; }
      }
      sSup[s2] = cp;
      sY[s2] = yp;
      cpPrev = cp; ypPrev = yp;
    }
    double below = 0.0;
    for (int k2 = Nr; k2 >= 1; k2--) {
      const int s2 = (k2 - 1) * NC_ + cc;
      const double v = (k2 == Nr) ? sY[s2] : sY[s2] - sSup[s2] * below;
      sSub[s2] = v;
      below = v;
    }
  }
  __syncthreads();
  if (valid) MG_COLF_K(k) g[MG_I3(d, i, j, k, t)] = sSub[(k - 1) * NC_ + cc];
}

// IMPLDIFF (model/src/impldiff.F:24-245, tracerId = 0: deltaTMom) on the CD scheme's D-grid
// velocities after the DYNAMICS k loop (dynamics.F:614-634): V = false vVelD with kappaRU and
// recip_hFacW, V = true uVelD with kappaRV and recip_hFacS (the reference's pairing: vVelD
// sits on u points), on i = 0..sNx+1, j = 0..sNy+1.  IMPLDIFF's own recurrence, not
// SOLVE_TRIDIAGONAL's: a(k) / c(k) vanish where recip_hFac of the level above / below is 0,
// bet = 1 (gam = c*bet) where a pivot is 0.  Column frame as k_mom_impl: k-parallel
// coefficients into LDS, one thread per column sweeps (gam overwrites c, the forward
// solution the right-hand side).
template <bool V>
__global__ void __launch_bounds__(256) k_impldiff_cd(Dims d, Params p, Fields f, int nc) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  MG_COLF(0, d.sNx + 2, 0, d.sNy + 2, nc)
  const int Nr = d.Nr, NS = Nr * NC_;
  double *sA = lds, *sC = lds + NS, *sY = lds + 2 * NS;
  double *g = V ? f.uVelD : f.vVelD;
  const double *rh = V ? f.recip_hFacS : f.recip_hFacW;
  if (valid) {
    MG_COLF_K(k) {
      const int me = (k - 1) * NC_ + cc;
      const long q3 = MG_I3(d, i, j, k, t);
      double a = 0.0, c = 0.0;   // kappaRU = kappaRV = viscArNr(k) (calc_viscosity.F)
      if (k >= 2) {
        a = -(p.deltaTMom * rh[q3] * f.recip_drF[k - 1] * p.viscAr * f.recip_drC[k - 1]);
        if (rh[MG_I3(d, i, j, k - 1, t)] == 0.0) a = 0.0;
      }
      if (k <= Nr - 1) {
        c = -(p.deltaTMom * rh[q3] * f.recip_drF[k - 1] * p.viscAr * f.recip_drC[k]);
        if (rh[MG_I3(d, i, j, k + 1, t)] == 0.0) c = 0.0;
      }
      sA[me] = a;
      sC[me] = c;
      sY[me] = g[q3];
    }
  }
  __syncthreads();
  if (valid && kk == 0) {
    double betPrev = 1.0, ltPrev = 0.0, cPrev = 0.0;
    for (int k2 = 1; k2 <= Nr; k2++) {
      const int s2 = (k2 - 1) * NC_ + cc;
      const double a = sA[s2], c = sC[s2];
      const double b = 1.0 - (a + c);
      double bet = 1.0, gam = 0.0;
      if (Nr > 1) {
        if (k2 == 1) {
          if (b != 0.0) bet = 1.0 / b;
        } else {
          gam = cPrev * betPrev;
          if ((b - a * gam) != 0.0) bet = 1.0 / (b - a * gam);
        }
      }
      const double lt = (k2 == 1) ? sY[s2] * bet : bet * (sY[s2] - a * ltPrev);
      sY[s2] = lt;
      sC[s2] = gam;   // gam(k2): read by level k2 - 1 on the way up
      betPrev = bet; ltPrev = lt; cPrev = c;
    }
    double above = sY[(Nr - 1) * NC_ + cc];
    for (int k2 = Nr - 1; k2 >= 1; k2--) {
      const int s2 = (k2 - 1) * NC_ + cc;
      const double v = sY[s2] - sC[s2 + NC_] * above;
      sY[s2] = v;
      above = v;
    }
  }
  __syncthreads();
  if (valid) MG_COLF_K(k) g[MG_I3(d, i, j, k, t)] = sY[(k - 1) * NC_ + cc];
}

static bool del2_needed(const Params &p) { return p.momViscosity && (p.viscA4D != 0.0 || p.viscA4Z != 0.0); }
// k_del2uv rides in CALC_PHI_HYD's launch (k_phi_del2) on the small grids
static bool phi_del2_fused(const Dims &d, const Params &p) { return del2_needed(p) && mg_hfuse(MG_FUSE_PHI, d.nx, d.ny, d.nT, d.Nr); }

// DO_OCEANIC_PHYS + CALC_PHI_HYD in one column pass (k_phys_phi) when that is exact: no
// GM/Redi tensor between them (it reads rhoInSitu at neighbours) and phi not already sharing
// a grid with del2uv; MGCM_STEP_FUSE bit MG_FUSE_PHYS.  Returns false when not applicable.
bool phys_phi_fusable(const Dims &d, const Params &p) {
  return mg_fuse_on(MG_FUSE_PHYS) && !p.useGMRedi && !phi_del2_fused(d, p);
}
hipError_t launch_phys_phi(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s) {
  const long ncol = (long)d.nx * d.ny * d.nT;
  const int nc = 16;   // columns per workgroup
  MG_ALLOW_LDS(k_phys_phi);
  hipLaunchKernelGGL(k_phys_phi, dim3(mg_colf_blocks(ncol, nc)), dim3(256), mg_colf_lds(d.Nr, nc, 6), s, d, p, f, nc,
                     iterPtr);
  return hipGetLastError();
}

hipError_t launch_phi_hyd(const Dims &d, const Params &p, const Fields &f, hipStream_t s) {
  const long ncol = (long)(d.sNx + 3) * (d.sNy + 3) * d.nT;
  // LDS slices: the phi sums need 3 (sM, sP, sPh); r* adds MOM_CALC_RTRANS's 3
  const bool rstar = p.nonlinFreeSurf > 0 && p.select_rStar > 0;
  const int nArr = rstar ? 6 : 3;
  const int nc = mg_colf_nc(ncol, d.Nr, nArr);
  if (phi_del2_fused(d, p)) {
    MG_ALLOW_LDS(k_phi_del2);
    const unsigned nbPhi = mg_colf_blocks(ncol, nc), nbDel = mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr);
    hipLaunchKernelGGL(k_phi_del2, dim3(nbPhi + nbDel), dim3(256), mg_colf_lds(d.Nr, nc, nArr), s, d, p, f, nc, (int)nbPhi);
    return hipGetLastError();
  }
  // the flat per-column form (phi_flat_on)
  if (phi_flat_on(p)) {
    const bool qh = p.quasiHydrostatic && (p.select3dCoriScheme >= 1 || p.useNHMTerms);
    // (round 4: a two-columns-per-thread form was bit-identical but slower on LLC-90, 32.8
    // against 30.4 us -- half the threads leave the chip under-filled; removed in round 5)
    auto kern = rstar ? (qh ? k_phi_flat<true, true> : k_phi_flat<true, false>)
                      : (qh ? k_phi_flat<false, true> : k_phi_flat<false, false>);
    // at BASELINE config 5's depth the chunk loop unrolled (round 5: LLC-90 24.3 against 30 us,
    // step 1.416-1.418 ms, profiles/r05/phi_n50/)
    if (!rstar && !qh && d.Nr == 50) kern = k_phi_flat<false, false, 50>;
    hipLaunchKernelGGL(kern, dim3((unsigned)phi_flat_blocks(d, p)), dim3(256), 0, s, d, p, f);
    return hipGetLastError();
  }
  MG_ALLOW_LDS(k_phi_hyd);
  hipLaunchKernelGGL(k_phi_hyd, dim3(mg_colf_blocks(ncol, nc)), dim3(256), mg_colf_lds(d.Nr, nc, nArr), s, d, p, f, nc);
  return hipGetLastError();
}

static hipError_t launch_mom_tail(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s);
// DYNAMICS after CALC_PHI_HYD (launch_phi_hyd): momentum tendencies, TIMESTEP, AB2, CD scheme,
// implicit vertical viscosity
// The VI path's ADAMS_BASHFORTH2 on the halo ring (k_mom_halo_ab) as a launch of its own:
// nothing of the step reads the ring's gU/gV before the end-of-step exchange overwrites the
// halos, and nothing else of DYNAMICS writes it (the CD scheme excepted, whose range reaches
// it), so the resident step may run it on the second stream beside the pressure solve
// (one_step, MG_FUSE_RING).  ring = false: launch_mom_step leaves it to launch_mom_ring.
static bool vi_march_path(const Dims &d, const Params &p) {
  return p.vectorInvariantMomentum && d.OLx >= 2 && d.OLy >= 2 && p.selectVortScheme <= 2;
}
bool mom_ring_separable(const Dims &d, const Params &p) {
  return vi_march_path(d, p) && !p.useCDscheme && 2 * (d.OLy - 1) * d.nx + (d.sNy + 2) * 2 * (d.OLx - 1) > 0;
}
hipError_t launch_mom_ring(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s) {
  const int ring = 2 * (d.OLy - 1) * d.nx + (d.sNy + 2) * 2 * (d.OLx - 1);
  if (ring > 0)
    hipLaunchKernelGGL(k_mom_halo_ab, dim3((unsigned)((ring + 255) / 256), d.Nr, d.nT), dim3(256), 0, s, d, p, f, iterPtr);
  return hipGetLastError();
}
hipError_t launch_mom_step(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s, bool ring) {
  if (del2_needed(p) && !phi_del2_fused(d, p))
    hipLaunchKernelGGL(k_del2uv, dim3(mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr)), dim3(MG_PLANE_THREADS), 0, s, d, p, f);
  // MOM_VECINV or MOM_FLUXFORM: separate instantiations (no register-pressure coupling)
  if (vi_march_path(d, p)) {
    int BX, BY;
    vi_tile_shape(d, BX, BY);
    const int nbx = (d.sNx + 2 + BX - 1) / BX, nby = (d.sNy + 2 + BY - 1) / BY;
    // levels per workgroup: enough workgroups to fill the chip, few enough that the two extra
    // staged levels per chunk stay a small overhead.  The k-march for deep grids (Nr >= 30
    // with >= 256 workgroups per level chunk), in two chunks of levels (round 4, k_mom_vi_m2:
    // LLC-90 448-456 us against 460 at five and 453-460 at three, step 1.531-1.545 against
    // 1.550-1.552 ms, profiles/r04/vikc/) or one (below); otherwise one level per
    // workgroup.  MGCM_VI_KERNEL = march | march_generic | level | tiled forces a form (the
    // tests run each: march_generic is the generic k-march that serves option sets without
    // a k_mom_vi_m2 instantiation; read per launch)
    const char *viEnv = getenv("MGCM_VI_KERNEL");
    const int nbt = nbx * nby * d.nT;
    // Round 6: the whole column per workgroup where the blocks then fit one resident round (2
    // workgroups of k_mom_vi_m2 per CU, 256 CUs): LLC-90's 468 blocks, 313 against 319-320 us
    // for two chunks (936 workgroups, 1.83 rounds) and 321 for three (profiles/r06/vikc/);
    // MGCM_VI_KC forces the levels per workgroup (tests: ragged chunks)
    const char *kcEnv = getenv("MGCM_VI_KC");
    const int KCm = kcEnv ? std::max(1, atoi(kcEnv)) : (nbx * nby * d.nT <= 512 ? d.Nr : (d.Nr + 1) / 2);
    const bool generic = viEnv && !strcmp(viEnv, "march_generic");
    const bool march = viEnv ? (!strcmp(viEnv, "march") || generic) : (d.Nr >= 30 && nbt >= 256);
    if (march) {
      const int nkc = (d.Nr + KCm - 1) / KCm;
      if (generic || !vi_m2_launch(d, p, f, iterPtr, BX, BY, nbx, nby, KCm, nkc, s))
        hipLaunchKernelGGL((k_mom_vi_march<false, false>), dim3((unsigned)(nbt * nkc)), dim3(VT_NT), 0, s, d, p, f, iterPtr,
                           BX, BY, nbx, nby, KCm, nkc);
    } else if (!(viEnv && !strcmp(viEnv, "tiled"))) {   // one level per workgroup
      hipLaunchKernelGGL(k_mom_vi_level, dim3((unsigned)(nbx * nby * d.nT * d.Nr)), dim3(VT_NT), 0, s, d, p, f, iterPtr, BX,
                         BY, nbx, nby);
    } else {            // KCm levels marched per workgroup, the tiled form
      const int nkc = (d.Nr + KCm - 1) / KCm;
      hipLaunchKernelGGL(k_mom_vi_tiled, dim3((unsigned)(nbt * nkc)), dim3(VT_NT), 0, s, d, p, f, iterPtr, BX, BY, nbx,
                         nby, KCm, nkc);
    }
    if (ring || p.useCDscheme) launch_mom_ring(d, p, f, iterPtr, s);
  } else if (p.vectorInvariantMomentum)
    hipLaunchKernelGGL(k_mom_step<true>, dim3(mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr)), dim3(MG_PLANE_THREADS), 0, s,
                       d, p, f, iterPtr);
  else if (mom_ff4_on())   // MOM_FLUXFORM: four threads per point (U, V x viscous or not)
    hipLaunchKernelGGL(k_mom_ff4, dim3((unsigned)mom_ff4_blocks(d)), dim3(256), 0, s, d, p, f, iterPtr);
  else   // MOM_FLUXFORM: U and V halves as separate threads (twice the workgroups, half the chain)
    hipLaunchKernelGGL(k_mom_step_uv<false>, dim3(2 * mg_plane_blocks(d.nx, d.ny, d.nT * d.Nr)), dim3(MG_PLANE_THREADS), 0,
                       s, d, p, f, iterPtr);
  return launch_mom_tail(d, p, f, iterPtr, s);
}

// the end of DYNAMICS after the tendencies: CD scheme, implicit vertical viscosity
static hipError_t launch_mom_tail(const Dims &d, const Params &p, const Fields &f, const int *iterPtr, hipStream_t s) {
  if (p.useCDscheme)
    hipLaunchKernelGGL(k_cd_scheme, dim3(mg_plane_blocks(d.nx - 2, d.ny - 2, d.nT * d.Nr)), dim3(MG_PLANE_THREADS), 0, s,
                       d, p, f, iterPtr);
  if (p.implicitViscosity && d.Nr > 1) {   // dynamics.F:568-580
    const long ncU = (long)(d.sNx + 1) * d.sNy * d.nT, ncV = (long)d.sNx * (d.sNy + 1) * d.nT;
    const int nc = mg_colf_nc(ncU, d.Nr, 3);
    MG_ALLOW_LDS(k_mom_impl<false>);
    MG_ALLOW_LDS(k_mom_impl<true>);
    hipLaunchKernelGGL(k_mom_impl<false>, dim3(mg_colf_blocks(ncU, nc)), dim3(256), mg_colf_lds(d.Nr, nc, 3), s, d, p, f, nc);
    hipLaunchKernelGGL(k_mom_impl<true>, dim3(mg_colf_blocks(ncV, nc)), dim3(256), mg_colf_lds(d.Nr, nc, 3), s, d, p, f, nc);
  }
  if (p.implicitViscosity && p.useCDscheme) {   // dynamics.F:614-634
    const long ncD = (long)(d.sNx + 2) * (d.sNy + 2) * d.nT;
    const int nc = mg_colf_nc(ncD, d.Nr, 3);
    MG_ALLOW_LDS(k_impldiff_cd<false>);
    MG_ALLOW_LDS(k_impldiff_cd<true>);
    hipLaunchKernelGGL(k_impldiff_cd<false>, dim3(mg_colf_blocks(ncD, nc)), dim3(256), mg_colf_lds(d.Nr, nc, 3), s, d, p, f, nc);
    hipLaunchKernelGGL(k_impldiff_cd<true>, dim3(mg_colf_blocks(ncD, nc)), dim3(256), mg_colf_lds(d.Nr, nc, 3), s, d, p, f, nc);
  }
  return hipGetLastError();
}

}  // namespace mgcm
