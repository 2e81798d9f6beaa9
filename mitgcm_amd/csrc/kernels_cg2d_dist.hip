// Distributed CG2D: the reference's own algorithm (model/src/cg2d.F:100-415) split at its
// global operations, for tile-sharded runs (mitgcm_amd/parallel.py drives the iteration).
// Every op runs one 1024-thread workgroup per tile this process owns and writes that tile's
// partial sum(s) to part[2*tile + s] -- the per-tile buffer GLOBAL_SUM_TILE_RL collects
// (eesupp/src/global_sum_tile.F:161-191): the host all-gathers the partials over
// torch.distributed (RCCL on MI355X nodes) and adds them in global tile order, so the sums,
// and with them every iterate, are the same at any process count.  Within a tile the
// partial is accumulated in a fixed order: each thread adds its points (q = tid, tid+1024,
// ... in i-fastest order), then a pairwise tree over the 1024 threads.
//   op 0  b = b*cg2dNorm, partial max|b|                    (cg2d.F:104-114)
//   op 1  b = b*rhsNorm, x = x*rhsNorm  (a0 = rhsNorm)      (cg2d.F:116-133)
//   op 2  r = s = 0 on 0..sN+1, r = b - A x; partials sum r*r, sum b   (cg2d.F:136-175)
//   op 3  q = M r (the preconditioner); partial sum q*r     (cg2d.F:205-230)
//   op 4  s = q + beta*s  (a0 = beta)                        (cg2d.F:246-254)
//   op 5  q = A s; partial sum s*q                           (cg2d.F:262-287)
//   op 6  x = x + alpha*s, r = r - alpha*q; partial sum r*r  (a0 = alpha, cg2d.F:297-318)
//   op 7  x = x/rhsNorm  (a0 = rhsNorm)                      (cg2d.F:372-385)
//   op 8  cg2d_min = x  (the lowest-residual solution so far, cg2dUseMinResSol; cg2d.F:148-155, 338-351)
//   op 9  x = cg2d_min  (the solve ended above its lowest residual, cg2d.F:358-369)
// CG2D_SR (cg2d_sr.F, useSRCGSolver): the same ops 0-2, 5, 7-9 and
//   op 10 y = M r, s = y; partial sum y*r                   (cg2d_sr.F:223-243)
//   op 11 x = x + a0*s, r = r - a0*q  (a0 = sigma)           (cg2d_sr.F:279-288, 396-401)
//   op 12 y = M r                                            (cg2d_sr.F:300-316)
//   op 13 v = A y; partials sum y*r, sum y*v                 (cg2d_sr.F:324-347)
//   op 14 partial sum r*r                                    (cg2d_sr.F:344-345, 411-422)
//   op 15 s = y + a0*s, q = v + a0*q  (a0 = cgBeta)          (cg2d_sr.F:394-399)
// (the reference's one GLOBAL_SUM_VECTOR_RL of three per-tile values, cg2d_sr.F:348-358, is
// three tile-ordered sums: ops 13 and 14 hand the host the same per-tile partials)
// The width-1 EXCH_S3D_RL of r and s (cg2d.F:175,255,353) and EXCH_XY_RL of x (:135) are
// the host's point-to-point exchange plus mgcm_exchange_field.
#include "common.h"

namespace mgcm {

constexpr int CGD_NT = 1024;

__device__ __forceinline__ double cgd_tree(double v, double *sh, bool isMax) {
  const int tid = threadIdx.x;
  __syncthreads();
  sh[tid] = v;
  __syncthreads();
  for (int st = CGD_NT / 2; st > 0; st >>= 1) {
    if (tid < st) sh[tid] = isMax ? fmax(sh[tid], sh[tid + st]) : sh[tid] + sh[tid + st];
    __syncthreads();
  }
  return sh[0];
}

__global__ void __launch_bounds__(CGD_NT) k_cgd(Dims d, Params p, Fields f, int op, double a0, double *part) {
  __shared__ double sh[CGD_NT];
  const int t = d.t0 + (int)blockIdx.x, tid = threadIdx.x;
  const int sNx = d.sNx, sNy = d.sNy;
#define A2(x, ii, jj) AR2(x, MG_I2(d, ii, jj, t))
  if (op == 2) {   // r = s = 0 on the ring 0..sN+1 (the interior is overwritten below)
    const int nr = (sNx + 2) * (sNy + 2);
    for (int q = tid; q < nr; q += CGD_NT) {
      const int i = q % (sNx + 2), j = q / (sNx + 2);
      A2(cg2d_r, i, j) = 0.0;
      A2(cg2d_s, i, j) = 0.0;
      A2(cg2d_y, i, j) = 0.0;
    }
    __syncthreads();
  }
  double s0 = 0.0, s1 = 0.0;
  const int npt = sNx * sNy;
  for (int q = tid; q < npt; q += CGD_NT) {
    const int i = 1 + q % sNx, j = 1 + q / sNx;
    switch (op) {
      case 0: {
        const double b = A2(cg2d_b, i, j) * p.cg2dNorm;
        A2(cg2d_b, i, j) = b;
        s0 = fmax(fabs(b), s0);
        break;
      }
      case 1:
        A2(cg2d_b, i, j) = A2(cg2d_b, i, j) * a0;
        A2(cg2d_x, i, j) = A2(cg2d_x, i, j) * a0;
        break;
      case 2: {
        const double r = A2(cg2d_b, i, j) -
                         (A2(aW2d, i, j) * A2(cg2d_x, i - 1, j) + A2(aW2d, i + 1, j) * A2(cg2d_x, i + 1, j) +
                          A2(aS2d, i, j) * A2(cg2d_x, i, j - 1) + A2(aS2d, i, j + 1) * A2(cg2d_x, i, j + 1) +
                          A2(aC2d, i, j) * A2(cg2d_x, i, j));
        A2(cg2d_r, i, j) = r;
        s0 = s0 + r * r;
        s1 = s1 + A2(cg2d_b, i, j);
        break;
      }
      case 3: {
        const double r = A2(cg2d_r, i, j);
        const double z = A2(pC, i, j) * r + A2(pW, i, j) * A2(cg2d_r, i - 1, j) + A2(pW, i + 1, j) * A2(cg2d_r, i + 1, j) +
                         A2(pS, i, j) * A2(cg2d_r, i, j - 1) + A2(pS, i, j + 1) * A2(cg2d_r, i, j + 1);
        A2(cg2d_q, i, j) = z;
        s0 = s0 + z * r;
        break;
      }
      case 4:
        A2(cg2d_s, i, j) = A2(cg2d_q, i, j) + a0 * A2(cg2d_s, i, j);
        break;
      case 5: {
        const double sv = A2(cg2d_s, i, j);
        const double q2 = A2(aW2d, i, j) * A2(cg2d_s, i - 1, j) + A2(aW2d, i + 1, j) * A2(cg2d_s, i + 1, j) +
                          A2(aS2d, i, j) * A2(cg2d_s, i, j - 1) + A2(aS2d, i, j + 1) * A2(cg2d_s, i, j + 1) +
                          A2(aC2d, i, j) * sv;
        A2(cg2d_q, i, j) = q2;
        s0 = s0 + sv * q2;
        break;
      }
      case 6: {
        A2(cg2d_x, i, j) = A2(cg2d_x, i, j) + a0 * A2(cg2d_s, i, j);
        const double r = A2(cg2d_r, i, j) - a0 * A2(cg2d_q, i, j);
        A2(cg2d_r, i, j) = r;
        s0 = s0 + r * r;
        break;
      }
      case 7:
        A2(cg2d_x, i, j) = A2(cg2d_x, i, j) / a0;
        break;
      case 8:
        A2(cg2d_min, i, j) = A2(cg2d_x, i, j);
        break;
      case 9:
        A2(cg2d_x, i, j) = A2(cg2d_min, i, j);
        break;
      case 10:
      case 12: {
        const double r = A2(cg2d_r, i, j);
        const double y = A2(pC, i, j) * r + A2(pW, i, j) * A2(cg2d_r, i - 1, j) + A2(pW, i + 1, j) * A2(cg2d_r, i + 1, j) +
                         A2(pS, i, j) * A2(cg2d_r, i, j - 1) + A2(pS, i, j + 1) * A2(cg2d_r, i, j + 1);
        A2(cg2d_y, i, j) = y;
        if (op == 10) {
          A2(cg2d_s, i, j) = y;
          s0 = s0 + y * r;
        }
        break;
      }
      case 11:
        A2(cg2d_x, i, j) = A2(cg2d_x, i, j) + a0 * A2(cg2d_s, i, j);
        A2(cg2d_r, i, j) = A2(cg2d_r, i, j) - a0 * A2(cg2d_q, i, j);
        break;
      case 13: {
        const double y = A2(cg2d_y, i, j);
        const double v = A2(aW2d, i, j) * A2(cg2d_y, i - 1, j) + A2(aW2d, i + 1, j) * A2(cg2d_y, i + 1, j) +
                         A2(aS2d, i, j) * A2(cg2d_y, i, j - 1) + A2(aS2d, i, j + 1) * A2(cg2d_y, i, j + 1) +
                         A2(aC2d, i, j) * y;
        A2(cg2d_v, i, j) = v;
        s0 = s0 + y * A2(cg2d_r, i, j);
        s1 = s1 + y * v;
        break;
      }
      case 14: {
        const double r = A2(cg2d_r, i, j);
        s0 = s0 + r * r;
        break;
      }
      case 15:
        A2(cg2d_s, i, j) = A2(cg2d_y, i, j) + a0 * A2(cg2d_s, i, j);
        A2(cg2d_q, i, j) = A2(cg2d_v, i, j) + a0 * A2(cg2d_q, i, j);
        break;
    }
  }
#undef A2
  if (op == 1 || op == 4 || (op >= 7 && op <= 9) || op == 11 || op == 12 || op == 15) return;
  const double v0 = cgd_tree(s0, sh, op == 0);
  const double v1 = (op == 2 || op == 13) ? cgd_tree(s1, sh, false) : 0.0;
  if (tid == 0) { part[2 * t] = v0; part[2 * t + 1] = v1; }
}

// the SolveRecord of this step (cg2d.F's output arguments), written where the device
// solvers write theirs
__global__ void k_cgd_record(SolveRecord *rec, const int *stepCounter, double first, double last, double rhsMax,
                             double sumRHS, int iters, double minResidualSq, int nIterMin) {
  SolveRecord &R = rec[stepCounter ? *stepCounter : 0];
  R.firstResidual = first;
  R.lastResidual = last;
  R.minResidualSq = minResidualSq;
  R.rhsMax = rhsMax;
  R.sumRHS = sumRHS;
  R.numIters = iters;
  R.nIterMin = nIterMin;
}

// gather (unpack = 0) or scatter (1) one 2-D field at whole-domain flat offsets idx[0..n)
__global__ void k_field_pack(double *a, const long *idx, long n, double *buf, int unpack) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  if (unpack) a[idx[q]] = buf[q];
  else buf[q] = a[idx[q]];
}

hipError_t launch_cgd(const Dims &d, const Params &p, const Fields &f, int op, double a0, double *part, hipStream_t s) {
  if (d.nT <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_cgd, dim3((unsigned)d.nT), dim3(CGD_NT), 0, s, d, p, f, op, a0, part);
  return hipGetLastError();
}

hipError_t launch_cgd_record(SolveRecord *rec, const int *stepCounter, double first, double last, double rhsMax,
                             double sumRHS, int iters, double minResidualSq, int nIterMin, hipStream_t s) {
  hipLaunchKernelGGL(k_cgd_record, dim3(1), dim3(1), 0, s, rec, stepCounter, first, last, rhsMax, sumRHS, iters,
                     minResidualSq, nIterMin);
  return hipGetLastError();
}

hipError_t launch_field_pack(double *a, const long *idx, long n, double *buf, int unpack, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_field_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, idx, n, buf, unpack);
  return hipGetLastError();
}

}  // namespace mgcm
