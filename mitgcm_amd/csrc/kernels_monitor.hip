// kernels_monitor.hip -- MONITOR's dynstat block on the device (pkg/monitor/monitor.F:103-129
// -> MON_CALC_STATS_RL, pkg/monitor/mon_calc_stats_rl.F:60-160 and mon_stats_rl.F:104-107):
// max, min, mean, standard deviation and the del2 roughness of eta, u, v, w, theta and salt,
// without downloading the fields.
//
// One workgroup per (field, tile, level) plane: its 256 threads sweep the plane's interior
// points (i fastest, point p by thread p mod 256), then reduce the thread terms by a fixed
// pairwise tree in LDS -- so the plane partials do not depend on placement or timing.  The
// host side (mgcm_monitor, model.hip) adds the plane partials in (tile, level) order, as
// MON_CALC_STATS_RL adds its per-tile sums with GLOBAL_SUM_TILE_RL, and runs the second
// (standard deviation) pass with the global mean.  The per-tile sums of the reference are
// sequential over (k, j, i); the device's are trees, so the statistics agree to rounding
// (tests/test_gpu_monitor.py: <= 1e-12 relative, min/max exact).
#include "common.h"

namespace mgcm {

__global__ void __launch_bounds__(256) k_mon_stats(Dims d, MonSpecs S, int nzmax, double *__restrict__ out, int pass) {
  __shared__ double red[MON_NV][256];
  const int b = (int)blockIdx.x;
  const int k = b % nzmax, t = d.t0 + (b / nzmax) % d.nT, fi = b / (nzmax * d.nT);
  const MonSpec &s = S.s[fi];
  if (k >= s.nz) return;   // the whole workgroup leaves: no barrier is reached
  const int tid = threadIdx.x;
  const long a0 = s.arr3d ? (long)t * d.n3 + (long)k * d.n2 : (long)t * d.n2;
  const long h0 = s.hf3d ? (long)t * d.n3 + (long)k * d.n2 : (long)t * d.n2;
  const long m0 = (long)t * d.n2;
  const double drk = s.dr[k];
  const double mean = S.mean[fi];
  double nb = 0.0, d2 = 0.0, vol = 0.0, mv = 0.0, mn = INFINITY, mx = -INFINITY;
  const int np = d.sNx * d.sNy;
  for (int p = tid; p < np; p += 256) {
    const int i = p % d.sNx + 1, j = p / d.sNx + 1;
    const long l = MG_I2(d, i, j, 0);
    const double v = s.arr[a0 + l];
    const double msk = s.mask[m0 + l] * s.hfac[h0 + l];
    if (!(msk > 0.0)) continue;
    const double tv = s.area[m0 + l] * drk * msk;
    if (pass == 0) {
      mn = fmin(mn, v);
      mx = fmax(mx, v);
      double ddx = s.hfac[h0 + l + 1] * s.hfac[h0 + l - 1];
      if (ddx > 0.0) ddx = (s.arr[a0 + l + 1] - v) + (s.arr[a0 + l - 1] - v);
      double ddy = s.hfac[h0 + l + d.nx] * s.hfac[h0 + l - d.nx];
      if (ddy > 0.0) ddy = (s.arr[a0 + l + d.nx] - v) + (s.arr[a0 + l - d.nx] - v);
      d2 = d2 + ddx * ddx + ddy * ddy;
      nb = nb + 1.0;
      vol = vol + tv;
      mv = mv + tv * v;
    } else {
      mv = mv + tv * (v - mean) * (v - mean);   // mon_calc_stats_rl.F: the SD pass
    }
  }
  red[0][tid] = nb; red[1][tid] = d2; red[2][tid] = vol; red[3][tid] = mv; red[4][tid] = mn; red[5][tid] = mx;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) {
      for (int q = 0; q < 4; q++) red[q][tid] = red[q][tid] + red[q][tid + w];
      red[4][tid] = fmin(red[4][tid], red[4][tid + w]);
      red[5][tid] = fmax(red[5][tid], red[5][tid + w]);
    }
    __syncthreads();
  }
  if (tid < MON_NV) out[(size_t)b * MON_NV + tid] = red[tid][0];
}

hipError_t launch_mon_stats(const Dims &d, const MonSpecs &S, int nzmax, double *out, int pass, hipStream_t st) {
  hipLaunchKernelGGL(k_mon_stats, dim3((unsigned)(MON_NF * d.nT * nzmax)), dim3(256), 0, st, d, S, nzmax, out, pass);
  return hipGetLastError();
}

}  // namespace mgcm
