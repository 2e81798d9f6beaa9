#!/usr/bin/env python3
"""Benchmark of the MI355X-native MITgcm hot path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME]

A "step" is one FORWARD_STEP of the device-resident hot path (DYNAMICS ->
SOLVE_FOR_PRESSURE/CG2D -> MOMENTUM_CORRECTION_STEP -> INTEGR_CONTINUITY ->
blocking exchanges) on inputs already resident in HBM.  Rank 0 prints ONE JSON
line.  `value` is BASELINE config 2 (90x40x15, one tile): at N>1 (one process per
GPU, torch.distributed.run) every rank runs an independent replica ("replicas
only") and value = the sum over ranks.

Fields of the JSON line beyond the driver contract:
  roofline     dominant kernel (the whole-solve CG2D): bound "latency" -- the f64
               VALU issue of the CU(s) it runs on plus per-iteration barriers;
               us_per_iteration, the VALU floor and, for completeness, its
               algorithmic bytes (136 B per point per iteration)
               over its mean HIP-event duration against the 8 TB/s HBM peak
  roofline_hbm the DYNAMICS momentum kernel(s) against the HBM roofline
               (SURVEY.md 8(d) algorithmic bytes per 3-D point)
  cs32x15      N=1: BASELINE config 3 (the other half of the metric), resident,
               the same steps/warmup, with its own rooflines
  sharded      N>1: the tile-sharded path -- cs32x15 over min(N,6) ranks and the
               LLC-90 synthetic over N ranks (RCCL subgroups, graph-replayed), each
               with the resident 1-GPU ms/step beside it and the CG2D placement
               chosen by parallel.cg2d_policy
  cpu_baseline the oracle (oracle/, C restatement, 1 core) on a bounded sample
               of the same workload, rank 0 only
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CG2D_BYTES_PER_POINT_ITER = 136  # two-sync-point minimum traffic
# CG2D arithmetic per interior point and iteration (cg2d.F:211-352 as the device runs it, unfused):
# A.s and M.r (5 mul + 4 add each), s, x, r updates (2 each), three dot products (2 each)
CG2D_F64_OPS_PER_POINT_ITER = 9 + 9 + 2 + 2 + 2 + 6
# one CU's f64 VALU issue rate: 4 SIMDs x 16 lanes per clock (a wave64 f64 op takes 4 cycles)
CU_F64_LANE_OPS_PER_CLK = 64
CLOCK_GHZ = 2.4                # MI355X peak engine clock (s_memtime/s_memrealtime: 2.40 GHz measured)
MOM_BYTES_PER_POINT = {15: 116.8, 50: 107.8}   # fused momentum, algorithmic
PMC_TAG = {"global_ocean.90x40x15": "ocean90", "global_ocean.cs32x15": "cs32x15", "llc90_synthetic": "llc90"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="N > 1: one process per GPU; launched under torch.distributed.run (WORLD_SIZE set) or, "
                         "without a launcher, bench.py starts the N ranks itself (spawn_ranks)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="global_ocean.90x40x15",
                    choices=["global_ocean.90x40x15", "global_ocean.cs32x15", "llc90_synthetic", "global_oce_latlon_90x40x15", "tutorial_global_oce_latlon", "baroclinic_gyre_dst3",
                             "tutorial_baroclinic_gyre", "tutorial_barotropic_gyre"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", action="store_true",
                    help="N>1: shard the workload's tiles over the N processes (RCCL, strong scaling, "
                         "mitgcm_amd/parallel.py) instead of running N replicas")
    ap.add_argument("--cg2d", choices=["auto", "replicated", "distributed", "device"], default="auto",
                    help="sharded runs (--shard, and the N > 1 sharded records): auto (default: "
                         "parallel.cg2d_policy's cost model -- one process keeps its resident solve; across "
                         "GPUs a single-CU kernel is always replicated, and the multi-workgroup solve is "
                         "replicated unless a 1/N share of its per-iteration work outweighs two fabric "
                         "hand-offs, which is the case for none of the BASELINE configs), CG2D replicated on "
                         "every GPU, the reference's distributed CG2D with GLOBAL_SUM_TILE_RL over the "
                         "collective, or the device CG2D whose parts run in every process on one IPC-shared "
                         "hand-off block (mitgcm_amd/parallel.py)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cs32", action="store_true", help="N = 1: skip the cs32x15 sub-record")
    ap.add_argument("--no-sharded", action="store_true", help="N > 1: skip the sharded cs32x15 / LLC-90 records")
    ap.add_argument("--sharded-timeout", type=float, default=300.0,
                    help="N > 1: seconds the sharded records may take before the line is printed without them")
    ap.add_argument("--set", action="append", default=[], metavar="NAME=VALUE",
                    help="override a namelist parameter of the GPU model (A/B runs, e.g. useSRCGSolver=1); "
                         "recorded in config.params_over")
    ap.add_argument("--pmc-summary", default=None,
                    help="tools/pmc_summary.py output of rocprofv3 --pmc passes of this command (roofline.traffic); "
                         "default profiles/r02/<config tag>/pmc_summary.json")
    return ap.parse_args()


WORKLOADS = {
    "global_ocean.90x40x15": "BASELINE config 2, verification/global_ocean.90x40x15 as verified: 90x40x15 "
                             "global lat-lon ocean, 1 tile of 90x40 (OL=3) on 1 GPU, restarted from the committed "
                             "pickup at nIter0=36000; r* coordinate with non-linear free surface (UPDATE_CG2D "
                             "every step), JMD95P, GM/Redi gkw91, CD scheme, biharmonic + harmonic viscosity, "
                             "quasi-hydrostatic + NH metric + 3-D Coriolis, implicit vertical diffusion, IVDC, "
                             "monthly forcing with real fresh-water flux; full FORWARD_STEP on device, "
                             "1 step = 1 model day",
    "global_ocean.cs32x15": "BASELINE config 3, verification/global_ocean.cs32x15: cubed sphere, 6 faces of "
                            "32x32 as 6 tiles (OL=4, pkg/exch2 halo maps) on 1 GPU, 15 levels, cold start from "
                            "lev_T/S_cs_15k; staggerTimeStep, vector-invariant momentum (harmonic viscosity), r* with "
                            "non-linear free surface (UPDATE_CG2D every step), JMD95Z, GM/Redi advective form "
                            "(GM_AdvForm), implicit vertical diffusion, IVDC, monthly forcing with real fresh-water "
                            "flux; full FORWARD_STEP on device, 1 step = 1 model day",
    "llc90_synthetic": "BASELINE config 5, the LLC-90-shaped synthetic of SURVEY.md 8(d): the 5 lat-lon-cap "
                       "facets of data.exch2.llc_120_5f at n=90 (13 tiles of 90x90, OL=4, pkg/exch2 maps), 50 "
                       "levels, uniform 100 km metrics, f-plane, cos-shaped bathymetry; vector-invariant momentum, "
                       "linear free surface + exactConserv, LINEAR EOS, C2 tracers, implicit vertical diffusion, "
                       "IVDC, zonal wind; multi-workgroup CG2D; full FORWARD_STEP on device, dt = 3600 s "
                       "(1 step = 1/24 model day)",
    "global_oce_latlon_90x40x15": "90x40x15 global lat-lon ocean (BASELINE config 2's grid, bathymetry, "
                                  "monthly forcing and 1-tile layout sNx=90, sNy=40, OL=3) with the physics "
                                  "verification/tutorial_global_oce_latlon pins: JMD95Z, GM/Redi gkw91, CD scheme, "
                                  "SST/SSS relaxation, Qnet, real fresh-water flux, IVDC, implicit diffusion, "
                                  "linear free surface (config 2 adds r*, JMD95P, biharmonic viscosity: not yet); "
                                  "full FORWARD_STEP on device, 1 step = 1 model day",
    "tutorial_global_oce_latlon": "tutorial_global_oce_latlon 90x40x15 as verified (2 tiles of 45x40, OL=2), "
                                  "full FORWARD_STEP on device, 1 step = 1 model day",
    "baroclinic_gyre_dst3": "BASELINE config 4: tutorial_baroclinic_gyre 62x62x15 (4 tiles of 31x31, "
                            "spherical-polar) with tempAdvScheme=33 (multi-dim DST3 flux-limited), full FORWARD_STEP "
                            "on device (dt=1200 s)",
    "tutorial_baroclinic_gyre": "tutorial_baroclinic_gyre 62x62x15 (4 tiles of 31x31, spherical-polar), "
                                "full FORWARD_STEP on device incl. THERMODYNAMICS (dt=1200 s)",
    "tutorial_barotropic_gyre": "tutorial_barotropic_gyre 62x62x1, 1 tile, full FORWARD_STEP on device (dt=1200 s)",
}


DATA = {
    "llc90_synthetic": "synthetic (SURVEY.md 8(d) C5 recipe): cos-shaped bathymetry, T = tRef + 0.01 N(0,1), "
                       "S = 35 + 0.001 N(0,1) from numpy default_rng(20261015), zonal wind -0.1 cos(2 pi y/L_y)",
    "global_ocean.cs32x15": "reference input fields of verification/global_ocean.cs32x15 (grid_cs32 facets, "
                            "bathy_Hmin50, lev_T/S_cs_15k, 12-month taux/tauy/Qnet/EmPmR/SST/SSS), cold start",
    "global_ocean.90x40x15": "reference input fields of verification/tutorial_global_oce_latlon (bathymetry, "
                             "12-month taux/tauy/Qnet/EmPmR/SST/SSS) and the committed pickup.0000036000 / "
                             "pickup_cd.0000036000 of verification/global_ocean.90x40x15",
    "global_oce_latlon_90x40x15": "reference input fields of verification/tutorial_global_oce_latlon (bathymetry, "
                                  "lev_t/lev_s record 1, 12-month taux/tauy/Qnet/EmPmR/SST/SSS), cold start",
    "tutorial_global_oce_latlon": "reference input fields of verification/tutorial_global_oce_latlon (bathymetry, "
                                  "lev_t/lev_s record 1, 12-month taux/tauy/Qnet/EmPmR/SST/SSS), cold start",
    "tutorial_barotropic_gyre": "reference input fields of verification/tutorial_barotropic_gyre (bathy, wind), "
                                "cold start",
}


def _overlap_info(m):
    from mitgcm_amd._lib import lib
    g = lambda n: lib().mgcm_get_param(m.h, n)
    return {"on": int(g(b"overlap")), "trial_ms_on": round(g(b"ovlMsOn"), 4), "trial_ms_off": round(g(b"ovlMsOff"), 4)}


def config_fn(name):
    """The mitgcm_amd.configs set-up behind a --config name."""
    from mitgcm_amd import configs
    if name == "baroclinic_gyre_dst3":
        return lambda: configs.baroclinic_gyre(tempAdvScheme=33)
    if name == "global_ocean.90x40x15":
        return configs.global_ocean_90x40x15
    if name == "global_ocean.cs32x15":
        return configs.global_ocean_cs32x15
    if name == "llc90_synthetic":
        return configs.llc_synthetic
    if name == "global_oce_latlon_90x40x15":
        return lambda: configs.global_oce_latlon(nSx=1, nSy=1, OL=3)
    if name == "tutorial_global_oce_latlon":
        return configs.global_oce_latlon
    return {"tutorial_baroclinic_gyre": configs.baroclinic_gyre,
            "tutorial_barotropic_gyre": configs.barotropic_gyre}[name]


def _host_cpu():
    """(model name, cores this process may use, the host's visible CPUs, its physical cores):
    the usable count is the affinity set capped by OMP_NUM_THREADS (16 on the GPU box, whose
    os.cpu_count() reports the whole machine); physical cores are the distinct (package, core)
    pairs of /proc/cpuinfo."""
    model = "unknown"
    phys = set()
    pkg = core = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name") and model == "unknown":
                model = ln.split(":", 1)[1].strip()
            elif ln.startswith("physical id"):
                pkg = ln.split(":", 1)[1].strip()
            elif ln.startswith("core id"):
                core = ln.split(":", 1)[1].strip()
            elif not ln.strip():
                if core is not None:
                    phys.add((pkg, core))
                pkg = core = None
    except OSError:
        pass
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    n = visible
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return model, max(1, n), visible, (len(phys) or None)


def _oracle_for(config, omp=False, **kw):
    from oracle import harness
    from oracle.harness import cs32x15_oracle, gyre_oracle, latlon_oracle, ocean90_oracle, oracle_from_config
    harness.USE_OMP = omp
    try:
        if config == "global_ocean.90x40x15":
            return ocean90_oracle(**kw)[0]
        if config == "global_ocean.cs32x15":
            return cs32x15_oracle(**kw)[0]
        if config == "llc90_synthetic":
            return oracle_from_config(config_fn(config), **kw)[0]
        if config == "tutorial_barotropic_gyre":
            return gyre_oracle()
        if config == "global_oce_latlon_90x40x15":
            return latlon_oracle(nSx=1, nSy=1, OL=3)[0]
        if config == "tutorial_global_oce_latlon":
            return latlon_oracle()[0]
        return oracle_from_config(config_fn(config))[0]
    finally:
        harness.USE_OMP = False


def _time_oracle(o, seconds):
    o.forward_step()  # warm
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.forward_step()
        n += 1
    return n, time.perf_counter() - t0


# tilings of each workload the multi-core baseline tries (the tile loops go over the threads;
# smaller tiles give more parallel work but more halo-extended work per owned point): the
# benched one-tile layout, the reference's own MPI decomposition where it has one (config 2's
# code/SIZE.h: 9 x 4 tiles of 10 x 10) and layouts between
CPU_TILINGS = {
    "global_ocean.90x40x15": [{}, {"nSx": 3, "nSy": 2}, {"nSx": 6, "nSy": 2}, {"nSx": 3, "nSy": 4},
                              {"nSx": 9, "nSy": 4}],
    "global_ocean.cs32x15": [{}, {"sNy": 16}],
    "llc90_synthetic": [{}, {"tile": 45}],
}


def _rate(n, dt, dt_clock):
    return n * dt_clock / 86400.0 / dt


def cpu_baseline(config, seconds):
    """The oracle (CPU restatement) timed on the same workload: as many steps as fit in
    ~`seconds`, in model-days/s.  `value`: one core on the benched tiling (the sequential
    build).  `all_cores`: the OpenMP build (every tile loop, the CG2D's included, and the halo
    exchanges over the threads; tile partials summed in tile order, bit-identical to one
    thread) on every core this process may use, on the fastest of CPU_TILINGS after a short
    trial of each (the trial rates are in the record)."""
    o = _oracle_for(config)
    dt_clock = o.get("deltaTClock")
    n, dt = _time_oracle(o, seconds)
    del o
    cpu, cores, visible, physical = _host_cpu()
    out = {"value": _rate(n, dt, dt_clock), "unit": "model-days/s", "cores": 1, "kind": "port",
           "sample": "%d FORWARD_STEPs of %s on the oracle (oracle/*.c, gcc -O2, 1 thread), %.1f s"
                     % (n, config, dt), "cpu_model": cpu, "host_cpus_visible": visible,
           "host_physical_cores": physical}
    if cores > 1:
        trial = max(1.0, seconds / 8.0)
        tried = {}
        best = None
        for til in CPU_TILINGS.get(config, [{}]):
            o = _oracle_for(config, omp=True, **til)
            o.set(nThreads=cores)
            r = _rate(*_time_oracle(o, trial), dt_clock)
            del o
            name = ",".join("%s=%s" % kv for kv in sorted(til.items())) or "benched"
            tried[name] = r
            if best is None or r > best[0]:
                best = (r, til, name)
        o = _oracle_for(config, omp=True, **best[1])
        o.set(nThreads=cores)
        n2, dt2 = _time_oracle(o, seconds)
        del o
        out["all_cores"] = {"value": _rate(n2, dt2, dt_clock), "unit": "model-days/s", "cores": cores,
                            "kind": "port", "tiling": best[2], "tilings_tried": tried,
                            "sample": "%d FORWARD_STEPs of %s on the OpenMP oracle build (%s tiling, %d threads), "
                                      "%.1f s" % (n2, config, best[2], cores, dt2)}
    return out


def pmc_traffic(path, kernel_keys):
    """HBM bytes per launch from the committed PMC passes (FETCH_SIZE x2 + WRITE_SIZE,
    tools/pmc_summary.py), summed over every kernel whose name contains one of
    `kernel_keys` (the launches of one timed block); (total, {kernel: bytes}) or
    (None, {}) when absent."""
    try:
        import json as _j
        ks = _j.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return None, {}
    if isinstance(kernel_keys, str):
        kernel_keys = (kernel_keys,)
    per = {k: v["hbm_bytes_per_launch"] for k, v in ks.items() if any(key in k for key in kernel_keys)}
    return (sum(per.values()) if per else None), per


def default_pmc_summary(config):
    """The newest committed PMC summary of this workload (profiles/r0N/<tag>_final/, then
    profiles/r0N/<tag>/)."""
    tag = PMC_TAG.get(config, config)
    for rnd in ("r06", "r05", "r04", "r03", "r02"):
        for sub in (tag + "_final", tag):
            p = os.path.join(ROOT, "profiles", rnd, sub, "pmc_summary.json")
            if os.path.exists(p):
                return p
    return os.path.join(ROOT, "profiles", "r06", tag, "pmc_summary.json")


def device_free_bytes(device):
    """hipMemGetInfo's free bytes of the device (None where the HIP runtime is not loadable)."""
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        free, total = ctypes.c_size_t(), ctypes.c_size_t()
        if hip.hipSetDevice(device) != 0 or hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) != 0:
            return None
        return free.value
    except OSError:
        return None


def stream_triad_gbs(device, n=64 << 20, reps=8):
    """SURVEY.md 8(d)'s roofline denominator measured on the box: a STREAM triad
    a = b + s*c over three fp64 arrays of n doubles (512 MB each at the default), 16 B per
    lane, best of `reps` (mgcm_stream_triad), in GB/s -- run after the timed region, a
    reference rate for the fractions."""
    import ctypes
    from mitgcm_amd._lib import check, lib
    g = ctypes.c_double()
    check(lib().mgcm_stream_triad(device, n, reps, ctypes.byref(g)), "mgcm_stream_triad")
    return g.value


def cg_kernel_key(m):
    return "k_cg2d_" + m.cg2d_kernel().replace("_ref", "")


def attribution(m, stepper, steps, config, pmc_summary, sync):
    """Per-kernel attribution of the timed workload: the same `steps` again, launched eagerly
    with HIP events recorded on the model's stream around every kernel (the graph path cannot
    be bracketed by events; rocprofv3 of the command must agree, profiles/), then the two
    roofline objects -- the dominant kernel (the whole-solve CG2D, latency-bound) and the
    DYNAMICS momentum block against the HBM roofline (SURVEY.md 8(d) algorithmic bytes)."""
    g = m.g
    npts = g.nTiles * g.sNx * g.sNy
    m.kernel_timing(True)
    stepper.forward_step(steps)
    sync()
    iters_t = [int(v) for v in m.solve_history(steps)[0]]
    cg_ms, cg_n = m.kernel_ms("cg2d")
    kern = {k: m.kernel_ms(k) for k in ("oceanic_phys", "temp_step", "phi_hyd", "mom_step", "sfp_rhs", "cg2d", "exchange",
                                         "eta_update", "correction", "continuity", "r_star")}
    m.kernel_timing(False)
    cg_traffic, _ = pmc_traffic(pmc_summary, cg_kernel_key(m))
    # the momentum block's launches as the timed graph runs them: on small grids with
    # THERMODYNAMICS folded into DYNAMICS' grids (config 2) the three fused grids k_dt_l1/l2/l3
    # (GM tensor | CALC_PHI_HYD | del2uv, MOM U | V | tracer right-hand sides, CD scheme |
    # implicit tracer solves); otherwise launch_mom_step's (del2uv, the MOM_FLUXFORM /
    # MOM_VECINV kernel, the VI halo AB pass, the CD scheme, the implicit viscosity columns)
    layout = m.step_layout()
    dt_fused = layout["dyn_thermo_fused"]
    mom_kernels = ("k_dt_l",) if dt_fused else ("k_del2uv", "k_mom_", "k_cd_scheme")
    mom_traffic, mom_traffic_per = pmc_traffic(pmc_summary, mom_kernels)
    its_per_solve = sum(iters_t) / max(1, len(iters_t))
    bytes_per_launch = CG2D_BYTES_PER_POINT_ITER * npts * its_per_solve
    achieved = bytes_per_launch / (cg_ms * 1e-3) / 1e9 if cg_ms > 0 else 0.0
    us_per_it = 1e3 * cg_ms / its_per_solve if its_per_solve > 0 else 0.0
    cus = int(m.cg2d_parts())
    # the f64 VALU bound of the CUs the solve runs on (one workgroup per CU)
    valu_us = CG2D_F64_OPS_PER_POINT_ITER * npts / (CU_F64_LANE_OPS_PER_CLK * cus * CLOCK_GHZ * 1e3)
    mom_ms = kern["mom_step"][0]
    mom_bpp = MOM_BYTES_PER_POINT.get(g.Nr, 104.0 + 24 * 8.0 / g.Nr)
    mom_bytes = mom_bpp * npts * g.Nr
    if dt_fused:   # + the stepped tracers' right-hand sides and solves (64 B + 96/Nr B a point)
        ntr = int(m.params.get("tempStepping", 1) != 0) + int(m.params.get("saltStepping", 1) != 0)
        mom_bytes += ntr * (64.0 + 96.0 / g.Nr) * npts * g.Nr
    mom_gbs = mom_bytes / (mom_ms * 1e-3) / 1e9 if mom_ms > 0 else 0.0
    # dominant kernel: the whole-solve CG2D.  It is not HBM-bound: its working set sits in
    # LDS/VGPRs of the workgroup(s) it runs on, so the chip-level HBM fraction is reported for
    # completeness; the bound that holds it is latency -- the f64 VALU issue of its CU(s) plus
    # the barriers/cross-wave sums (one CU) or grid hand-offs (many) of each iteration
    # (valu_floor_us_per_iter, profiles/r02/ocean90/cg2d_geometry.txt)
    roofline = {"bound": "latency", "kernel": "k_cg2d_" + m.cg2d_kernel(), "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": cg_traffic,
                "traffic_unit": "bytes per launch (rocprofv3 --pmc, %s)" % os.path.relpath(pmc_summary, ROOT),
                "bytes_per_launch": bytes_per_launch, "launch_ms": cg_ms, "launches": cg_n,
                "us_per_iteration": us_per_it, "cus_used": cus,
                "valu_floor_us_per_iter": valu_us,
                "valu_frac": valu_us / us_per_it if us_per_it > 0 else 0.0}
    roofline_hbm = {"bound": "hbm",
                    "kernel": ("fused DYNAMICS + THERMODYNAMICS grids k_dt_l1/l2/l3 (the launches the timed graph "
                               "runs; bytes: momentum + the stepped tracers)" if dt_fused else
                               "DYNAMICS momentum block (MOM_FLUXFORM/MOM_VECINV + TIMESTEP + AB2; "
                               "CALC_PHI_HYD timed apart as phi_hyd), streams serialised"),
                    "kernels": list(mom_kernels), "bytes_per_launch": mom_bytes,
                    "achieved": mom_gbs,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": mom_gbs / HBM_PEAK_GBS,
                    "bytes_per_point": mom_bpp, "launch_ms": mom_ms,
                    "traffic": mom_traffic,
                    "traffic_per_kernel": {k.split("(")[0]: v for k, v in mom_traffic_per.items()}}
    return iters_t, kern, layout, roofline, roofline_hbm


def check_iters(iters, what):
    """numIters = -1 marks a multi-workgroup CG2D that gave up (hand-off timeout): a graph
    batch would otherwise carry on silently."""
    failed = [i for i in iters if i < 0]
    if failed:
        raise SystemExit("bench: %s: %d of %d CG2D solves failed (numIters < 0): %s" % (what, len(failed), len(iters),
                                                                                         iters))


def resident_ms(config, steps, warmup, device):
    """ms/step of the resident (1-GPU, graph-replayed) path of a workload, and its model;
    the caller closes the model."""
    from mitgcm_amd import configs
    m = configs.make_model(config_fn(config), device=device)
    if warmup > 0:
        m.forward_step(warmup)
    m.sync()
    m.prepare()
    m.sync()
    t0 = time.perf_counter()
    m.forward_step(steps)
    m.sync()
    el = time.perf_counter() - t0
    iters = [int(v) for v in m.solve_history(steps)[0]]
    check_iters(iters, config)
    return m, 1e3 * el / steps, iters, el


def cs32x15_record(a, device):
    """BASELINE config 3 (the other half of BASELINE.json's metric) at N = 1: the resident
    graph-replayed step, `steps` timed after `warmup`, with its own attribution pass and
    rooflines.  Reported beside `value` (config 2), not instead of it."""
    cfg = "global_ocean.cs32x15"
    steps, warmup = max(2, a.steps), a.warmup
    m, ms, iters, el = resident_ms(cfg, steps, warmup, device)
    dt_clock = m.params["deltaTClock"]
    iters_t, kern, layout, roof, roof_hbm = attribution(m, m, steps, cfg, default_pmc_summary(cfg), m.sync)
    check_iters(iters_t, cfg)
    st = m.solve_stats()
    assert st["cg2d_last_res"] < 1e-6, st
    m.close()
    rec = {"config": cfg, "workload": WORKLOADS[cfg], "steps": steps, "warmup": warmup, "ms_per_step": ms,
           "value": steps * dt_clock / 86400.0 / el, "unit": "model-days/s",
           "cg2d_iters_per_s": sum(iters) / el, "cg2d_mean_iters_per_solve": sum(iters) / max(1, len(iters)),
           "kernel_ms_mean": {k: v[0] for k, v in kern.items()}, "roofline": roof, "roofline_hbm": roof_hbm}
    if not a.no_cpu_baseline:   # its own CPU baseline, half the headline's sample
        rec["cpu_baseline"] = cpu_baseline(cfg, max(2.0, a.cpu_seconds / 2))
    return rec


def sharded_records(a, dist, world, rank, local, backend):
    """N > 1: the tile-sharded path the north_star scales -- cs32x15 over min(N, 6) ranks (one
    cube face per GPU) and the LLC-90 synthetic over N ranks (13 tiles) -- each stepped by
    mitgcm_amd.parallel.ShardedModel over a subgroup (RCCL; gloo when MGCM_SHARD_BACKEND=gloo
    rehearses on one GPU), graph-replayed over RCCL, `steps` (rounded up to even) timed after
    `warmup`, max over the subgroup's ranks; beside each the same workload's resident 1-GPU
    ms/step (rank 0).  Strong scaling: the work is the whole workload at every N."""
    import torch
    from mitgcm_amd import configs
    from mitgcm_amd.parallel import ShardedModel
    steps = a.steps + (a.steps & 1)
    warm = max(2, a.warmup + (a.warmup & 1))
    out = []
    for cfg, n in (("global_ocean.cs32x15", min(world, 6)), ("llc90_synthetic", world)):
        rec = {"config": cfg, "ranks": n, "transport": "RCCL" if backend == "nccl" else "gloo (host-staged)"}
        sub = dist.new_group(list(range(n)), backend=backend)   # collective over every rank
        try:
            if rank == 0:
                m1, ms1, _, _ = resident_ms(cfg, steps, warm, local)
                m1.close()
                rec["resident_1gpu_ms_per_step"] = ms1
            if rank < n:
                m = configs.make_model(config_fn(cfg), device=local)
                sm = ShardedModel(m, dist, cg2d=a.cg2d, group=sub)
                graph = backend == "nccl"
                if graph:
                    sm.capture_step()
                    sm.replay(warm // 2)
                else:
                    sm.forward_step(warm)
                m.sync()
                torch.cuda.synchronize(local)
                sm.dist.barrier()
                t0 = time.perf_counter()
                if graph:
                    sm.replay(steps // 2, check=False)
                else:
                    sm.forward_step(steps, check=False)
                m.sync()
                torch.cuda.synchronize(local)
                el = time.perf_counter() - t0
                sm.dist.barrier()
                t = torch.tensor([el], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
                sm.dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = float(t.item())
                iters = [int(v) for v in m.solve_history(steps)[0]]
                check_iters(iters, cfg + " sharded")
                dt_clock = m.params["deltaTClock"]
                rec.update({"ms_per_step": 1e3 * el / steps, "value": steps * dt_clock / 86400.0 / el,
                            "unit": "model-days/s", "steps": steps, "warmup": warm,
                            "tiles_per_rank": sm.part.counts, "cg2d": sm.cg2d, "cg2d_policy": sm.cg2d_reason,
                            "step_path": "graph-replayed (collectives captured)" if graph else "eager",
                            "cg2d_mean_iters_per_solve": sum(iters) / max(1, len(iters))})
                if "resident_1gpu_ms_per_step" in rec:
                    rec["speedup_vs_resident_1gpu"] = rec["resident_1gpu_ms_per_step"] / rec["ms_per_step"]
                m.close()
        except Exception as e:   # reported in the record; the headline line stands
            rec["error"] = "%s: %s" % (type(e).__name__, e)
            print("bench: sharded %s failed on rank %d: %r" % (cfg, rank, e), file=sys.stderr)
        dist.barrier()
        out.append(rec)
    return out


def spawn_ranks(n, argv, script=None):
    """`--gpus N` (N > 1) without a launcher: start N fresh worker processes of this same
    command, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set the way
    torch.distributed.run sets them (127.0.0.1, a free port), and exit with the first failing
    rank's status.  The parent has touched no GPU (nothing above imports torch), so the workers
    are plain children, not an exec of a GPU process.  Rank 0's stdout (the one JSON line) is
    the parent's; the other ranks print nothing there."""
    import signal
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                c = p.poll()
                if c is None:
                    continue
                pending.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print("bench: rank %d exited with %d; stopping the others" % (procs.index(p), c), file=sys.stderr)
                    for q in pending:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in procs:
            p.send_signal(signal.SIGTERM)
        raise
    return rc


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    if a.gpus != int(os.environ.get("WORLD_SIZE", "1")):
        raise SystemExit("bench: --gpus %d but WORLD_SIZE=%s: launch one process per GPU (or give --gpus alone)"
                         % (a.gpus, os.environ.get("WORLD_SIZE", "1")))
    # stdout carries ONE JSON line: whatever libraries print (RCCL's version banner at
    # communicator creation, ...) goes to stderr
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # --shard at N = 1 runs the sharded driver over a one-rank RCCL group: its per-step
    # overhead against the resident graph is then measured on one GPU
    shard = a.shard
    if shard and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            sk.close()
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    # MGCM_SHARD_BACKEND=gloo: host-staged transport, lets several ranks share one GPU
    # (rehearsal on a 1-GPU box; RCCL refuses two ranks per device)
    shard_backend = os.environ.get("MGCM_SHARD_BACKEND", "nccl")
    sharded_rec = world > 1 and not shard and not a.no_sharded
    if world > 1 or shard:
        import torch
        import torch.distributed as dist
        if shard_backend == "gloo":
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if shard:
            if shard_backend == "gloo":
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))   # RCCL over xGMI
        else:
            dist.init_process_group("gloo")   # replicas: barrier + max-reduce of host timers only
    # the GPUs the job's ranks actually run on (a gloo rehearsal puts several ranks on one)
    devices_used = 1
    if world > 1:
        devs = [None] * world
        dist.all_gather_object(devs, "%s:%d" % (os.uname()[1], local))
        devices_used = len(set(devs))
    # the sharded records run after the headline; a hang there (a collective a failed rank never
    # joins) must not cost the line: past the deadline rank 0 prints what it has and every
    # rank leaves
    emitted = {"done": False}
    out = {}

    def emit():
        if rank == 0 and not emitted["done"]:
            emitted["done"] = True
            sys.stdout.flush()
            os.write(json_fd, (json.dumps(out) + "\n").encode())

    import numpy as np
    from mitgcm_amd import configs

    over = {}
    for kv in a.set:
        k, v = kv.split("=", 1)
        over[k] = float(v)
    cfn = config_fn(a.config)
    if shard and a.cg2d == "device":
        over.setdefault("cg2dForceMwg", 1.0)   # the device CG2D runs the multi-workgroup solver's parts
    if over:
        cfn = (lambda f: lambda: (lambda r: (r[0], {**r[1], **over}) + tuple(r[2:]))(f()))(cfn)
    free0 = device_free_bytes(local)
    m = configs.make_model(cfn, device=local)
    g = m.g
    # the model's device footprint (the whole domain on every GPU): free HBM before
    # and after building it
    free1 = device_free_bytes(local)
    model_gb = (free0 - free1) / 1e9 if free0 is not None and free1 is not None else None
    dt_clock = m.params["deltaTClock"]
    stepper = m
    if shard:
        from mitgcm_amd.parallel import ShardedModel
        stepper = ShardedModel(m, dist, cg2d=a.cg2d)

    def sync():
        m.sync()
        if shard:
            torch.cuda.synchronize(local)

    # the sharded step over RCCL with the replicated solve is graph-captured (two steps per
    # graph, collectives included: ShardedModel.capture_step) and replayed, as the resident
    # path is; gloo and the host-driven distributed CG2D step eagerly
    graph_shard = shard and dist.get_backend() == "nccl" and stepper.cg2d != "distributed"
    if graph_shard and a.steps % 2:
        raise SystemExit("bench: --shard over RCCL replays pairs of steps: --steps must be even")

    # warmup (untimed)
    if graph_shard:
        stepper.capture_step()            # one eager step, then the capture
        stepper.replay(max(1, a.warmup // 2))
    elif a.warmup > 0:
        stepper.forward_step(a.warmup)
    sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    if not shard:
        m.prepare()
    # timed region: K steps replayed from hipGraphs (kernel timing off)
    barrier()
    sync()
    t0 = time.perf_counter()
    if graph_shard:
        stepper.replay(a.steps // 2)
    else:
        stepper.forward_step(a.steps)
    sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cuda" if shard and dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    iters = [int(v) for v in m.solve_history(a.steps)[0]]
    if a.pmc_summary is None:
        a.pmc_summary = default_pmc_summary(a.config)
    iters_t, kern, layout, roofline, roofline_hbm = attribution(m, stepper, a.steps, a.config, a.pmc_summary, sync)
    # sanity: the solution is finite and the solver converged every step
    stats = m.solve_stats()
    eta = m.get("etaN")
    assert np.isfinite(eta).all() and stats["cg2d_last_res"] < 1e-6, stats
    # every solve of both batches converged without a hand-off timeout
    check_iters(iters + iters_t, a.config)
    model_days = a.steps * dt_clock / 86400.0
    copies = 1 if shard else world   # independent model integrations in the job
    value = copies * model_days / elapsed
    iters_total = sum(iters)
    cg2d_iters_per_s = copies * iters_total / elapsed
    out.update({
        "metric": "model-days/wallclock-sec",
        "value": value,
        # replica mode: value sums the N independent integrations; one integration's rate
        "value_per_integration": model_days / elapsed,
        "unit": "model-days/s",
        "n_gpus": world,
        "ranks": world,
        "distinct_gpus": devices_used,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * elapsed / a.steps,
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": DATA.get(a.config, "reference input fields of verification/tutorial_baroclinic_gyre (bathy, wind, "
                                   "SST_relax), cold start"),
        "config": {"workload": WORKLOADS[a.config] + ("; tiles sharded over %d processes (%s)" % (
                                                           world, "RCCL" if dist.get_backend() == "nccl" else
                                                           "gloo, host-staged") if shard
                                                       else "; replicas only"),
                   "tiles_per_gpu": stepper.nT if shard else g.nTiles, "points_per_tile": [g.sNx, g.sNy, g.Nr],
                   "parallelism": ("tiles%d" if shard else "replicas%d") % world,
                   "cg2d": stepper.cg2d if shard else "single-GPU kernel",
                   **({"step_path": "graph-replayed sharded step (RCCL collectives captured)" if graph_shard
                       else "eager sharded step"} if shard else {}),
                   **({"params_over": over} if over else {})},
        "cg2d_iters_per_s": cg2d_iters_per_s,
        "device_model_gb": model_gb,
        # THERMODYNAMICS on a second stream beside DYNAMICS: picked per workload by timing both
        # graphs over the first 20 graph-replayed steps (results identical either way)
        "thermo_overlap": _overlap_info(m),
        "cg2d_mean_iters_per_solve": iters_total / max(1, len(iters)),
        "kernel_ms_mean": {k: v[0] for k, v in kern.items()},
        # those times: an eager pass of the same steps with events around every launch, in the
        # launch layout the timed graph replays (one stream: a second-stream THERMODYNAMICS,
        # C5's, is serialised there); with the fused grids "mom_step" is k_dt_l1+l2+l3
        "kernel_ms_layout": {"eager_pass_of_the_graph_layout": True, **layout},
        "roofline": roofline,
        "roofline_hbm": roofline_hbm,
    })
    m.close()
    # the measured STREAM triad of this box beside the 8 TB/s spec
    try:
        triad = stream_triad_gbs(local)
        out["roofline_hbm"]["stream_triad_gbs"] = triad
        out["roofline_hbm"]["frac_of_triad"] = out["roofline_hbm"]["achieved"] / triad
    except Exception as e:   # a reference number only: its absence does not fail the bench
        out["roofline_hbm"]["stream_triad_gbs"] = None
        print("bench: stream triad not measured: %s" % e, file=sys.stderr)
    if rank == 0 and world == 1 and not shard and a.config != "global_ocean.cs32x15" and not a.no_cs32:
        # the other half of BASELINE.json's metric, timed in the same run
        out["cs32x15"] = cs32x15_record(a, local)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:   # the CPU baseline is an N=1 line
        out["cpu_baseline"] = cpu_baseline(a.config, a.cpu_seconds)
    if sharded_rec:
        import threading
        out["sharded"] = [{"error": "not finished within %d s" % a.sharded_timeout}]

        def deadline():
            emit()
            os._exit(0)
        timer = threading.Timer(a.sharded_timeout, deadline)
        timer.daemon = True
        timer.start()
        out["sharded"] = sharded_records(a, dist, world, rank, local, shard_backend)
        timer.cancel()
    emit()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
