"""Tile-sharded device path (mitgcm_amd/parallel.py + the C-ABI phase API) on a
real MI355X: 2 to 6 processes share cuda:0 over gloo (host-staged transport;
RCCL refuses two ranks on one GPU) and step
  * BASELINE config 4 (baroclinic gyre, 4 lat-lon tiles) for 6 steps,
  * BASELINE config 3 (global_ocean.cs32x15: 6 cube faces, pkg/exch2 vector maps and
    corners, r* with UPDATE_CG2D, staggerTimeStep, GM_AdvForm) for 4 steps, and
  * BASELINE config 5's LLC topology (13 tiles on 5 facets) at n = 30 for 4 steps, with
    the tracers' halo exchange overlapping DYNAMICS and the solve;
every process's tiles must be bit-identical to a single-process run (SURVEY.md 8(c)
parity item 6: same results at any GPU count)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("uVel", "vVel", "wVel", "theta", "salt", "etaN", "etaH")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# option variants of the solver: cfg + "_minres" keeps the lowest-residual solution
# (cg2dUseMinResSol, 8 iterations at most so that the solve stops above its minimum),
# cfg + "_sr" solves with CG2D_SR (useSRCGSolver)
SOLVER_VARIANTS = {"minres": {"cg2dUseMinResSol": 1, "cg2dMaxIters": 8}, "sr": {"useSRCGSolver": 1}}


def _make(cfg, force_mwg=False):
    from mitgcm_amd import configs
    over = {}
    for v, o in SOLVER_VARIANTS.items():
        if cfg.endswith("_" + v):
            cfg, over = cfg[:-len(v) - 1], o
    if cfg == "gyre":
        fn = lambda: configs.baroclinic_gyre(tempAdvScheme=33)
    elif cfg == "llc30":   # BASELINE config 5's LLC topology at n = 30 (13 tiles, pkg/exch2 facets)
        fn = lambda: configs.llc_synthetic(n=30, Nr=10)
    elif cfg == "llc90":   # BASELINE config 5 at full size
        fn = configs.llc_synthetic
    else:
        fn = configs.global_ocean_cs32x15
    if force_mwg:   # the multi-workgroup CG2D also where a single-workgroup kernel would be chosen
        over = {**over, "cg2dForceMwg": 1}
    if over:
        fn = (lambda f: lambda: (lambda r: (r[0], {**r[1], **over}) + tuple(r[2:]))(f()))(fn)
    return configs.make_model(fn)


def _worker(rank, world, port, cfg, nsteps, q, cg2d="replicated", overlap="thermo", keep_full=True, pre_solve=False):
    import torch
    import torch.distributed as dist
    from mitgcm_amd.parallel import ShardedModel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        dev_cg = cg2d in ("device", "auto")
        m = _make(cfg, dev_cg)
        if pre_solve and rank == 0:
            # a multi-workgroup solve on this rank only before the block is shared: its launch
            # epoch advances and its granules stay in the block the others then map
            n = m.g.nTiles * m.g.ny * m.g.nx
            b = np.zeros(n)
            b[n // 2] = 1.0e-3
            m.cg2d(b, np.zeros(n), 5)
        sm = ShardedModel(m, dist, device=torch.device("cuda", 0), cg2d=cg2d, overlap=overlap)
        sm.forward_step(nsteps)
        m.sync()
        full = {n: sm.gather_field(n) for n in FIELDS}
        stats = [m.solve_stats(back=b) for b in range(nsteps)]
        minres = [m.solve_minres(back=b) for b in range(nsteps)]
        res = {"t0": sm.t0, "nT": sm.nT, "stats": stats, "minres": minres, "overlap": sm.overlap, "fork": sm.fork, "cg2d": sm.cg2d,
               "cg2d_reason": sm.cg2d_reason}
        if cg2d == "distributed":
            res["iters"] = list(sm.cg_iters)
        if cg2d in ("distributed", "device") and rank == 0 and keep_full:
            res["full"] = full
        if rank == 0:
            ref = _make(cfg, dev_cg)
            ref.forward_step(nsteps)
            ref.sync()
            res["diff"] = {n: float(np.max(np.abs(full[n] - ref.get(n)))) for n in FIELDS}
            res["equal"] = {n: bool(np.array_equal(full[n], ref.get(n))) for n in FIELDS}
            res["ref_stats"] = [ref.solve_stats(back=b) for b in range(nsteps)]
            res["ref_minres"] = [ref.solve_minres(back=b) for b in range(nsteps)]
            ref.close()
        m.close()
        q.put((rank, res))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg,world,nsteps,ntiles,overlap", [("gyre", 2, 6, 4, "thermo"), ("gyre", 4, 6, 4, "thermo"),
                                                             ("gyre", 2, 6, 4, "halo"), ("gyre", 2, 6, 4, False),
                                                             ("cs32x15", 2, 4, 6, "thermo"),
                                                             ("cs32x15", 4, 4, 6, "thermo"),
                                                             ("cs32x15", 6, 4, 6, "thermo"),
                                                             ("llc30", 2, 4, 13, "thermo"), ("llc30", 4, 4, 13, "thermo"),
                                                             ("llc30", 2, 4, 13, "halo")])
def test_sharded_bit_identical(cfg, world, nsteps, ntiles, overlap):
    """llc30: BASELINE config 5's 13-tile LLC topology (5 facets, rotated pkg/exch2 maps) at
    n = 30.  overlap (parallel.ShardedModel.step), non-staggered configurations: "thermo" runs
    THERMODYNAMICS on the model's second stream as the resident step does (mgcm_step_phase
    16), "halo" exchanges the tracers' halo sources while DYNAMICS, the solve and the
    continuity step run; the staggered cs32x15 keeps one stream and one exchange."""
    import torch.multiprocessing as mp
    from mitgcm_amd.parallel import TilePartition
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, nsteps, q, "replicated", overlap))
             for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0 = out[0]
    assert "error" not in r0, r0["error"]
    assert r0["overlap"] == (overlap == "halo" and cfg != "cs32x15"), r0["overlap"]
    assert r0["fork"] == (overlap == "thermo" and cfg != "cs32x15"), r0["fork"]
    print("%s sharded x%d (overlap %s) max |diff| vs 1 process:" % (cfg, world, overlap), r0["diff"])
    assert all(r0["equal"].values()), r0["diff"]
    for rank, r in out.items():
        assert r["stats"] == r0["ref_stats"], "rank %d: CG2D records differ" % rank
    part = TilePartition(ntiles, world)
    assert sorted((r["t0"], r["nT"]) for r in out.values()) == [part.range(r) for r in range(world)]


def _spawn(cfg, world, nsteps, cg2d):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, nsteps, q, cg2d)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        rank, res = q.get(timeout=300)
        assert "error" not in res, "rank %d: %s" % (rank, res["error"])
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("cfg,worlds,nsteps", [("gyre", (1, 2, 4), 4), ("cs32x15", (1, 3, 6), 3),
                                               ("gyre_minres", (1, 2, 4), 3), ("cs32x15_sr", (1, 2, 3), 3)])
def test_distributed_cg2d(cfg, worlds, nsteps):
    """cg2d="distributed": the reference's CG2D over the processes' tiles, its global sums
    GLOBAL_SUM_TILE_RL (all-gather of per-tile partials, added in tile order); also with
    cg2dUseMinResSol (cg2d.F:148-155, 338-369) and with CG2D_SR (cg2d_sr.F).  Bars: the
    fields and every solve record identical bit for bit at every process count; against
    the replicated single-process solve (other summation order) the same iteration counts,
    the same lowest-residual iteration, and fields within 1e-10 of their maximum."""
    runs = {w: _spawn(cfg, w, nsteps, "distributed") for w in worlds}
    base = runs[worlds[0]][0]
    for w in worlds[1:]:
        r0 = runs[w][0]
        for n in FIELDS:
            assert np.array_equal(r0["full"][n], base["full"][n]), (w, n, np.abs(r0["full"][n] - base["full"][n]).max())
        for rank, r in runs[w].items():
            assert r["stats"] == base["stats"], (w, rank)
            assert r["iters"] == base["iters"], (w, rank)
            assert r["minres"] == base["minres"], (w, rank)
    its_rep = [s["cg2d_iters"] for s in base["ref_stats"]]
    assert [n for _, n in base["minres"]] == [n for _, n in base["ref_minres"]], (base["minres"], base["ref_minres"])
    if cfg.endswith("_minres"):
        assert all(n >= 0 for _, n in base["minres"]), base["minres"]
    its_dist = [s["cg2d_iters"] for s in base["stats"]]
    print("%s distributed CG2D iterations %s (replicated %s); max |diff| vs replicated %s" % (
        cfg, its_dist, its_rep, base["diff"]))
    assert its_dist == its_rep
    for n in FIELDS:
        sc = max(np.abs(base["full"][n]).max(), 1e-300)
        assert base["diff"][n] <= 1e-10 * sc, (n, base["diff"][n], sc)


@pytest.mark.parametrize("cfg,worlds,nsteps", [("cs32x15", (1, 2, 3), 3), ("llc30", (1, 2, 4), 3),
                                               ("gyre", (1, 2, 4), 4)])
def test_device_cg2d_across_processes(cfg, worlds, nsteps):
    """cg2d="device": each process launches the multi-workgroup CG2D's parts of its own tiles,
    all meeting on rank 0's hand-off block mapped by IPC (system-scope granules); nothing on
    the host inside an iteration.  Bars: at every process count the fields and every solve
    record are bit-identical to the single-process model running the same multi-workgroup
    solver (its sums keep the single-launch order)."""
    for w in worlds:
        out = _spawn(cfg, w, nsteps, "device")
        r0 = out[0]
        its = [s["cg2d_iters"] for s in r0["stats"]]
        print("%s device CG2D x%d: iterations %s, max |diff| vs 1 process %s" % (cfg, w, its, r0["diff"]))
        assert all(r0["equal"].values()), (w, r0["diff"])
        for rank, r in out.items():
            assert r["stats"] == r0["ref_stats"], (w, rank, r["stats"], r0["ref_stats"])
        assert all(i > 0 for i in its), its


@pytest.mark.timeout(600)
@pytest.mark.parametrize("cg2d", ["replicated", "device"])
def test_llc90_eight_way_partition(cg2d):
    """BASELINE config 5 at full size (13 tiles of 90 x 90 x 50) in the exact partition of
    the 8-GPU node -- tiles 2,2,2,2,2,1,1,1 over 8 processes, rehearsed here on one GPU over
    gloo -- for 2 steps with the replicated CG2D (what cg2d="auto" picks across GPUs,
    parallel.cg2d_policy) and with the device CG2D (117 parts launched by 8 processes on one
    IPC-shared hand-off block).  Bars: every field bit-identical to one process, every solve
    record equal."""
    import torch.multiprocessing as mp
    from mitgcm_amd.parallel import TilePartition
    world, nsteps = 8, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, "llc90", nsteps, q, cg2d, "thermo", False))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        rank, res = q.get(timeout=540)
        assert "error" not in res, "rank %d: %s" % (rank, res["error"])
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0 = out[0]
    print("llc90 x8 (%s CG2D): iterations %s, max |diff| vs 1 process %s" % (
        cg2d, [s["cg2d_iters"] for s in r0["stats"]], r0["diff"]))
    assert all(r0["equal"].values()), r0["diff"]
    for rank, r in out.items():
        assert r["stats"] == r0["ref_stats"], (rank, r["stats"], r0["ref_stats"])
    part = TilePartition(13, world)
    assert part.counts == [2, 2, 2, 2, 2, 1, 1, 1]
    assert sorted((r["t0"], r["nT"]) for r in out.values()) == [part.range(r) for r in range(world)]


def test_device_cg2d_after_unshared_solve():
    """Rank 0 runs a multi-workgroup solve of its own before ShardedModel shares its hand-off
    block: sharing restarts every sharer's launch epoch and zeroes the block
    (mgcm_cg2d_shared_export / _import), so the shared solves still match tag for tag and the
    run stays bit-identical to one process."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world, nsteps = 2, 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, "llc30", nsteps, q, "device", "thermo", False, True))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in procs:
        rank, res = q.get(timeout=300)
        assert "error" not in res, "rank %d: %s" % (rank, res["error"])
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0 = out[0]
    assert all(r0["equal"].values()), r0["diff"]
    for rank, r in out.items():
        assert r["stats"] == r0["ref_stats"], (rank, r["stats"], r0["ref_stats"])
    assert all(s["cg2d_iters"] > 0 for s in r0["stats"])


@pytest.mark.parametrize("cfg,world,want", [("cs32x15", 2, "replicated"), ("llc30", 2, "replicated")])
def test_auto_cg2d_policy(cfg, world, want):
    """cg2d="auto" (ShardedModel's default) on the multi-workgroup grids: the cost model
    (parallel.cg2d_policy) picks the replicated solve across processes on C3 and the LLC, and
    the run stays bit-identical to one process with the same solver."""
    out = _spawn(cfg, world, 3, "auto")
    r0 = out[0]
    print("%s x%d cg2d=auto -> %s (%s)" % (cfg, world, r0["cg2d"], r0["cg2d_reason"]))
    assert all(r["cg2d"] == want for r in out.values()), [r["cg2d"] for r in out.values()]
    assert all(r0["equal"].values()), r0["diff"]
    for rank, r in out.items():
        assert r["stats"] == r0["ref_stats"], (rank, r["stats"], r0["ref_stats"])
