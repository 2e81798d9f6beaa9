"""Host logic of the tile-sharded path (mitgcm_amd/parallel.py) on CPU, gloo,
world sizes 2 and 3: the tile partition, the halo plan and the point-to-point
exchange reproduce the single-process EXCH (topology.py, restating
eesupp/src/exch1_rx.template:170-198) on every process's tiles, and the 2-D
block all-gather rebuilds the whole field.  Fields are numpy stand-ins for the
device arrays; pack/unpack index exactly as k_halo_pack does
(buf[(f*Nr + k)*n + h])."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mitgcm_amd.parallel import HaloPlan, TilePartition, exchange
from mitgcm_amd.topology import LatLonTopology

LAYOUTS = [  # sNx, sNy, OLx, OLy, nSx, nSy
    (31, 31, 2, 2, 2, 2),   # tutorial_baroclinic_gyre tiling (BASELINE config 4)
    (15, 8, 3, 3, 3, 2),    # 6 tiles, wide overlap
    (45, 40, 2, 2, 2, 1),   # tutorial_global_oce_latlon tiling
]


def test_partition():
    p = TilePartition(13, 8)   # two tiles on GPUs 0-4
    assert p.counts == [2, 2, 2, 2, 2, 1, 1, 1]
    assert p.starts[5] == 10 and p.maxT == 2
    assert list(p.owner(np.arange(13))) == [0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 6, 7]
    with pytest.raises(ValueError):
        TilePartition(4, 8)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, layout, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sNx, sNy, OLx, OLy, nSx, nSy = layout
        topo = LatLonTopology(sNx, sNy, OLx, OLy, nSx, nSy)
        nT, ny, nx, nz, nf = topo.nTiles, topo.ny, topo.nx, 3, 2
        n2 = nx * ny
        rng = np.random.default_rng(7)
        truth = [rng.standard_normal((nT, nz, ny, nx)) for _ in range(nf)]
        expect = [topo.exchange(a) for a in truth]
        part = TilePartition(nT, world)
        t0, c = part.range(rank)
        # this process: interior of its own tiles valid, everything else NaN
        mine = []
        for a in truth:
            b = np.full_like(a, np.nan)
            b[t0:t0 + c, :, OLy:OLy + sNy, OLx:OLx + sNx] = a[t0:t0 + c, :, OLy:OLy + sNy, OLx:OLx + sNx]
            mine.append(b)
        plan = HaloPlan(topo.src_of_point(), n2, part, rank)

        def flat(f, k):   # level k of field f as a (nT*n2,) view
            return mine[f][:, k].reshape(nT, n2)

        def pack(peer):
            idx = plan.send[peer]
            buf = np.empty(nf * nz * idx.size)
            for f in range(nf):
                for k in range(nz):
                    buf[(f * nz + k) * idx.size:(f * nz + k + 1) * idx.size] = flat(f, k).reshape(-1)[idx]
            return torch.from_numpy(buf)

        def make_buf(peer):
            return torch.empty(nf * nz * plan.recv[peer].size, dtype=torch.float64)

        def unpack(peer, buf):
            idx, b = plan.recv[peer], buf.numpy()
            for f in range(nf):
                for k in range(nz):
                    v = mine[f][:, k].reshape(-1)
                    v[idx] = b[(f * nz + k) * idx.size:(f * nz + k + 1) * idx.size]
                    mine[f][:, k] = v.reshape(nT, ny, nx)

        exchange(dist, plan, pack, unpack, make_buf)
        # local halo map restricted to this process's destination tiles (upload_halo)
        src = topo.src_of_point()
        dst = np.arange(src.size)
        sel = (src != dst) & (dst // n2 >= t0) & (dst // n2 < t0 + c)
        for f in range(nf):
            for k in range(nz):
                v = mine[f][:, k].reshape(-1)
                v[dst[sel]] = v[src[sel]]
                mine[f][:, k] = v.reshape(nT, ny, nx)
        ok = all(np.array_equal(mine[f][t0:t0 + c], expect[f][t0:t0 + c]) for f in range(nf))
        # 2-D block all-gather (ShardedModel._gather_2d, padded to maxT tiles)
        e2 = truth[0][:, 0]
        blk = np.zeros((part.maxT, ny, nx))
        blk[:c] = e2[t0:t0 + c]
        out = [torch.empty(part.maxT * n2, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(out, torch.from_numpy(blk.reshape(-1)))
        full = np.full_like(e2, np.nan)
        for r in range(world):
            s, cc = part.range(r)
            full[s:s + cc] = out[r].numpy().reshape(part.maxT, ny, nx)[:cc]
        ok = ok and np.array_equal(full, e2)
        nsend = sum(v.size for v in plan.send.values())
        q.put((rank, ok, nsend))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_exchange_matches_single_process(layout, world):
    nT = layout[4] * layout[5]
    if world > nT:
        pytest.skip("more processes than tiles")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, layout, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, nsend in res:
        assert ok, "rank %d: sharded exchange differs from the single-process EXCH" % rank
        assert nsend > 0


def _cube_worker(rank, world, port, q):
    """cs cube (pkg/exch2, 6 or 24 tiles): u, v travel with the union of the scalar and
    vector-map sources; the local vector map then reproduces EXCH2_UV_3D_RX on this
    process's tiles (signs and cube corners included)."""
    from mitgcm_amd.exch2 import cube_topology
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = True
        for sN, OL in ((8, 3), (4, 2)):
            topo = cube_topology(8, sN, sN, OL)
            nT, ny, nx = topo.nTiles, topo.ny, topo.nx
            n2, N = nx * ny, topo.nTiles * topo.ny * topo.nx
            rng = np.random.default_rng(11)
            truth = []
            for _ in range(2):
                a = np.full((nT, ny, nx), np.nan)
                a[:, OL:OL + sN, OL:OL + sN] = rng.standard_normal((nT, sN, sN))
                truth.append(a)
            eu, ev = topo.exchange_uv(truth[0], truth[1], True)
            part = TilePartition(nT, world)
            t0, c = part.range(rank)
            mine = [np.full(N, np.nan) for _ in range(2)]
            own = slice(t0 * n2, (t0 + c) * n2)
            for f in range(2):
                mine[f][own] = truth[f].reshape(-1)[own]
            cu, cv = topo.uv_codes(True)
            plan = HaloPlan(topo.src_of_point(), n2, part, rank, (cu, cv))

            def pack(peer):
                idx = plan.send[peer]
                return torch.from_numpy(np.concatenate([mine[0][idx], mine[1][idx]]))

            def make_buf(peer):
                return torch.empty(2 * plan.recv[peer].size, dtype=torch.float64)

            def unpack(peer, buf):
                idx, b = plan.recv[peer], buf.numpy()
                mine[0][idx], mine[1][idx] = b[:idx.size], b[idx.size:]

            exchange(dist, plan, pack, unpack, make_buf)
            uv = np.concatenate(mine)
            out = [m.copy() for m in mine]
            for f, code in enumerate((cu, cv)):
                d = np.nonzero(code)[0]
                d = d[(d // n2 >= t0) & (d // n2 < t0 + c)]
                out[f][d] = np.sign(code[d]) * uv[np.abs(code[d]) - 1]
            for f, e in enumerate((eu, ev)):
                ok = ok and np.array_equal(out[f][own], e.reshape(-1)[own], equal_nan=True)
        q.put((rank, ok, 1))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_cube_vector_exchange(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cube_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, _ in res:
        assert ok, "rank %d: sharded cube vector exchange differs from EXCH2_UV_3D_RX" % rank


def _tilesum_worker(rank, world, port, nTiles, q):
    """GLOBAL_SUM_TILE_RL over gloo: every process contributes the partials of its own
    tiles; the gathered buffer and its tile-ordered sum must be the single-process ones."""
    from mitgcm_amd.parallel import gather_tile_partials, tile_sum
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(11)
        allp = rng.standard_normal((nTiles, 2)) * 10.0 ** rng.integers(-8, 8, size=(nTiles, 2))
        part = TilePartition(nTiles, world)
        t0, nT = part.range(rank)
        local = torch.zeros((part.maxT, 2), dtype=torch.float64)
        local[:nT] = torch.as_tensor(allp[t0:t0 + nT])
        got = gather_tile_partials(dist, part, local, t0, nT, world, part.maxT, nTiles, "gloo")
        q.put((rank, got, [tile_sum(got[:, k]) for k in range(2)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nTiles", [(2, 6), (3, 6), (3, 13)])
def test_global_sum_tile_order_independent_of_world(world, nTiles):
    """The distributed CG2D's sums (parallel.tile_sum over gather_tile_partials) equal the
    sequential tile-order sum of global_sum_tile.F:185-190 on one process, bit for bit."""
    from mitgcm_amd.parallel import tile_sum
    ctx = mp.get_context("spawn")
    qq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tilesum_worker, args=(r, world, port, nTiles, qq)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict((r, (g, s)) for r, g, s in (qq.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(11)
    allp = rng.standard_normal((nTiles, 2)) * 10.0 ** rng.integers(-8, 8, size=(nTiles, 2))
    ref = []
    for k in range(2):
        acc = 0.0
        for t in range(nTiles):
            acc = acc + allp[t, k]
        ref.append(acc)
    assert tile_sum(allp[:, 0]) == ref[0]
    for r, (g, s) in out.items():
        assert np.array_equal(g, allp), r
        assert s == ref, (r, s, ref)


def _overlap_worker(rank, world, port, q):
    """The sharded step's exchange order (ShardedModel.step, THERMODYNAMICS forked): the
    tracers' halo batch posted at the join, a 2-D all-gather, the velocities' batch posted
    after the correction step, work in between, then both finished -- two outstanding
    isend/irecv batches per peer pair.  Every field's halo must equal the single-process
    EXCH, as with one exchange at the step's end."""
    from mitgcm_amd.parallel import start_exchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        topo = LatLonTopology(6, 5, 2, 2, 3, 2)
        nT, ny, nx = topo.nTiles, topo.ny, topo.nx
        n2 = nx * ny
        rng = np.random.default_rng(5)
        truth = [rng.standard_normal((nT, ny, nx)) for _ in range(4)]   # theta, salt | u, v
        expect = [topo.exchange(a[:, None])[:, 0] for a in truth]
        part = TilePartition(nT, world)
        t0, c = part.range(rank)
        mine = []
        for a in truth:
            b = np.full(a.size, np.nan)
            own = slice(t0 * n2, (t0 + c) * n2)
            b[own] = a.reshape(-1)[own]
            mine.append(b)
        plan = HaloPlan(topo.src_of_point(), n2, part, rank)

        def group(fields):
            def pack(peer):
                idx = plan.send[peer]
                return torch.from_numpy(np.concatenate([mine[f][idx] for f in fields]))

            def make_buf(peer):
                return torch.empty(len(fields) * plan.recv[peer].size, dtype=torch.float64)

            def unpack(peer, buf):
                idx, b = plan.recv[peer], buf.numpy()
                for n, f in enumerate(fields):
                    mine[f][idx] = b[n * idx.size:(n + 1) * idx.size]
            return pack, unpack, make_buf

        pk, up, mk = group((0, 1))
        fin_tr = start_exchange(dist, plan, pk, up, mk)          # at the THERMODYNAMICS join
        eta = torch.full((part.maxT * n2,), float(rank))
        out = [torch.empty_like(eta) for _ in range(world)]
        dist.all_gather(out, eta)                                 # exactConserv's eta gather
        pk, up, mk = group((2, 3))
        fin_vel = start_exchange(dist, plan, pk, up, mk)          # after the correction step
        work = sum(float(o[0]) for o in out)                      # phase 3 stands here
        fin_tr()
        fin_vel()
        src = topo.src_of_point()
        dst = np.arange(src.size)
        sel = (src != dst) & (dst // n2 >= t0) & (dst // n2 < t0 + c)
        ok = work == sum(range(world))
        for f in range(4):
            mine[f][dst[sel]] = mine[f][src[sel]]
            own = slice(t0 * n2, (t0 + c) * n2)
            ok = ok and np.array_equal(mine[f][own], expect[f].reshape(-1)[own])
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_overlapped_group_exchanges(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok in res:
        assert ok, "rank %d: overlapped tracer / velocity exchanges differ from the single-process EXCH" % rank


def _sub_worker(rank, world, port, q):
    """A subgroup of the default group (bench.py shards cs32x15 over min(N, 6) of N ranks):
    ranks 1 and 2 of 3 exchange halos and gather partials through parallel.Comm, whose
    group-local peers must map to the right global ranks."""
    from mitgcm_amd.parallel import Comm, gather_tile_partials, start_exchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sub = dist.new_group([1, 2], backend="gloo")   # collective over the default group
        if rank == 0:
            q.put((rank, True))
            return
        comm = Comm(dist, sub)
        me, w = comm.get_rank(), comm.get_world_size()
        topo = LatLonTopology(15, 8, 3, 3, 2, 2)
        nT, ny, nx = topo.nTiles, topo.ny, topo.nx
        n2 = nx * ny
        truth = np.random.default_rng(3).standard_normal((nT, ny, nx))
        part = TilePartition(nT, w)
        t0, c = part.range(me)
        mine = np.full_like(truth, np.nan)
        mine[t0:t0 + c, 3:11, 3:18] = truth[t0:t0 + c, 3:11, 3:18]
        plan = HaloPlan(topo.src_of_point(), n2, part, me)
        flat = mine.reshape(-1)

        def unpack(peer, buf):
            flat[plan.recv[peer]] = buf.numpy()
        start_exchange(comm, plan, lambda p: torch.from_numpy(flat[plan.send[p]].copy()), unpack,
                       lambda p: torch.empty(plan.recv[p].size, dtype=torch.float64))()
        src = topo.src_of_point()
        dst = np.arange(src.size)
        sel = (src != dst) & (dst // n2 >= t0) & (dst // n2 < t0 + c)
        flat[dst[sel]] = flat[src[sel]]
        ok = np.array_equal(mine[t0:t0 + c], topo.exchange(truth[:, None])[:, 0][t0:t0 + c])
        local = torch.zeros((part.maxT, 2), dtype=torch.float64)
        for i in range(c):
            local[i] = torch.tensor([t0 + i, 10.0 * (t0 + i)])
        allp = gather_tile_partials(comm, part, local, t0, c, w, part.maxT, nT, "gloo")
        ok = ok and np.array_equal(allp[:, 0], np.arange(nT)) and comm.get_backend() == "gloo"
        obj = ["from local rank 0" if me == 0 else None]
        comm.broadcast_object_list(obj, src=0)
        comm.barrier()
        q.put((rank, ok and obj[0] == "from local rank 0"))
    finally:
        dist.destroy_process_group()


def test_comm_subgroup():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sub_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(res.values()), res


def test_cg2d_policy():
    """cg2d="auto" (parallel.cg2d_policy): a single-CU solver stays replicated; the
    multi-workgroup solve stays on the device with one process and is replicated across
    GPUs while its hand-offs dominate an iteration (C3 pinned, C5 chip-wide), device only
    when the iteration work a 1/N share saves outweighs the fabric hand-offs."""
    from mitgcm_amd.parallel import MWG_COMPUTE_US_PER_ITER, cg2d_policy
    assert cg2d_policy("bxy", 8)[0] == "replicated"
    assert cg2d_policy("mwg", 1, 117)[0] == "device"
    assert cg2d_policy("mwg", 6, 6, pinned=True, compute_us=MWG_COMPUTE_US_PER_ITER)[0] == "replicated"
    assert cg2d_policy("mwg", 8, 117, pinned=False, compute_us=MWG_COMPUTE_US_PER_ITER)[0] == "replicated"
    assert cg2d_policy("mwg", 8, 4096, pinned=False, compute_us=100.0)[0] == "device"


def test_solve_check_default():
    """ShardedModel.replay / forward_step with check=None read the solve records back whenever
    the solver is the multi-workgroup one -- replicated (phases 2 / 19 launch it too, and its
    hand-off can time out) as well as across processes -- and not for a single-CU kernel or
    the host-decided distributed solve."""
    from mitgcm_amd.parallel import ShardedModel

    class _M:
        def __init__(self, k):
            self.k = k

        def cg2d_kernel(self):
            return self.k

    def may(kernel, mode):
        sm = ShardedModel.__new__(ShardedModel)   # no process group: only the predicate
        sm.m, sm.cg2d = _M(kernel), mode
        return sm._may_time_out()

    assert may("mwg", "replicated") and may("mwg", "device") and may("bxy", "device")
    assert not may("bxy", "replicated") and not may("mwg", "distributed")
