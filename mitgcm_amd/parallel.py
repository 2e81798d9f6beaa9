"""Tile-sharded FORWARD_STEP: one process per GPU over torch.distributed.

The reference runs its tiles over MPI ranks: each rank steps its own tiles
(myBxLo..myBxHi, eesupp/src/ini_procs.F), EXCH fills halos from neighbouring
ranks (eesupp/src/exch1_rx.template:170-198 via MPI send/recv) and every CG2D
iteration does three GLOBAL_SUM_TILE_RL (eesupp/src/global_sum_tile.F:14-237,
an MPI_Allreduce of per-tile partials summed in tile order).

The MI355X design keeps the 3-D work sharded; the 2-D solve runs where it is fastest:

* every process holds the WHOLE domain's arrays in HBM (memory is not the
  constraint: the largest BASELINE grid is 13 x 98^2 x 50 points) and its
  3-D kernels step only its contiguous tile range [t0, t0+nT)
  (mgcm_set_tile_range);
* per step the collectives are: the CG2D right-hand side's halo sources (device solve) or
  an all-gather of its tile blocks (replicated solve), one all-gather of the new free
  surface (exactConserv), and one point-to-point exchange of the 3-D halo sources
  (u, v, w, theta, salt) with each neighbouring process (twice with
  staggerTimeStep: the new velocities before THERMODYNAMICS, then the
  tracers);
* cg2d="auto" (the default) decides by the cost model of cg2d_policy: "replicated" for a
  single-CU kernel (C2, C4: ~4k points, one CU's solve at ~1.6 us per iteration beats any
  iteration that crosses GPUs) and, across processes, for the multi-workgroup solve too
  whenever its two hand-offs per iteration over the fabric cost more than the iteration
  work a 1/N share of the parts saves (C3: 6 parts on one XCD, ~1 us hand-offs; C5: 117
  parts chip-wide, ~0.9 us of compute per ~6 us iteration); "device" with one process;
* cg2d="device": the multi-workgroup CG2D (kernels_cg2d_mwg.hip) with every process
  launching only the parts of its own tiles; all parts meet on ONE hand-off block (rank 0's,
  mapped into the others by IPC, system-scope granules).  No host step and no collective
  inside an iteration; its sums keep the single-launch order, so the solve is the
  1-process multi-workgroup solve bit for bit, at any process count;
* cg2d="replicated": every GPU solves the gathered global problem with the 1-GPU kernel.
  No collective inside the iteration, and its sums are exactly the 1-GPU sums, so results
  are bit-identical at any GPU count (SURVEY.md 8(c) parity item 6);
* cg2d="distributed" is the reference's own distributed CG2D (cg2d.F:100-415):
  each process iterates on its own tiles only (mgcm_cg2d_op), the three global
  sums per iteration are GLOBAL_SUM_TILE_RL -- an all-gather of the per-tile
  partials, added in global tile order on every process
  (global_sum_tile.F:161-191, tile_sum below) -- and the two width-1 EXCH_S3D_RL
  of r and s are point-to-point exchanges of the halo sources.  Its iterates do
  not depend on the process count either (the per-tile partials are fixed-order
  device sums); 5 collectives per iteration make it latency-bound on RCCL: the
  reference-faithful option, kept for parity.

Transport: backend "nccl" (RCCL over xGMI) moves device tensors directly on
the model's stream; backend "gloo" stages through host memory (CPU tests,
and several ranks sharing one GPU on a 1-GPU box).
"""
import ctypes

import numpy as np


class TilePartition:
    """Contiguous balanced tile ranges in global tile order (SURVEY.md 8(e):
    tile index -> device in global-tile order; C5: 13 tiles on 8 GPUs = two
    tiles on GPUs 0-4)."""

    def __init__(self, nTiles, world):
        if world > nTiles:
            raise ValueError("%d tiles cannot be sharded over %d processes" % (nTiles, world))
        self.nTiles, self.world = nTiles, world
        base, rem = divmod(nTiles, world)
        self.counts = [base + (1 if r < rem else 0) for r in range(world)]
        self.starts = [sum(self.counts[:r]) for r in range(world)]
        self.maxT = max(self.counts)

    def range(self, rank):
        return self.starts[rank], self.counts[rank]

    def owner(self, tile):
        t = np.asarray(tile)
        return np.searchsorted(np.asarray(self.starts), t, side="right") - 1


class HaloPlan:
    """Which interior points each pair of processes must exchange so that every
    halo point of a process's tiles can be filled by the local halo map.

    src_of_point: flat (t, j, i) source of every halo-inclusive 2-D point (the
    topology's EXCH map, topology.py); uv_codes: the pkg/exch2 vector maps
    (exch2.py uv_codes), whose sources are added to the scalar ones.  Values travel to the SAME global offset
    on the receiver (every process holds the whole domain), so both sides list
    source offsets, sorted: send[peer] (in my tiles, needed by peer) equals the
    peer's recv[me]."""

    def __init__(self, src_of_point, n2, part, rank, uv_codes=None):
        src = np.asarray(src_of_point, dtype=np.int64)
        dst = np.arange(src.size, dtype=np.int64)
        halo = src != dst
        dst, src = dst[halo], src[halo]
        if uv_codes is not None:
            # pkg/exch2 vector maps (exch2_uv_3d_rx.template): a u or v halo point reads
            # u or v at (|code| - 1) mod N; both components travel, so only the point matters
            N = src_of_point.size if hasattr(src_of_point, "size") else len(src_of_point)
            for c in uv_codes:
                c = np.asarray(c, dtype=np.int64)
                d = np.nonzero(c)[0]
                dst = np.concatenate([dst, d])
                src = np.concatenate([src, (np.abs(c[d]) - 1) % N])
        dst_owner = part.owner(dst // n2)
        src_owner = part.owner(src // n2)
        self.rank, self.part = rank, part
        self.send, self.recv = {}, {}
        for peer in range(part.world):
            if peer == rank:
                continue
            s = np.unique(src[(src_owner == rank) & (dst_owner == peer)])
            r = np.unique(src[(src_owner == peer) & (dst_owner == rank)])
            if s.size:
                self.send[peer] = s
            if r.size:
                self.recv[peer] = r

    def peers(self):
        return sorted(set(self.send) | set(self.recv))


class Comm:
    """torch.distributed bound to one process group: the default group, or a subgroup (bench.py
    shards cs32x15 over min(N, 6) of N ranks).  It offers the module functions this file calls,
    with ranks local to the group (point-to-point peers are translated to global ranks), so
    the exchange helpers below take either this or the torch.distributed module itself."""

    def __init__(self, dist, group=None):
        self.d, self.group = dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.isend, self.irecv = dist.isend, dist.irecv

    def get_rank(self):
        return self.rank

    def get_world_size(self):
        return self.world

    def get_backend(self):
        return self.d.get_backend(self.group)

    def _g(self, r):
        return r if self.group is None else self.d.get_global_rank(self.group, r)

    def P2POp(self, op, tensor, peer):
        return self.d.P2POp(op, tensor, self._g(peer), group=self.group)

    def batch_isend_irecv(self, ops):
        return self.d.batch_isend_irecv(ops)

    def all_gather(self, out, t):
        return self.d.all_gather(out, t, group=self.group)

    def all_gather_into_tensor(self, out, t):
        return self.d.all_gather_into_tensor(out, t, group=self.group)

    def all_reduce(self, t, op=None):
        return self.d.all_reduce(t, op=op if op is not None else self.d.ReduceOp.SUM, group=self.group)

    def broadcast_object_list(self, obj, src=0):
        return self.d.broadcast_object_list(obj, src=self._g(src), group=self.group)

    def barrier(self):
        return self.d.barrier(group=self.group)


# CG2D placement across processes (cg2d="auto").  Per iteration the multi-workgroup solve makes
# two grid-wide hand-offs (kernels_cg2d_mwg.hip); its compute per iteration is small against
# them (LLC-90: ~2 150 of ~17 750 shader cycles, profiles/r03/mwg_stamps/).  Across processes
# the hand-off block lives on ONE GPU, so every part off that GPU polls it over the fabric: each
# hand-off costs at least a fabric round trip instead of an on-chip one, while the work that
# sharding removes is only that small compute share.  Replicated, every GPU runs the one-GPU
# solve on the gathered right-hand side (one all-gather of cg2d_b per step, no fabric inside an
# iteration).  The policy compares the two per solve with these constants (us):
HANDOFF_ONCHIP_US = {"pinned": 1.0, "spread": 3.0}   # one-XCD / chip-wide hand-off
HANDOFF_FABRIC_US = 5.0    # one hand-off polled across xGMI: >= one round trip (MI355X_MICROARCH.md)
MWG_COMPUTE_US_PER_ITER = 0.9   # LLC-90: ~2 150 shader cycles of an iteration's own work at 2.4 GHz


def cg2d_policy(solver, world, parts=0, pinned=False, compute_us=0.0):
    """(mode, reason) for cg2d="auto".  solver: the model's CG2D kernel ('mwg' or a single-CU
    one); parts: workgroups of the multi-workgroup solve; compute_us: its per-iteration compute
    (the part of an iteration that a 1/world share of the parts shrinks)."""
    if solver != "mwg":
        return "replicated", "single-CU CG2D: one CU's solve beats any iteration that crosses GPUs"
    if world <= 1:
        return "device", "one process: the resident multi-workgroup solve"
    h1 = HANDOFF_ONCHIP_US["pinned" if pinned else "spread"]
    replicated = 2 * h1 + compute_us
    device = 2 * HANDOFF_FABRIC_US + compute_us / world
    if device < replicated:
        return "device", "modelled %.1f us/iteration across %d GPUs < %.1f replicated" % (device, world, replicated)
    return "replicated", ("modelled %.1f us/iteration replicated <= %.1f with the hand-offs across %d GPUs "
                          "(%d parts, %s)" % (replicated, device, world, parts, "one XCD" if pinned else "chip-wide"))


def exchange(dist, plan, pack, unpack, make_buf):
    """Point-to-point exchange of halo sources with every neighbouring process.
    pack(peer) -> tensor to send; make_buf(peer) -> receive tensor;
    unpack(peer, tensor).  Grouped isend/irecv (one batch), lower rank posts first."""
    start_exchange(dist, plan, pack, unpack, make_buf)()


def start_exchange(dist, plan, pack, unpack, make_buf):
    """exchange() split at the reference's PUT/send | recv/GET boundary
    (pkg/exch2/exch2_rx1_cube.template:118-247): the sends and receives are posted now,
    and the returned finish() waits for them and unpacks -- work issued in between
    overlaps the transfer."""
    ops, recvs = [], {}
    for peer in plan.peers():
        if peer in plan.send:
            ops.append(dist.P2POp(dist.isend, pack(peer), peer))
        if peer in plan.recv:
            recvs[peer] = make_buf(peer)
            ops.append(dist.P2POp(dist.irecv, recvs[peer], peer))
    works = dist.batch_isend_irecv(ops) if ops else []

    def finish():
        for w in works:
            w.wait()
        for peer, buf in recvs.items():
            unpack(peer, buf)
    return finish


def tile_sum(partials):
    """GLOBAL_SUM_TILE_RL's final sum (eesupp/src/global_sum_tile.F:185-190): sumAllP = 0,
    then + every tile's partial in global tile order (Python floats are IEEE doubles, one
    rounding per addition, as the reference)."""
    acc = 0.0
    for v in partials:
        acc = acc + float(v)
    return acc


def gather_tile_partials(dist, part, local, t0, nT, world, maxT, nTiles, backend):
    """All-gather the per-tile partials of every process's tile range [t0, t0+nT):
    local is (maxT, m) on this process (rows 0..nT-1 valid); returns the (nTiles, m)
    global-tile-indexed buffer (host numpy), the same on every process."""
    import torch
    m = local.shape[1]
    if backend == "gloo":
        src = local.cpu() if local.is_cuda else local
        out = [torch.empty_like(src) for _ in range(world)]
        dist.all_gather(out, src)
        allp = torch.cat(out)
    else:
        allp = torch.empty((world * maxT, m), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(allp, local)
    allp = allp.cpu().numpy().reshape(world, maxT, m)
    res = np.empty((nTiles, m))
    for r in range(world):
        s, c = part.range(r)
        res[s:s + c] = allp[r, :c]
    return res


class ShardedModel:
    """A Model (model.py) stepped tile-sharded across the processes of the
    default torch.distributed group.  Every process must construct the same
    configuration; after init(), step()/forward_step() keep the tiles a
    process owns bit-identical to a single-process run."""

    def __init__(self, model, dist, device=None, cg2d="auto", overlap="thermo", model_stream="shared", group=None):
        import torch
        from ._lib import check, lib
        dist = dist if isinstance(dist, Comm) else Comm(dist, group)
        self.torch, self.dist, self.m = torch, dist, model
        self.L, self.check = lib(), check
        g = model.g
        self.g = g
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.part = TilePartition(g.nTiles, self.world)
        self.t0, self.nT = self.part.range(self.rank)
        self.backend = dist.get_backend()
        self.dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        h = model.h
        check(self.L.mgcm_set_tile_range(h, self.t0, self.nT), "mgcm_set_tile_range")
        if model_stream not in ("shared", "own"):
            raise ValueError("model_stream must be 'shared' or 'own'")
        self.model_stream = model_stream
        if self.backend == "nccl":
            # RCCL orders its work after the current stream: torch runs on one dedicated stream;
            # the model shares it ("shared", mgcm_set_stream -- the legacy default stream's
            # handle is NULL, which mgcm_set_stream reads as "the model's own stream") or keeps
            # its own ("own").  Either way every buffer crosses between the two through
            # mgcm_stream_handoff (_publish / _consume), so correctness does not rest on the
            # streams being one.
            self.stream = torch.cuda.Stream(self.dev)
            torch.cuda.set_stream(self.stream)
            if model_stream == "shared":
                check(self.L.mgcm_set_stream(h, ctypes.c_void_p(self.stream.cuda_stream)), "mgcm_set_stream")
        n2 = g.nx * g.ny
        self.n2 = n2
        uv = g.topo.uv_codes(True) if hasattr(g.topo, "uv_codes") else None
        self.plan = HaloPlan(g.topo.src_of_point(), n2, self.part, self.rank, uv)
        self.stagger = bool(model.params.get("staggerTimeStep", 0))
        self.nf = self.L.mgcm_exchange_nfields(h)
        # the halo field groups (mgcm_halo_pack_group): 0 all, 1 the tracers, 2 the rest
        self.nfg = {grp: self.L.mgcm_exchange_nfields_group(h, grp) for grp in (0, 1, 2)}
        # overlap (non-staggered steps):
        #   "thermo" (default, True): THERMODYNAMICS on the model's second stream as the resident
        #     step runs it -- beside DYNAMICS under r*, beside the pressure solve under the linear
        #     free surface (mgcm_step_phase 16) -- and the halos leave together at the step's end;
        #   "halo": THERMODYNAMICS first, then the tracers' halo sources travel while DYNAMICS,
        #     the solve and the continuity step compute;
        #   False: one stream, one exchange at the step's end.
        if overlap is True:
            overlap = "thermo"
        if overlap not in (False, None, "thermo", "halo"):
            raise ValueError("overlap must be 'thermo', 'halo' or False")
        tracers = bool(model.params.get("tempStepping", 1)) or bool(model.params.get("saltStepping", 1))
        self.fork = overlap == "thermo" and not self.stagger and tracers
        self.overlap = overlap == "halo" and not self.stagger and self.nfg[1] > 0
        dv = self.dev
        self.idx = {p: torch.as_tensor(v, device=dv) for p, v in
                    list(self.plan.send.items()) + [(("r", q), w) for q, w in self.plan.recv.items()]}
        self.sbuf = {grp: {p: torch.empty(max(1, self.nfg[grp]) * g.Nr * v.size, dtype=torch.float64, device=dv)
                           for p, v in self.plan.send.items()} for grp in (0, 1, 2)}
        self.rbuf = {grp: {p: torch.empty(max(1, self.nfg[grp]) * g.Nr * v.size, dtype=torch.float64, device=dv)
                           for p, v in self.plan.recv.items()} for grp in (0, 1, 2)}
        mt = self.part.maxT
        self.g_in = torch.empty(mt * n2, dtype=torch.float64, device=dv)
        self.g_out = torch.empty(self.world * mt * n2, dtype=torch.float64, device=dv)
        if cg2d not in ("auto", "replicated", "distributed", "device"):
            raise ValueError("cg2d must be 'auto', 'replicated', 'distributed' or 'device'")
        self.cg2d_reason = "requested"
        if cg2d == "auto":
            pinned = self.L.mgcm_get_param(model.h, b"cg2dPinned") != 0.0
            cg2d, self.cg2d_reason = cg2d_policy(model.cg2d_kernel(), self.world, model.cg2d_parts(), pinned,
                                                 MWG_COMPUTE_US_PER_ITER)
        self.cg2d = cg2d
        if cg2d == "device" and self.world > 1:
            # (one process: the model's own hand-off block as the resident solve uses it --
            # coarse-grained and one-XCD-pinned where that is faster, e.g. the cube -- nothing to map)
            self._share_cg2d_handoff()
        elif cg2d == "device" and self.m.cg2d_kernel() != "mwg":
            raise ValueError('cg2d="device" needs the multi-workgroup CG2D (set the parameter cg2dForceMwg=1)')
        if cg2d == "distributed":
            self.cg_part = torch.zeros(2 * g.nTiles, dtype=torch.float64, device=dv)   # part[2*tile + s]
            self.cg_local = torch.zeros((mt, 2), dtype=torch.float64, device=dv)
            self.cg_iters = []   # iterations of every distributed solve (host record)
        if cg2d in ("distributed", "device"):
            self.sbuf2 = {p: torch.empty(v.size, dtype=torch.float64, device=dv) for p, v in self.plan.send.items()}
            self.rbuf2 = {p: torch.empty(v.size, dtype=torch.float64, device=dv) for p, v in self.plan.recv.items()}

    def _share_cg2d_handoff(self):
        """cg2d="device": the multi-workgroup CG2D's hand-off block of rank 0 (granules,
        launch epoch, timeout word) mapped into every process by IPC, so that each process
        launches only its own tiles' parts and all of them meet on one block."""
        L, h, ck = self.L, self.m.h, self.check
        if self.m.cg2d_kernel() != "mwg":
            raise ValueError('cg2d="device" needs the multi-workgroup CG2D (set the parameter cg2dForceMwg=1)')
        nb = L.mgcm_cg2d_shared_bytes(h)
        buf = ctypes.create_string_buffer(nb)
        if self.rank == 0:
            ck(L.mgcm_cg2d_shared_export(h, buf), "mgcm_cg2d_shared_export")
        obj = [buf.raw if self.rank == 0 else None]
        self.dist.broadcast_object_list(obj, src=0)
        if self.rank != 0:
            ck(L.mgcm_cg2d_shared_import(h, ctypes.create_string_buffer(obj[0], nb)), "mgcm_cg2d_shared_import")
        self.dist.barrier()

    # ---- transport -------------------------------------------------------------
    def _cur(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.dev).cuda_stream)

    def _publish(self):
        """torch's stream waits for the model's work so far (its outputs become readable)."""
        self.check(self.L.mgcm_stream_handoff(self.m.h, self._cur(), 0), "mgcm_stream_handoff")

    def _consume(self):
        """the model's stream waits for torch's work so far (received buffers)."""
        self.check(self.L.mgcm_stream_handoff(self.m.h, self._cur(), 1), "mgcm_stream_handoff")

    def _gather_2d(self, name):
        """all-gather the tile blocks of a 2-D field from their owners."""
        L, h, n2 = self.L, self.m.h, self.n2
        mt = self.part.maxT
        self.check(L.mgcm_tile_copy(h, name.encode(), self.t0, self.nT, ctypes.c_void_p(self.g_in.data_ptr()), 0),
                   "mgcm_tile_copy")
        self._publish()
        if self.backend == "gloo":
            self.torch.cuda.synchronize(self.dev)
            src = self.g_in.cpu()
            out = [self.torch.empty_like(src) for _ in range(self.world)]
            self.dist.all_gather(out, src)
            self.g_out.copy_(self.torch.cat(out))
            self.torch.cuda.synchronize(self.dev)
        else:
            self.dist.all_gather_into_tensor(self.g_out, self.g_in)
        self._consume()
        for r in range(self.world):
            if r == self.rank:
                continue
            s, c = self.part.range(r)
            buf = self.g_out[r * mt * n2:]
            self.check(L.mgcm_tile_copy(h, name.encode(), s, c, ctypes.c_void_p(buf.data_ptr()), 1),
                       "mgcm_tile_copy")

    def _halo(self, group=0, start_only=False):
        """The 3-D halo sources of a field group with every neighbouring process; with
        start_only the transfer is posted and the finish() that completes it returned."""
        L, h = self.L, self.m.h

        def pack(peer):
            buf = self.sbuf[group][peer]
            self.check(L.mgcm_halo_pack_group(h, group, ctypes.c_void_p(self.idx[peer].data_ptr()),
                                              self.plan.send[peer].size, ctypes.c_void_p(buf.data_ptr()), 0),
                       "mgcm_halo_pack_group")
            self._publish()
            if self.backend == "gloo":
                self.torch.cuda.synchronize(self.dev)
                return buf.cpu()
            return buf

        def make_buf(peer):
            return self.rbuf[group][peer].cpu() if self.backend == "gloo" else self.rbuf[group][peer]

        def unpack(peer, buf):
            dev = self.rbuf[group][peer]
            if buf is not dev:
                dev.copy_(buf)
                self.torch.cuda.synchronize(self.dev)
            self._consume()
            self.check(L.mgcm_halo_pack_group(h, group, ctypes.c_void_p(self.idx[("r", peer)].data_ptr()),
                                              self.plan.recv[peer].size, ctypes.c_void_p(dev.data_ptr()), 1),
                       "mgcm_halo_pack_group")

        fin = start_exchange(self.dist, self.plan, pack, unpack, make_buf)
        if start_only:
            return fin
        fin()
        return None

    def _exch_2d(self, name):
        """EXCH of one 2-D field across processes: the sources of my tiles' halo points
        arrive from their owners (HaloPlan point lists, one value per point), then the
        local halo fill (EXCH_XY_RL / EXCH_S3D_RL on this process's copy)."""
        L, h, ck, torch = self.L, self.m.h, self.check, self.torch
        gloo = self.backend == "gloo"
        nm = name.encode()

        def pack(peer):
            buf = self.sbuf2[peer]
            ck(L.mgcm_field_pack(h, nm, ctypes.c_void_p(self.idx[peer].data_ptr()), self.plan.send[peer].size,
                                 ctypes.c_void_p(buf.data_ptr()), 0), "mgcm_field_pack")
            self._publish()
            if gloo:
                torch.cuda.synchronize(self.dev)
                return buf.cpu()
            return buf

        def make_buf(peer):
            return self.rbuf2[peer].cpu() if gloo else self.rbuf2[peer]

        def unpack(peer, buf):
            dev = self.rbuf2[peer]
            if buf is not dev:
                dev.copy_(buf)
                torch.cuda.synchronize(self.dev)
            self._consume()
            ck(L.mgcm_field_pack(h, nm, ctypes.c_void_p(self.idx[("r", peer)].data_ptr()), self.plan.recv[peer].size,
                                 ctypes.c_void_p(dev.data_ptr()), 1), "mgcm_field_pack")

        exchange(self.dist, self.plan, pack, unpack, make_buf)
        ck(L.mgcm_exchange_field(h, nm), "mgcm_exchange_field")

    def _tile_sums(self, op, a0=0.0):
        """One cg2d.F operation on my tiles, then GLOBAL_SUM_TILE_RL's collection of the
        per-tile partials: the (nTiles, 2) buffer, identical on every process."""
        L, h = self.L, self.m.h
        self.check(L.mgcm_cg2d_op(h, op, float(a0), ctypes.c_void_p(self.cg_part.data_ptr())), "mgcm_cg2d_op(%d)" % op)
        self._publish()
        if self.backend == "gloo":   # the model runs on its own stream: wait for the partials
            self.torch.cuda.synchronize(self.dev)
        if self.nT:
            self.cg_local[:self.nT].copy_(self.cg_part[2 * self.t0:2 * (self.t0 + self.nT)].view(self.nT, 2))
        if self.backend == "gloo":
            self.torch.cuda.synchronize(self.dev)
        return gather_tile_partials(self.dist, self.part, self.cg_local, self.t0, self.nT, self.world,
                                    self.part.maxT, self.g.nTiles, self.backend)

    def _cg2d_distributed(self):
        """CG2D (model/src/cg2d.F:100-415) over the processes' tiles: 3 GLOBAL_SUM_TILE_RL
        and 2 EXCH_S3D_RL per iteration, scalars (beta, alpha, the residual) on the host
        in the reference's arithmetic; with useSRCGSolver CG2D_SR (cg2d_sr.F): one exchange
        (y) and one round of sums per iteration; cg2dUseMinResSol keeps the lowest-residual
        solution in both."""
        import math
        L, h, ck = self.L, self.m.h, self.check
        prm = lambda n: L.mgcm_get_param(h, n.encode())
        normalise = prm("cg2dNormaliseRHS") != 0.0
        tol_sq, maxit = prm("cg2dTolerance_sq"), int(prm("cg2dMaxIters"))
        # cg2dUseMinResSol: SOLVE_FOR_PRESSURE passes nIterMin = cg2dUseMinResSol - 1, >= 0 keeps
        # the lowest-residual solution (cg2d.F:148-155, 190-193, 338-351, 358-369)
        keepMin = int(prm("cg2dUseMinResSol")) - 1 >= 0
        sr = prm("useSRCGSolver") != 0.0
        minResSq, nIterMin = -1.0, -1
        P = self._tile_sums(0)                         # cg2d.F:104-114, rhsMax per tile
        rhsMax = float(np.max(P[:, 0]))                # _GLOBAL_MAX_RL (order-free)
        rhsNorm = 1.0
        if normalise:                                  # cg2d.F:116-133
            if rhsMax != 0.0:
                rhsNorm = 1.0 / rhsMax
            ck(L.mgcm_cg2d_op(h, 1, rhsNorm, ctypes.c_void_p(self.cg_part.data_ptr())), "mgcm_cg2d_op(1)")
        self._exch_2d("cg2d_x")                        # EXCH_XY_RL(cg2d_x), cg2d.F:135
        P = self._tile_sums(2)                         # r = b - A x, cg2d.F:136-179
        if keepMin:
            ck(L.mgcm_cg2d_op(h, 8, 0.0, None), "mgcm_cg2d_op(8)")
        err_sq, sumRHS = tile_sum(P[:, 0]), tile_sum(P[:, 1])
        first, its = math.sqrt(err_sq), 0
        if keepMin:
            minResSq, nIterMin = err_sq, 0
        self._exch_2d("cg2d_r")
        eta_qrNM1 = 1.0
        if sr and not err_sq < tol_sq:                 # CG2D_SR, cg2d_sr.F:220-422
            eta_qrN = tile_sum(self._tile_sums(10)[:, 0])      # y = M r, s = y, (y, r)
            self._exch_2d("cg2d_s")
            eta_qrNM1 = eta_qrN
            alpha = tile_sum(self._tile_sums(5)[:, 0])         # q = A s, (s, q)
            sigma = eta_qrN / alpha
            ck(L.mgcm_cg2d_op(h, 11, sigma, None), "mgcm_cg2d_op(11)")
            self._exch_2d("cg2d_r")
            conv, it = False, 1
            while it <= maxit - 1:
                ck(L.mgcm_cg2d_op(h, 12, 0.0, None), "mgcm_cg2d_op(12)")   # y = M r
                self._exch_2d("cg2d_y")
                P = self._tile_sums(13)                        # v = A y, (y, r), (y, v)
                eta_qrN, delta = tile_sum(P[:, 0]), tile_sum(P[:, 1])
                err_sq = tile_sum(self._tile_sums(14)[:, 0])   # (r, r)
                if err_sq < tol_sq:
                    conv = True
                    break
                if err_sq < minResSq:
                    minResSq, nIterMin = err_sq, it
                    ck(L.mgcm_cg2d_op(h, 8, 0.0, None), "mgcm_cg2d_op(8)")
                cgBeta = eta_qrN / eta_qrNM1
                eta_qrNM1 = eta_qrN
                alpha = delta - (cgBeta * cgBeta) * alpha
                sigma = eta_qrN / alpha
                ck(L.mgcm_cg2d_op(h, 15, cgBeta, None), "mgcm_cg2d_op(15)")
                ck(L.mgcm_cg2d_op(h, 11, sigma, None), "mgcm_cg2d_op(11)")
                self._exch_2d("cg2d_r")
                it += 1
            if not conv:                               # the residual of the last update
                err_sq = tile_sum(self._tile_sums(14)[:, 0])
            its = it                                   # numIters = it2d (cg2d_sr.F:449)
        elif not err_sq < tol_sq:
            for it in range(1, maxit + 1):
                eta_qrN = tile_sum(self._tile_sums(3)[:, 0])   # q = M r, (q, r)
                beta = eta_qrN / eta_qrNM1
                eta_qrNM1 = eta_qrN
                ck(L.mgcm_cg2d_op(h, 4, beta, ctypes.c_void_p(self.cg_part.data_ptr())), "mgcm_cg2d_op(4)")
                self._exch_2d("cg2d_s")
                alpha = eta_qrN / tile_sum(self._tile_sums(5)[:, 0])   # q = A s, (s, q)
                err_sq = tile_sum(self._tile_sums(6, alpha)[:, 0])     # x, r update, (r, r)
                its = it
                if err_sq < tol_sq:
                    break
                if err_sq < minResSq:
                    minResSq, nIterMin = err_sq, it
                    ck(L.mgcm_cg2d_op(h, 8, 0.0, None), "mgcm_cg2d_op(8)")
                self._exch_2d("cg2d_r")
        if nIterMin >= 0 and err_sq > minResSq:
            ck(L.mgcm_cg2d_op(h, 9, 0.0, None), "mgcm_cg2d_op(9)")
        if normalise:                                  # un-normalise, cg2d.F:372-385
            ck(L.mgcm_cg2d_op(h, 7, rhsNorm, ctypes.c_void_p(self.cg_part.data_ptr())), "mgcm_cg2d_op(7)")
        ck(L.mgcm_cg2d_record(h, first, math.sqrt(err_sq), rhsMax, sumRHS, its, minResSq, nIterMin), "mgcm_cg2d_record")
        self.cg_iters.append(its)

    # ---- stepping ----------------------------------------------------------------
    def step(self):
        L, h, ck = self.L, self.m.h, self.check
        fin_tracers = None
        if self.fork:
            ck(L.mgcm_step_phase(h, 16), "mgcm_step_phase(16)")
            ck(L.mgcm_step_phase(h, 9), "mgcm_step_phase(9)")
        elif self.overlap:
            # DO_OCEANIC_PHYS + THERMODYNAMICS, then the tracers' halo sources leave while
            # DYNAMICS, the solve and the continuity step compute
            ck(L.mgcm_step_phase(h, 8), "mgcm_step_phase(8)")
            fin_tracers = self._halo(1, start_only=True)
            ck(L.mgcm_step_phase(h, 9), "mgcm_step_phase(9)")
        else:
            ck(L.mgcm_step_phase(h, 1), "mgcm_step_phase(1)")
        # with THERMODYNAMICS forked, the correction step is split off its phase (17 | 18): the
        # new tracers' halo sources leave at the join and travel while the correction and
        # continuity pass runs (the velocities' follow it)
        split = self.fork

        def after_solve(p6):
            nonlocal fin_tracers
            if split:
                ck(L.mgcm_step_phase(h, 17), "mgcm_step_phase(17)")
                fin_tracers = self._halo(1, start_only=True)
                ck(L.mgcm_step_phase(h, 18), "mgcm_step_phase(18)")
            else:
                ck(L.mgcm_step_phase(h, p6), "mgcm_step_phase(%d)" % p6)
        if self.cg2d == "distributed":
            self._cg2d_distributed()
            self._exch_2d("cg2d_x")      # the halo sources of the new x before etaN everywhere
            after_solve(6)
        elif self.cg2d == "device":
            # the parts' rings reach into the neighbours' tiles: their b and x first
            self._exch_2d("cg2d_b")
            self._exch_2d("cg2d_x")
            ck(L.mgcm_step_phase(h, 10), "mgcm_step_phase(10)")   # this process's parts
            self._exch_2d("cg2d_x")
            after_solve(6)
        else:
            self._gather_2d("cg2d_b")
            self._gather_2d("cg2d_x")
            if split:
                ck(L.mgcm_step_phase(h, 19), "mgcm_step_phase(19)")
                after_solve(None)
            else:
                ck(L.mgcm_step_phase(h, 2), "mgcm_step_phase(2)")
        if self.m.params.get("exactConserv", 0):
            self._gather_2d("cg2d_b")
        # the velocities' halo sources (u, v, w, the CD-scheme copies, phi) are final after the
        # correction step: they leave before the end of FORWARD_STEP's 2-D work (EXCH eta +
        # UPDATE_ETAH, CALC_R_STAR -- phase 3 touches no 3-D field) and are received after it,
        # the reference's PUT/send -> recv/GET split (exch2_rx1_cube.template:118-247)
        fin_rest = self._halo(2 if fin_tracers is not None else 0, start_only=True)
        ck(L.mgcm_step_phase(h, 3), "mgcm_step_phase(3)")
        if fin_tracers is not None:
            fin_tracers()
        fin_rest()
        if self.stagger:
            # DO_STAGGER_FIELDS_EXCHANGES, then THERMODYNAMICS with the new velocities
            ck(L.mgcm_step_phase(h, 5), "mgcm_step_phase(5)")
            self._halo()
        ck(L.mgcm_step_phase(h, 4), "mgcm_step_phase(4)")

    def capture_step(self):
        """Capture two steps (replicated CG2D; RCCL all-gathers and point-to-point exchanges
        included) into a HIP graph via torch.cuda.graph, for replay(): the model runs on a
        side stream that is also the capture stream.  Two, because CYCLE_TRACER swaps the
        theta/salt buffers on the host: after two steps the kernels' pointers are back where
        they started.  Runs one warm-up step eagerly first (so the communicators exist before
        capture): the model advances by that step."""
        if self.backend != "nccl" or self.cg2d == "distributed":
            raise ValueError("graph capture needs the nccl (RCCL) backend and a device-decided CG2D "
                             "(the host-distributed solve decides on the host each iteration)")
        torch, L, h = self.torch, self.L, self.m.h
        s = torch.cuda.Stream(self.dev)
        self.check(L.mgcm_set_stream(h, ctypes.c_void_p(s.cuda_stream)), "mgcm_set_stream")
        with torch.cuda.stream(s):
            self.check(L.mgcm_begin_steps(h), "mgcm_begin_steps")
            self.step()
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            self.step()
            self.step()
        torch.cuda.synchronize(self.dev)
        # back onto the model's stream (torch's current one, where the collectives of eager
        # steps and replay() run): begin_steps' memset and eager steps after a capture are
        # then ordered with the replays and the RCCL calls on one stream
        self.check(L.mgcm_set_stream(h, ctypes.c_void_p(self.stream.cuda_stream) if self.model_stream == "shared"
                                     else None), "mgcm_set_stream")
        self._graph, self._gstream = g, s

    def _check_records(self, nsteps):
        """Refuse a batch whose solves wrote past the device's record ring (mgcm_end_steps
        validates nsteps against it) -- checked BEFORE the steps run."""
        self.check(self.L.mgcm_end_steps(self.m.h, nsteps), "mgcm_end_steps")

    def check_solves(self, nsteps):
        """Raise if any solve of the last nsteps steps failed: a device CG2D whose grid
        hand-off timed out records numIters = -1 (kernels_cg2d_mwg.hip) and leaves cg2d_x
        unconverged.  The device CG2D's parts spin-wait for each other across processes, so
        every process must launch its parts of a solve while the others' are running (host
        work between steps -- Python, gloo staging -- delays a launch; past ~2^22 polls every
        part gives up rather than hang)."""
        if nsteps <= 0:
            return
        its = (ctypes.c_int * nsteps)()
        self.check(self.L.mgcm_solve_history(self.m.h, nsteps, its, None, None), "mgcm_solve_history")
        bad = [i for i, n in enumerate(its) if n < 0]
        if bad:
            raise RuntimeError("CG2D failed (grid hand-off timeout, numIters = -1) in step(s) %s of the last %d"
                               % (bad, nsteps))

    def replay(self, npairs=1, check=None):
        """Replay the captured pair of steps npairs times (the device's per-step record ring
        restarts at the first replay); with check, the batch's solve records are read back
        and a failed solve raises (check_solves).  check=None: whenever the model's solver is
        the multi-workgroup one (its grid hand-offs can time out, numIters = -1), whether it
        runs across processes (cg2d="device") or replicated per process (phases 2 / 19);
        the single-CU kernels cannot time out (the read-back synchronises the host)."""
        self._check_records(2 * npairs)
        self.check(self.L.mgcm_begin_steps(self.m.h), "mgcm_begin_steps")   # on self.stream
        if self.model_stream != "shared":
            self._publish()   # the record reset (model stream) before the replays (torch's)
        with self.torch.cuda.stream(self.stream):
            for _ in range(npairs):
                self._graph.replay()
        if self.model_stream != "shared":
            self._consume()   # the model's later work after the replays
        self.check(self.L.mgcm_end_steps(self.m.h, 2 * npairs), "mgcm_end_steps")
        if check or (check is None and self._may_time_out()):
            self.check_solves(2 * npairs)

    def forward_step(self, nsteps=1, check=None):
        """nsteps sharded FORWARD_STEPs; with check, a failed solve raises (check_solves);
        check=None: whenever the solver is the multi-workgroup one (as replay)."""
        self._check_records(nsteps)
        self.check(self.L.mgcm_begin_steps(self.m.h), "mgcm_begin_steps")
        for _ in range(nsteps):
            self.step()
        if check or (check is None and self._may_time_out()):
            self.check_solves(nsteps)

    def _may_time_out(self):
        """The solves whose records must be read back: the multi-workgroup CG2D's grid
        hand-off can time out in the device and the replicated mode alike; the distributed
        solve is decided on the host and raises there."""
        return self.cg2d != "distributed" and (self.cg2d == "device" or self.m.cg2d_kernel() == "mwg")

    def gather_field(self, name):
        """The whole-domain field assembled from every owner (host numpy), e.g.
        for monitors / parity checks; collective."""
        a = self.m.get(name)
        t = self.torch.as_tensor(a.reshape(a.shape[0], -1))
        if self.backend != "gloo":
            t = t.to(self.dev)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        out = [o.cpu() for o in out]
        res = a.copy()
        for r in range(self.world):
            s, c = self.part.range(r)
            res[s:s + c] = out[r].numpy().reshape(a.shape)[s:s + c]
        return res
