"""RCCL on the MI355X: the tile-sharded driver (mitgcm_amd/parallel.py) with the "nccl"
backend (RCCL) at world size 1 -- the only RCCL world a 1-GPU box can host; the multi-GPU
node runs the same calls with peers.  BASELINE config 4 (baroclinic gyre + DST3-FL, 4 tiles):
  * eager sharded stepping over RCCL (device all-gathers of the CG2D right-hand side and
    of eta, the tracers' halo exchange overlapping DYNAMICS): bit-identical to the
    single-process model, with the model on torch's stream and on its own stream (ordered
    by mgcm_stream_handoff events only);
  * the distributed CG2D (GLOBAL_SUM_TILE_RL as an RCCL all-gather of per-tile partials):
    iteration counts of the replicated solve, fields within 1e-10;
  * two steps captured into a HIP graph with their RCCL collectives (torch.cuda.graph on
    a side stream) and replayed: bit-identical to stepping eagerly; an eager step after
    the replays (back on the collectives' stream) stays bit-identical;
  * BASELINE config 5's LLC topology at n = 30 with the device multi-workgroup CG2D and
    THERMODYNAMICS on the second stream, captured and replayed: bit-identical."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("uVel", "vVel", "wVel", "theta", "etaN")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _make():
    from mitgcm_amd import configs
    return configs.make_model(configs.baroclinic_gyre, tempAdvScheme=33)


def _make_llc():
    from mitgcm_amd import configs
    return configs.make_model(lambda: (lambda r: (r[0], {**r[1], "cg2dForceMwg": 1}) + tuple(r[2:]))(
        configs.llc_synthetic(n=30, Nr=10)))


def _worker(port, q):
    try:
        import torch
        import torch.distributed as dist
        from mitgcm_amd.parallel import ShardedModel
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        res = {}
        ref = _make()
        ref.forward_step(4)
        ref.sync()
        want = {n: ref.get(n) for n in FIELDS}
        ref_its = [ref.solve_stats(back=b)["cg2d_iters"] for b in range(4)]
        ref.forward_step(1)
        ref.sync()
        want5 = {n: ref.get(n) for n in FIELDS}
        ref.forward_step(1)
        ref.sync()
        want6 = {n: ref.get(n) for n in FIELDS}
        ref.close()
        # eager, replicated CG2D
        m = _make()
        sm = ShardedModel(m, dist)
        sm.forward_step(4)
        torch.cuda.synchronize()
        res["eager"] = {n: bool(np.array_equal(sm.gather_field(n), want[n])) for n in FIELDS}
        m.close()
        # the model on its own stream, torch's collectives on another: every buffer crosses
        # through mgcm_stream_handoff
        m = _make()
        sm = ShardedModel(m, dist, model_stream="own")
        sm.forward_step(4)
        torch.cuda.synchronize()
        res["own_stream"] = {n: bool(np.array_equal(sm.gather_field(n), want[n])) for n in FIELDS}
        m.close()
        # distributed CG2D over RCCL
        m = _make()
        sm = ShardedModel(m, dist, cg2d="distributed")
        sm.forward_step(4)
        torch.cuda.synchronize()
        res["dist_iters"] = (list(reversed(sm.cg_iters)), ref_its)
        res["dist_diff"] = {n: float(np.abs(sm.gather_field(n) - want[n]).max() / max(np.abs(want[n]).max(), 1e-300))
                            for n in FIELDS}
        m.close()
        # graph capture: 1 eager warm-up step + 2 replays of the captured pair of steps
        m = _make()
        sm = ShardedModel(m, dist)
        sm.capture_step()
        sm.replay(2)
        torch.cuda.synchronize()
        res["graph"] = {n: bool(np.array_equal(sm.gather_field(n), want5[n])) for n in FIELDS}
        # an eager step after the replays: the model is back on the stream of the collectives
        sm.forward_step(1)
        torch.cuda.synchronize()
        res["eager_after_graph"] = {n: bool(np.array_equal(sm.gather_field(n), want6[n])) for n in FIELDS}
        m.close()
        # BASELINE config 5's LLC topology (n = 30, 13 tiles): the device multi-workgroup CG2D
        # (cg2d="device", its hand-off block exported by IPC), THERMODYNAMICS on the second
        # stream beside the solve (overlap="thermo"), captured with the collectives and replayed
        ref = _make_llc()
        ref.forward_step(5)
        ref.sync()
        want_llc = {n: ref.get(n) for n in FIELDS}
        ref.close()
        m = _make_llc()
        sm = ShardedModel(m, dist, cg2d="device")
        res["llc_cg2d"] = sm.cg2d
        res["llc_fork"] = sm.fork
        sm.capture_step()
        sm.replay(2)
        torch.cuda.synchronize()
        res["llc_graph"] = {n: bool(np.array_equal(sm.gather_field(n), want_llc[n])) for n in FIELDS}
        m.close()
        dist.destroy_process_group()
        q.put(res)
    except Exception:
        import traceback
        q.put({"error": traceback.format_exc()})


def test_rccl_world1_eager_distributed_and_graph():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=60)
    assert "error" not in res, res.get("error")
    print("RCCL world 1:", res)
    assert all(res["eager"].values()), res["eager"]
    assert all(res["own_stream"].values()), res["own_stream"]
    its, ref_its = res["dist_iters"]
    assert its == ref_its, res["dist_iters"]   # per step, most recent first in both lists
    assert max(res["dist_diff"].values()) <= 1e-10, res["dist_diff"]
    assert all(res["graph"].values()), res["graph"]
    assert all(res["eager_after_graph"].values()), res["eager_after_graph"]
    assert res["llc_cg2d"] == "device" and res["llc_fork"], res
    assert all(res["llc_graph"].values()), res["llc_graph"]
