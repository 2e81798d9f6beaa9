"""Diagnose a tile-sharded run: after each step, which fields differ from a single-process
run on which tiles.  python tools/shard_diag.py WORLD NSTEPS [config]"""
import os
import socket
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIELDS = ("uVel", "vVel", "wVel", "theta", "salt", "etaN", "etaH", "gtNm1", "guNm1", "gvNm1", "rStarFacC", "hFacC",
          "cg2d_b", "cg2d_x", "PmEpR", "totPhiHyd", "rhoInSitu", "Kwx", "GM_PsiX")


def make(cfg):
    from mitgcm_amd import configs
    if cfg == "gyre":
        return configs.make_model(configs.baroclinic_gyre, tempAdvScheme=33)
    return configs.make_model(configs.global_ocean_cs32x15)


def worker(rank, world, port, nsteps, cfg, q):
    import torch
    import torch.distributed as dist
    from mitgcm_amd.parallel import ShardedModel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    m = make(cfg)
    sm = ShardedModel(m, dist, device=torch.device("cuda", 0))
    ref = make(cfg) if rank == 0 else None
    L = sm.L
    L.mgcm_begin_steps(m.h)
    for s in range(nsteps):
        sm.step()
        m.sync()
        full = {}
        for n in FIELDS:
            try:
                full[n] = sm.gather_field(n)
            except Exception:
                pass
        if rank == 0:
            ref.forward_step(1)
            ref.sync()
            for n, a in full.items():
                b = ref.get(n)
                bad = [t for t in range(a.shape[0]) if not np.array_equal(a[t], b[t], equal_nan=True)]
                if bad:
                    print("step %d %-10s tiles %s max %.3g" % (s + 1, n, bad, np.nanmax(np.abs(a - b))), flush=True)
    q.put(rank)
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    world, nsteps = int(sys.argv[1]), int(sys.argv[2])
    cfg = sys.argv[3] if len(sys.argv) > 3 else "cs32x15"
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, nsteps, cfg, q)) for r in range(world)]
    for p in ps:
        p.start()
    for _ in ps:
        q.get(timeout=600)
    for p in ps:
        p.join(60)
    print("world", world, "done")
