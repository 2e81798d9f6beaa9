"""Per-GPU work of an N-way tile partition, measured on one GPU.

For N in 1, 2, 4, 8 the model steps the largest share of the partition (parallel.TilePartition:
rank 0's range, ceil(nTiles/N) tiles) through the sharded step's phases -- DO_OCEANIC_PHYS +
THERMODYNAMICS on the second stream (16), DYNAMICS + the pressure right-hand side (9), the
correction and continuity step (6), CALC_R_STAR (3), the blocking exchanges (4) -- with the
CG2D and the collectives left out: K steps captured into one HIP graph and replayed, timed
with events.  The CG2D of the resident step at N = 1 is timed beside it (graph-replayed
FORWARD_STEP minus the same phases), the part of the step no partition shrinks.

    python tools/partition_time.py [config] [K]      (prints one JSON object)
"""
import ctypes
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from mitgcm_amd import configs
    from mitgcm_amd._lib import check, lib
    from mitgcm_amd.parallel import TilePartition
    L = lib()
    cfg = sys.argv[1] if len(sys.argv) > 1 else "llc90_synthetic"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    torch.cuda.set_device(0)
    out = {"config": cfg, "steps_per_graph": K}
    # the resident step (graph-replayed, CG2D included) for reference
    m = configs.make_model(bench.config_fn(cfg))
    m.forward_step(2)
    m.prepare()
    m.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    m.sync()
    import time
    t0 = time.perf_counter()
    m.forward_step(2 * K)
    m.sync()
    out["resident_ms_per_step"] = 1e3 * (time.perf_counter() - t0) / (2 * K)
    m.kernel_timing(True)
    m.forward_step(4)
    m.sync()
    out["resident_cg2d_ms"] = m.kernel_ms("cg2d")[0]
    m.kernel_timing(False)
    m.close()
    nt = None
    rows = []
    for N in (1, 2, 4, 8):
        m = configs.make_model(bench.config_fn(cfg))
        h = m.h
        nt = m.g.nTiles
        if N > nt:
            m.close()
            continue
        part = TilePartition(nt, N)
        t0_, nT = part.range(0)
        check(L.mgcm_set_tile_range(h, t0_, nT), "mgcm_set_tile_range")
        s = torch.cuda.Stream()
        check(L.mgcm_set_stream(h, ctypes.c_void_p(s.cuda_stream)), "mgcm_set_stream")

        def step():
            for ph in (16, 9, 6, 3, 4):
                check(L.mgcm_step_phase(h, ph), "mgcm_step_phase(%d)" % ph)
        with torch.cuda.stream(s):
            check(L.mgcm_begin_steps(h), "mgcm_begin_steps")
            step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(K):
                step()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(3):
            with torch.cuda.stream(s):
                e0.record(s)
                g.replay()
                e1.record(s)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / K)
        rows.append({"gpus": N, "tiles": nT, "ms_per_step_without_cg2d": best})
        del g
        check(L.mgcm_set_stream(h, None), "mgcm_set_stream")
        m.close()
    out["partition"] = rows
    base = rows[0]["ms_per_step_without_cg2d"]
    cg = out["resident_cg2d_ms"]
    for r in rows:
        # Amdahl with the CG2D at its 1-GPU time (a lower bound: its hand-offs cross xGMI at N > 1)
        # and the collectives left out
        r["projected_ms_per_step_bound"] = r["ms_per_step_without_cg2d"] + cg
        r["projected_speedup_bound"] = (base + cg) / r["projected_ms_per_step_bound"]
        r["work_ratio"] = base / r["ms_per_step_without_cg2d"]
        r["tile_ratio"] = nt / r["tiles"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
