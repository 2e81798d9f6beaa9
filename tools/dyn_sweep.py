#!/usr/bin/env python3
"""Time DYNAMICS (k_phi_hyd + momentum kernels) on a bench workload with HIP events:
    python tools/dyn_sweep.py [config] [reps]
Environment knobs of the momentum launch (MGCM_VI_POINT, MGCM_VI_KC) select variants."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "llc90_synthetic"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import bench
    from mitgcm_amd import configs
    m = configs.make_model(bench.config_fn(cfg))
    m.forward_step(2)
    m.sync()
    m.kernel_timing(True)
    for _ in range(reps):
        m.dynamics()
    ms, n = m.kernel_ms("mom_step")
    m.kernel_timing(False)
    print("%s VI_POINT=%s VI_KC=%s: DYNAMICS %.1f us (%d launches)" % (
        cfg, os.environ.get("MGCM_VI_POINT", "-"), os.environ.get("MGCM_VI_KC", "-"), ms * 1e3, n), flush=True)
    m.close()


if __name__ == "__main__":
    main()
