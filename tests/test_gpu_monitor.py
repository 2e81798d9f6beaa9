"""MONITOR's dynstat block on the device (mgcm_monitor, kernels_monitor.hip) against the
host restatement in the reference's summation order (model.dynstat, MON_CALC_STATS_RL:
pkg/monitor/mon_calc_stats_rl.F), on the fields of the same device model.
Bars: min / max exact; mean, sd, del2 within 1e-12 of the field's magnitude (the device
adds tree partials per level, the reference sums each tile sequentially)."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(m):
    from mitgcm_amd.model import dynstat, monitor
    t0 = time.perf_counter()
    dev = monitor(m)
    t1 = time.perf_counter()
    ref = dynstat(m)
    bad = []
    for f in ("eta", "uvel", "vvel", "wvel", "theta", "salt"):
        scale = max(abs(ref["dynstat_%s_max" % f]), abs(ref["dynstat_%s_min" % f]), 1e-300)
        for s in ("max", "min", "mean", "sd", "del2"):
            k = "dynstat_%s_%s" % (f, s)
            if s in ("max", "min"):
                ok = dev[k] == ref[k]
            else:
                ok = abs(dev[k] - ref[k]) <= 1e-12 * max(scale, abs(ref[k]))
            if not ok:
                bad.append((k, dev[k], ref[k]))
    return bad, t1 - t0


@pytest.mark.parametrize("cfg", ["ocean90", "cs32x15", "llc30"])
def test_device_monitor_matches_reference_order(cfg):
    from mitgcm_amd import configs
    fn = {"ocean90": configs.global_ocean_90x40x15, "cs32x15": configs.global_ocean_cs32x15,
          "llc30": lambda: configs.llc_synthetic(n=30, Nr=10)}[cfg]
    m = configs.make_model(fn)
    m.forward_step(3)
    m.sync()
    bad, dt = _check(m)
    print("%s: device MONITOR %.2f ms" % (cfg, dt * 1e3))
    m.close()
    assert not bad, bad
