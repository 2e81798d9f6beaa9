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


def test_advect_xy_ab3_c4_oracle_matches_reference_output(golden_dir):
    """verification/advect_xy/input.ab3_c4 (results/output.ab3_c4.txt): theta and salt with the
    centred 4th-order scheme (GAD_C4_ADV_X/Y) stepped by ADAMS_BASHFORTH3, 100 steps, monitor
    every 10: min/max/mean/sd of both tracers at print precision."""
    from mitgcm_amd import configs
    from oracle.harness import oracle_from_config
    gold = json.load(open(os.path.join(golden_dir, "advect_xy", "monitor.ab3_c4.json")))
    o, g = oracle_from_config(configs.advect_xy_ab3_c4)
    worst = (99.0, None)
    for n in range(0, 101):
        if n > 0:
            o.forward_step()
        if n % 10:
            continue
        gs = gold[n // 10]
        assert gs["time_tsnumber"] == n
        for tr in ("theta", "salt"):
            st = o.stats(o.arr(tr), 1, o.arr("hFacC"), 1, o.arr("maskInC"), o.arr("rA"), o.arr("drF")[:1].copy())
            for v, k in zip(st[:4], ("min", "max", "mean", "sd")):
                d = digits(v, gs["dynstat_%s_%s" % (tr, k)])
                if d < worst[0]:
                    worst = (d, (n, tr, k, v, gs["dynstat_%s_%s" % (tr, k)]))
    print("advect_xy ab3_c4 oracle vs output.ab3_c4.txt: worst %.2f digits at %s" % (worst[0], worst[1]))
    assert worst[0] >= 12.0, worst
