"""The oracle's multi-dimensional advection on the cubed sphere (GAD_ADVECTION's 3-pass
cube split, gad_advection.F:339-367, with FILL_CS_CORNER_TR_RL / FILL_CS_CORNER_UV_RS and
GAD_MULTIDIM_COMPRESSIBLE) pinned against the reference's committed
verification/advect_cs/results/output.txt: theta advected by a solid-body rotation
(code/ini_vel.F) on cs32, DST3 flux-limited (tempAdvScheme=33), 192 steps, monitor every
8 steps.  Bars: the initial velocity field's uvel statistics and theta min/max/mean/sd at
every monitor step >= 13 digits."""
import json
import os

from conftest import digits


def test_advect_cs_oracle_matches_reference_output(golden_dir):
    from mitgcm_amd import configs
    from oracle.harness import oracle_from_config
    gold = json.load(open(os.path.join(golden_dir, "advect_cs", "monitor.json")))
    o, g = oracle_from_config(configs.advect_cs)
    dr = o.arr("drF")[:1].copy()
    su = o.stats(o.arr("uVel"), 1, o.arr("hFacW"), 1, o.arr("maskInW"), o.arr("rAw"), dr)
    worst = (99.0, None)
    for v, k in zip(su[:4], ("min", "max", "mean", "sd")):
        worst = min(worst, (digits(v, gold[0]["dynstat_uvel_" + k]), (0, "uvel_" + k)))
    for n in range(1, 193):
        o.forward_step()
        if n % 8:
            continue
        st = o.stats(o.arr("theta"), 1, o.arr("hFacC"), 1, o.arr("maskInC"), o.arr("rA"), dr)
        gs = gold[n // 8]
        assert gs["time_tsnumber"] == n
        for v, k in zip(st[:4], ("min", "max", "mean", "sd")):
            worst = min(worst, (digits(v, gs["dynstat_theta_" + k]), (n, k, v, gs["dynstat_theta_" + k])))
    print("advect_cs 192 steps: worst digits %.2f at %s" % worst)
    assert worst[0] >= 13.0, worst
