"""GPU parity of CG2D_SR (model/src/cg2d_sr.F; solve_for_pressure.F selects it with
useSRCGSolver): the single-reduction conjugate gradient in k_cg2d_bxy<..., SR> on BASELINE
config 2 (global_ocean.90x40x15) with useSRCGSolver = 1.

The multi-workgroup solver runs it too (kernels_cg2d_mwg.hip, one grid hand-off per
iteration): config 3 on the cube below, config 2 in tests/test_gpu_cg2d_mwg.py.

Bars: 10 steps against the oracle's CG2D_SR summing in the device's order
(mgcm_cg2d_sum_plan -> oracle_set_sum_plan): iteration counts, residuals and the state arrays
identical, bit for bit; against the oracle's CG2D_SR in the reference's order: the same
iteration counts and >= 10 digits on every dynstat value.  No reference output in the tree
runs useSRCGSolver (parity unpinned against the reference; tests/test_oracle_cg2d_sr.py checks
the oracle's SR against its standard CG2D)."""
import numpy as np
import pytest

from conftest import digits

pytestmark = pytest.mark.gpu
OVER = {"useSRCGSolver": 1}


def test_ocean90_cg2d_sr_10_steps():
    from mitgcm_amd import configs
    from mitgcm_amd.model import dynstat
    from oracle.harness import ocean90_oracle
    m = configs.make_model(configs.global_ocean_90x40x15, params_over=OVER)
    o, g = ocean90_oracle(params_over=OVER)
    od, _ = ocean90_oracle(params_over=OVER)
    plan, NT, PPT, NG = m.cg2d_sum_plan()
    od.set_sum_plan(plan, NT, PPT, NG, fma=m.cg2d_fma())
    worst = (99.0, None)
    its = []
    for step in range(1, 11):
        m.forward_step(1)
        o.forward_step()
        od.forward_step()
        md = m.solve_stats()
        md.update(dynstat(m))
        so, sd = o.dynstat(), od.dynstat()
        its.append(md["cg2d_iters"])
        assert md["cg2d_iters"] == so["cg2d_iters"], (step, md["cg2d_iters"], so["cg2d_iters"])
        for k, v in md.items():
            if k in sd:
                assert v == sd[k], ("device-order oracle", step, k, v, sd[k])
            if k in so and not k.startswith("cg2d"):
                worst = min(worst, (digits(v, so[k]), (step, k)))
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    for n in ("uVel", "vVel", "wVel", "theta", "salt", "etaN", "etaH"):
        dev = m.get(n)
        ref = np.array(od.arr(n)).reshape(dev.shape)
        assert np.array_equal(dev[inner], ref[inner]), (n, np.abs(dev - ref)[inner].max())
    m.close()
    print("ocean90 CG2D_SR 10 steps: iterations %s; device == device-order oracle bit for bit; "
          "vs reference-order oracle %.2f digits at %s" % ((its,) + worst))
    assert worst[0] >= 10.0, worst


def test_cs32x15_cg2d_sr_multi_workgroup():
    """CG2D_SR in the multi-workgroup solver on the cube (BASELINE config 3: 6 faces, EXCH2
    maps, parts pinned to one XCD): one grid hand-off per iteration; 4 steps bit-identical to
    the oracle's CG2D_SR summing in the device's order (iterations, residuals, every dynstat
    value)."""
    from mitgcm_amd import configs
    from mitgcm_amd.model import dynstat
    from oracle.harness import cs32x15_oracle
    m = configs.make_model(configs.global_ocean_cs32x15, params_over=OVER)
    assert m.cg2d_kernel() == "mwg"
    od, g = cs32x15_oracle(params_over=OVER)
    plan, NT, PPT, NG = m.cg2d_sum_plan()
    od.set_sum_plan(plan, NT, PPT, NG, fma=m.cg2d_fma())
    its = []
    for step in range(1, 5):
        m.forward_step(1)
        od.forward_step()
        md = m.solve_stats()
        md.update(dynstat(m))
        sd = od.dynstat()
        its.append(md["cg2d_iters"])
        for k, v in md.items():
            if k in sd:
                assert v == sd[k], ("device-order oracle", step, k, v, sd[k])
    m.close()
    print("cs32x15 CG2D_SR on the multi-workgroup solver: iterations %s, bit for bit" % its)
