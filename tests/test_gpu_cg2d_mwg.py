"""The multi-workgroup CG2D (kernels_cg2d_mwg.hip) through the C-ABI.

Bars:
  * BASELINE config 2 (90x40x15, 1 tile) with the single-workgroup solvers switched off
    (row-strip parts of NT x OPT points: 4 at the default 256 x 4): 6 steps bit-identical to the oracle summing CG2D in the device's
    order (mgcm_cg2d_sum_plan: per-thread terms, pairwise trees, partials in part order);
  * the same solve with every part pinned to one XCD and with the parts spread over the
    chip: bit-identical (the sums do not depend on placement);
  * cg2d_iters identical to the reference-order oracle.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ocean90_mwg(spread=False):
    from mitgcm_amd import configs
    env = {"MGCM_CG2D_NOBLOCKED": "1"}
    if spread:
        env["MGCM_CG2D_SPREAD"] = "1"
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = configs.make_model(configs.global_ocean_90x40x15)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return m


def test_mwg_ocean90_bitexact_vs_device_order_oracle():
    from mitgcm_amd._lib import lib
    from oracle.harness import ocean90_oracle
    m = _ocean90_mwg()
    assert m.cg2d_kernel() == "mwg"
    plan, NT, PPT, NG = m.cg2d_sum_plan()
    parts = -(-40 // ((NT * PPT) // 90))   # row strips of the 90 x 40 tile, NT*PPT points each
    assert lib().mgcm_get_param(m.h, b"cg2dParts") == float(parts) and NG == parts, (NG, parts)
    od, g = ocean90_oracle()
    od.set_sum_plan(plan, NT, PPT, NG, fma=m.cg2d_fma())
    o_ref, _ = ocean90_oracle()
    for step in range(1, 7):
        m.forward_step(1)
        od.forward_step()
        o_ref.forward_step()
        st = m.solve_stats()
        assert st["cg2d_iters"] == int(od.get("numIters")) == int(o_ref.get("numIters")), step
        assert st["cg2d_init_res"] == od.get("firstResidual"), (step, st["cg2d_init_res"], od.get("firstResidual"))
        assert st["cg2d_last_res"] == od.get("lastResidual"), step
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    for n in ("uVel", "vVel", "theta", "salt", "etaN"):
        dev = m.get(n)
        ref = np.array(od.arr(n)).reshape(dev.shape)
        assert np.array_equal(dev[inner], ref[inner]), (n, np.abs(dev - ref)[inner].max())
    m.close()


def test_mwg_pinned_vs_spread_identical():
    a = _ocean90_mwg(spread=False)
    b = _ocean90_mwg(spread=True)
    a.forward_step(3)
    b.forward_step(3)
    for n in ("etaN", "uVel", "theta"):
        assert np.array_equal(a.get(n), b.get(n)), n
    for k in range(3):
        assert a.solve_stats(back=k) == b.solve_stats(back=k)
    a.close()
    b.close()


def test_mwg_min_residual_solution_vs_oracle():
    """cg2dUseMinResSol (cg2d.F:148-155, 190-193, 338-347, 358-368) in the multi-workgroup
    solver: with the iterations capped below convergence (cg2dMaxIters = 12) the solve keeps
    the lowest-residual iterate; 4 steps bit-identical to the device-order oracle with the
    same switches, and the recorded nIterMin / minResidualSq equal the oracle's."""
    from mitgcm_amd._lib import lib
    from oracle.harness import ocean90_oracle
    m = _ocean90_mwg()
    assert m.cg2d_kernel() == "mwg"
    L = lib()
    for k, v in (("cg2dUseMinResSol", 1), ("cg2dMaxIters", 12)):
        assert L.mgcm_set_param(m.h, k.encode(), float(v)) == 0, k
    plan, NT, PPT, NG = m.cg2d_sum_plan()
    od, g = ocean90_oracle()
    od.set(cg2dUseMinResSol=1, cg2dMaxIters=12)
    od.set_sum_plan(plan, NT, PPT, NG, fma=m.cg2d_fma())
    used_min = 0
    for step in range(1, 5):
        m.forward_step(1)
        od.forward_step()
        st = m.solve_stats()
        assert st["cg2d_iters"] == int(od.get("numIters")) == 12, step
        assert st["cg2d_last_res"] == od.get("lastResidual"), step
        mr, nmin = m.solve_minres()
        # the oracle keeps SQRT(minResidualSq), as SOLVE_FOR_PRESSURE prints it
        assert np.sqrt(mr) == od.get("minResidualSq"), (step, mr, od.get("minResidualSq"))
        assert nmin == int(od.get("nIterMin")), (step, nmin, od.get("nIterMin"))
        used_min += int(nmin < 12)
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    for n in ("uVel", "vVel", "theta", "etaN"):
        dev = m.get(n)
        ref = np.array(od.arr(n)).reshape(dev.shape)
        assert np.array_equal(dev[inner], ref[inner]), (n, np.abs(dev - ref)[inner].max())
    m.close()
    print("mwg min-residual: %d of 4 solves kept an earlier iterate" % used_min)


@pytest.mark.parametrize("minres", [0, 1])
def test_mwg_cg2d_sr_vs_oracle(minres):
    """useSRCGSolver (CG2D_SR, cg2d_sr.F) in the multi-workgroup solver: one grid hand-off per
    iteration (the three sums with the rings' v = A y), the rings' r and q kept as copies.
    6 steps of config 2 bit-identical to the oracle's CG2D_SR summing in the device's order,
    iterations, residuals and (minres) the min-residual record equal; with minres the
    iterations are capped below convergence so the lowest-residual iterate is used."""
    from mitgcm_amd._lib import lib
    from oracle.harness import ocean90_oracle
    m = _ocean90_mwg()
    assert m.cg2d_kernel() == "mwg"
    L = lib()
    sets = {"useSRCGSolver": 1}
    if minres:
        sets.update(cg2dUseMinResSol=1, cg2dMaxIters=12)
    for k, v in sets.items():
        assert L.mgcm_set_param(m.h, k.encode(), float(v)) == 0, k
    plan, NT, PPT, NG = m.cg2d_sum_plan()
    od, g = ocean90_oracle()
    od.set(**sets)
    od.set_sum_plan(plan, NT, PPT, NG, fma=m.cg2d_fma())
    its = []
    for step in range(1, 7 if not minres else 5):
        m.forward_step(1)
        od.forward_step()
        st = m.solve_stats()
        its.append(st["cg2d_iters"])
        assert st["cg2d_iters"] == int(od.get("numIters")), (step, st, od.get("numIters"))
        assert st["cg2d_init_res"] == od.get("firstResidual"), step
        assert st["cg2d_last_res"] == od.get("lastResidual"), (step, st["cg2d_last_res"], od.get("lastResidual"))
        if minres:
            mr, nmin = m.solve_minres()
            assert (np.sqrt(mr), nmin) == (od.get("minResidualSq"), int(od.get("nIterMin"))), (step, mr, nmin)
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    for n in ("uVel", "vVel", "theta", "salt", "etaN"):
        dev = m.get(n)
        ref = np.array(od.arr(n)).reshape(dev.shape)
        assert np.array_equal(dev[inner], ref[inner]), (n, np.abs(dev - ref)[inner].max())
    m.close()
    print("mwg CG2D_SR (minres %d): iterations %s" % (minres, its))
