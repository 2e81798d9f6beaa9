"""GPU parity of BASELINE config 5, the synthetic LLC (the 5 lat-lon-cap
facets of data.exch2.llc_120_5f, pkg/exch2 halo maps with rotated facets, the
multi-workgroup CG2D), through the C-ABI.

Bars:
  * LLC-30 (13 tiles of 30 x 30, 10 levels, OL = 4): 8 steps bit-identical to the oracle
    summing CG2D in the device's order, with the flat and the k-march tracer kernels;
    cg2d_iters identical to the reference-order oracle;
  * LLC-90 as benched (13 tiles of 90 x 90, 50 levels): the initial state round-trips; 4
    steps' monitored values (dynstat, CG2D residuals and iterations) and the final fields
    are bit-identical to the device-order oracle's at full size, and every iteration count
    equals the reference-order oracle's.  The synthetic set-up has no reference output: parity
    unpinned against the reference, pinned device-vs-oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("march", [None, "tracer", "tracer:v1", "tracer:fwd", "tracer:fwdback", "tracer:rows", "vi",
                                   "vi:kc3", "vi:generic", "fuse:29", "fuse:45", "fuse:77"])
def test_llc30_8_steps_bitexact_vs_device_order_oracle(march, monkeypatch):
    """march: the LLC-90 default kernel forms forced on LLC-30 (too small to pick them by
    itself).  "tracer": the tracer right-hand side as the k-march (MGCM_TRACER_MARCH=1, five
    level chunks) instead of the flat kernel; ":v1" the other forms of the 16-byte switches --
    the one-column k-march (the default is its two-column form) and the two-column
    DO_OCEANIC_PHYS forced (at full size the default; below 2^21 points the one-column form
    runs).  "vi": MOM_VECINV as the k-march in its compile-time specialisation
    (k_mom_vi_m2<32, 8, LLC options>; ":kc3" in chunks of 3 levels), "vi:generic" the generic k-march that serves option sets
    without an instantiation (MGCM_VI_KERNEL=march | march_generic).  "fuse:MASK": the
    MGCM_STEP_FUSE launch fusions (29: the opt-in k_phys_phi pass; 45: the opt-in
    EXCH(cg2d_x) + etaN beside the correction step; 77: the tracers' halo exchange on their own
    stream)."""
    if march in ("tracer:fwd", "tracer:fwdback", "tracer:rows"):   # the implicit solve's forward sweep inside the
        # whole-column march, then the back substitution as a kernel of its own (2) or by the same
        # threads (3, its column pairs dealt evenly over the workgroups); "rows": (3) with whole
        # tile rows per workgroup (MGCM_TRACER_MARCH2=1)
        monkeypatch.setenv("MGCM_TRACER_MARCH", "2" if march == "tracer:fwd" else "3")
        if march == "tracer:rows":
            monkeypatch.setenv("MGCM_TRACER_MARCH2", "1")
        march = None
    if march and march.endswith(":v1"):
        monkeypatch.setenv("MGCM_TRACER_MARCH2", "0")
        monkeypatch.setenv("MGCM_PHYS_V2", "2")
        march = march[:-3]
    if march and march.startswith("fuse:"):   # MGCM_STEP_FUSE mask: 29 adds DO_OCEANIC_PHYS + CALC_PHI_HYD in one pass
        monkeypatch.setenv("MGCM_STEP_FUSE", march.split(":")[1])
    elif march and march.startswith("vi"):
        monkeypatch.setenv("MGCM_VI_KERNEL", "march_generic" if march.endswith("generic") else "march")
        if march.endswith(":kc3"):   # ragged level chunks (3, 3, 3, 1) instead of the whole column
            monkeypatch.setenv("MGCM_VI_KC", "3")
    elif march == "tracer":
        monkeypatch.setenv("MGCM_TRACER_MARCH", "1")
    from mitgcm_amd import configs
    from mitgcm_amd.model import dynstat
    from oracle.harness import oracle_from_config
    cfg = lambda: configs.llc_synthetic(n=30, Nr=10)
    m = configs.make_model(cfg)
    assert m.cg2d_kernel() == "mwg"
    plan, NT, PPT, NG = m.cg2d_sum_plan()
    od, g = oracle_from_config(cfg)
    od.set_sum_plan(plan, NT, PPT, NG, fma=m.cg2d_fma())
    o_ref, _ = oracle_from_config(cfg)
    for step in range(1, 9):
        m.forward_step(1)
        od.forward_step()
        o_ref.forward_step()
        md = m.solve_stats()
        md.update(dynstat(m))
        dd = od.dynstat()
        assert md["cg2d_iters"] == dd["cg2d_iters"] == int(o_ref.get("numIters")), step
        for k, v in md.items():
            if k in dd:
                assert v == dd[k], (step, k, v, dd[k])
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    for n in ("uVel", "vVel", "wVel", "theta", "salt", "etaN"):
        dev = m.get(n)
        ref = np.array(od.arr(n)).reshape(dev.shape)
        assert np.array_equal(dev[inner], ref[inner]), (n, np.abs(dev - ref)[inner].max())
    m.close()


@pytest.mark.parametrize("pairs", [None, "1"])
def test_llc90_full_size_steps(pairs, monkeypatch):
    """pairs "1": the tracers' whole-column march with whole tile rows per workgroup
    (MGCM_TRACER_MARCH2=1) instead of its column pairs dealt evenly over the workgroups (the
    default)."""
    if pairs:
        monkeypatch.setenv("MGCM_TRACER_MARCH2", pairs)
    from mitgcm_amd import configs
    from mitgcm_amd.model import dynstat
    from oracle.harness import oracle_from_config
    g, params, state = configs.llc_synthetic()
    m = configs.make_model(lambda: (g, params, state))
    assert np.array_equal(m.get("theta"), state["theta"])
    # the first step against the oracle at full size: iterations equal to the reference-order
    # oracle's, and every monitored value bit-identical to the device-order oracle's
    plan, NT, PPT, NG = m.cg2d_sum_plan()
    od, _ = oracle_from_config(configs.llc_synthetic)
    od.set_sum_plan(plan, NT, PPT, NG, fma=m.cg2d_fma())
    o_ref, _ = oracle_from_config(configs.llc_synthetic)
    iters = []
    for step in range(1, 5):   # 4 steps, each compared with both oracles
        m.forward_step(1)
        od.forward_step()
        o_ref.forward_step()
        md = m.solve_stats()
        md.update(dynstat(m))
        dd = od.dynstat()
        assert md["cg2d_iters"] == dd["cg2d_iters"] == int(o_ref.get("numIters")), (
            step, md["cg2d_iters"], dd["cg2d_iters"], o_ref.get("numIters"))
        for k, v in md.items():
            if k in dd:
                assert v == dd[k], (step, k, v, dd[k])
        iters.append(md["cg2d_iters"])
    g = m.g
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    for n in ("uVel", "vVel", "wVel", "theta", "salt", "etaN"):
        dev = m.get(n)
        ref = np.array(od.arr(n)).reshape(dev.shape)
        assert np.array_equal(dev[inner], ref[inner]), (n, np.abs(dev - ref)[inner].max())
    st = m.solve_stats()
    assert all(0 < i < params["cg2dMaxIters"] for i in iters), iters
    assert st["cg2d_last_res"] < st["cg2d_init_res"]
    for n in ("uVel", "vVel", "theta", "etaN"):
        assert np.isfinite(m.get(n)).all(), n
    m.close()


def test_llc30_thermodynamics_overlap_bit_identical(monkeypatch):
    """THERMODYNAMICS on the second stream (forced on: under the linear free surface forked
    after DYNAMICS, beside the pressure solve, joined before the correction step) against one
    stream (forced off): 8 graph-replayed steps bit-identical."""
    from mitgcm_amd import configs
    cfg = lambda: configs.llc_synthetic(n=30, Nr=10)
    out = {}
    for mode in ("on", "off"):
        monkeypatch.setenv("MGCM_OVERLAP", "1" if mode == "on" else "0")
        m = configs.make_model(cfg)
        m.forward_step(8)
        m.sync()
        out[mode] = {n: m.get(n) for n in ("uVel", "vVel", "wVel", "theta", "salt", "etaN")}
        out[mode]["iters"] = [int(v) for v in m.solve_history(8)[0]]
        m.close()
    for n in out["on"]:
        assert np.array_equal(out["on"][n], out["off"][n]), n
