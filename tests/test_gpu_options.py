"""GPU parity of the options outside the five BASELINE namelists that the device path
implements on top of them:

  * implicitViscosity: MOM_U_IMPLICIT_R / MOM_V_IMPLICIT_R (pkg/mom_common/mom_u_implicit_r.F,
    dynamics.F:568-580) on the flux-form (tutorial_baroclinic_gyre) and vector-invariant
    (global_ocean.cs32x15: cube, r*, stagger) momentum paths;
  * implicitViscosity with the CD scheme: IMPLDIFF on the D-grid velocities (impldiff.F,
    dynamics.F:614-634) on global_ocean.90x40x15;
  * tempAdvScheme = 30: DST3 without limiter (gad_dst3_adv_x.F:71-118, gad_dst3_adv_r.F:70-119)
    through the multi-dimensional split, lat-lon (baroclinic gyre) and cube (cs32x15).

Bars: one DYNAMICS / THERMODYNAMICS call from an oracle-stepped state bit-exact against the
oracle, and 6 steps within 1e-10 (relative to each field's maximum) of the oracle.  These
variants have no reference output in the tree (parity unpinned against the reference); the
oracle restatements cite the reference lines they follow.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gyre(scheme=2, **over):
    from mitgcm_amd import configs

    def cfg(**kw):
        g, params, state = configs.baroclinic_gyre(tempAdvScheme=scheme, **kw)
        params.update(over)
        return g, params, state
    return cfg


def _put_state(m, o, names):
    from mitgcm_amd._lib import lib
    for n in names:
        m.put(n, np.array(o.arr(n)))
    lib().mgcm_set_param(m.h, b"myIter", float(o.get("myIter")))


@pytest.mark.parametrize("scheme", [2, 33])
def test_gyre_implicit_viscosity_dynamics_bitexact(scheme):
    from mitgcm_amd import configs
    from oracle.harness import oracle_from_config
    cfg = _gyre(scheme, implicitViscosity=1)
    o, g = oracle_from_config(cfg)
    for _ in range(3):
        o.forward_step()
    o.L.oracle_oceanic_phys(o.h)
    m = configs.make_model(cfg)
    _put_state(m, o, ("uVel", "vVel", "wVel", "guNm1", "gvNm1", "etaN", "rhoInSitu"))
    m.dynamics()
    o.L.oracle_dynamics(o.h)
    for n in ("gU", "gV", "guNm1", "gvNm1"):
        dev, ref = m.get(n), np.array(o.arr(n))
        assert np.array_equal(dev, ref), (n, np.abs(dev - ref).max())
    m.close()


def test_gyre_dst3_scheme30_thermodynamics_bitexact():
    from mitgcm_amd import configs
    from oracle.harness import oracle_from_config
    cfg = _gyre(30)
    o, g = oracle_from_config(cfg)
    for _ in range(3):
        o.forward_step()
    o.arr("theta")[:, 1, 10:16, 8:20] += 12.0
    m = configs.make_model(cfg)
    _put_state(m, o, ("uVel", "vVel", "wVel", "theta", "gtNm1", "etaN"))
    m.thermodynamics()
    o.L.oracle_oceanic_phys(o.h)
    o.L.oracle_thermodynamics(o.h)
    inner = (slice(None), slice(None)) + g.sl(1, g.sNx, 1, g.sNy)
    dev, ref = m.get("theta")[inner], np.array(o.arr("theta"))[inner]
    assert np.array_equal(dev, ref), np.abs(dev - ref).max()
    m.close()


@pytest.mark.parametrize("scheme,over", [(30, {}), (30, {"implicitViscosity": 1})])
def test_gyre_variants_6_steps_vs_oracle(scheme, over):
    from mitgcm_amd import configs
    from oracle.harness import oracle_from_config
    cfg = _gyre(scheme, **over)
    o, g = oracle_from_config(cfg)
    m = configs.make_model(cfg)
    for _ in range(6):
        o.forward_step()
    m.forward_step(6)
    m.sync()
    for n in ("uVel", "vVel", "wVel", "theta", "etaN"):
        dev, ref = m.get(n), np.array(o.arr(n)).reshape(m.get(n).shape)
        sc = np.abs(ref).max()
        assert np.abs(dev - ref).max() <= 1e-10 * sc, (n, np.abs(dev - ref).max(), sc)
    m.close()


def _cs_model(**over):
    from mitgcm_amd import configs
    return configs.make_model(configs.global_ocean_cs32x15, params_over=over)


def test_cs32x15_implicit_viscosity_vecinv_dynamics_bitexact():
    from oracle.harness import cs32x15_oracle
    from test_gpu_cs32x15 import STATE, _cmp
    o, g = cs32x15_oracle(params_over={"implicitViscosity": 1})
    for _ in range(2):
        o.forward_step()
    o.L.oracle_fields_load(o.h)
    o.L.oracle_oceanic_phys(o.h)
    m = _cs_model(implicitViscosity=1)
    _put_state(m, o, STATE + ("rhoInSitu", "fu", "fv"))
    m.dynamics()
    o.L.oracle_dynamics(o.h)
    inner = (Ellipsis,) + g.sl(1, g.sNx + 1, 1, g.sNy + 1)
    bad = _cmp(m, o, ("gU", "gV", "guNm1", "gvNm1"), inner)
    m.close()
    assert not bad, bad


def test_cs32x15_dst3_scheme30_and_implicit_viscosity_4_steps_vs_oracle():
    from oracle.harness import cs32x15_oracle
    over = {"implicitViscosity": 1, "tempAdvScheme": 30, "tempVertAdvScheme": 30, "saltAdvScheme": 30,
            "saltVertAdvScheme": 30, "GM_AdvForm": 0, "GM_skewflx": 1.0}
    o, g = cs32x15_oracle(params_over=over)
    m = _cs_model(**over)
    for _ in range(4):
        o.forward_step()
    m.forward_step(4)
    m.sync()
    for n in ("uVel", "vVel", "theta", "salt", "etaN"):
        dev, ref = m.get(n), np.array(o.arr(n)).reshape(m.get(n).shape)
        sc = np.abs(ref).max()
        assert np.abs(dev - ref).max() <= 1e-10 * sc, (n, np.abs(dev - ref).max(), sc)
    m.close()


def test_overlap_trial_leaves_the_state_untouched():
    """The THERMODYNAMICS-overlap auto-selection (model.hip ovl_trial) times both step graphs
    on the live state and copies it back: a 10-step graph batch after it equals ten single
    steps of a model that never ran the trial, bit for bit."""
    from mitgcm_amd import configs
    from mitgcm_amd._lib import lib
    cfg = _gyre(33)
    a, b = configs.make_model(cfg), configs.make_model(cfg)
    a.forward_step(10)
    for _ in range(10):
        b.forward_step(1)
    a.sync()
    b.sync()
    assert lib().mgcm_get_param(a.h, b"overlap") in (0.0, 1.0)
    assert lib().mgcm_get_param(b.h, b"overlap") == -1.0   # b never ran a graph batch
    for n in ("uVel", "vVel", "wVel", "theta", "salt", "etaN"):
        assert np.array_equal(a.get(n), b.get(n)), n
    assert a.solve_stats() == b.solve_stats()
    a.close()
    b.close()


# implicitViscosity with the CD scheme (BASELINE config 2 carries useCDscheme): after
# MOM_U/V_IMPLICIT_R on gU, gV, DYNAMICS runs IMPLDIFF on the D-grid velocities vVelD
# (kappaRU, recip_hFacW) and uVelD (kappaRV, recip_hFacS) (dynamics.F:614-634, impldiff.F);
# k_impldiff_cd against the oracle's restatement: one DYNAMICS bit-exact on the ring
# 0..sN+1, and 4 steps within 1e-10 of each field's maximum.
def test_ocean90_cd_implicit_viscosity_dynamics_bitexact():
    from mitgcm_amd import configs
    from oracle.harness import ocean90_oracle
    over = {"implicitViscosity": 1}
    o, g = ocean90_oracle(params_over=over)
    for _ in range(2):
        o.forward_step()
    o.L.oracle_fields_load(o.h)
    o.L.oracle_oceanic_phys(o.h)
    m = configs.make_model(lambda: configs.global_ocean_90x40x15(params_over=over))
    from test_gpu_ocean90 import STATE
    _put_state(m, o, STATE + ("rhoInSitu", "fu", "fv"))
    m.dynamics()
    o.L.oracle_dynamics(o.h)
    ring = (Ellipsis,) + g.sl(0, g.sNx + 1, 0, g.sNy + 1)
    bad = []
    for n in ("gU", "gV", "uVelD", "vVelD"):
        dev, ref = m.get(n), np.array(o.arr(n)).reshape(m.get(n).shape)
        if not np.array_equal(dev[ring], ref[ring]):
            bad.append((n, float(np.abs(dev[ring] - ref[ring]).max())))
    m.close()
    assert not bad, bad


def test_ocean90_cd_implicit_viscosity_4_steps_vs_oracle():
    from mitgcm_amd import configs
    from oracle.harness import ocean90_oracle
    over = {"implicitViscosity": 1}
    o, g = ocean90_oracle(params_over=over)
    m = configs.make_model(lambda: configs.global_ocean_90x40x15(params_over=over))
    for _ in range(4):
        o.forward_step()
    m.forward_step(4)
    m.sync()
    for n in ("uVel", "vVel", "theta", "salt", "etaN", "uVelD", "vVelD"):
        dev, ref = m.get(n), np.array(o.arr(n)).reshape(m.get(n).shape)
        sc = np.abs(ref).max()
        assert np.abs(dev - ref).max() <= 1e-10 * sc, (n, np.abs(dev - ref).max(), sc)
    m.close()


# Options the device does not restate are refused at mgcm_init with the reason, never run
# silently: ADAMS_BASHFORTH3 with momentum stepping or from
# a pickup, the U3 / C4 schemes on a pkg/exch2 topology, a scheme the device does not carry.
@pytest.mark.parametrize("case", ["ab3_momentum", "ab3_pickup", "c4_cube", "os7mp"])
def test_unsupported_options_refused(case):
    from mitgcm_amd import configs
    from mitgcm_amd._lib import MgcmError

    def cfg():
        if case == "c4_cube":
            g, p, s = configs.global_ocean_cs32x15(sNy=32)[:3]
            p.update(tempAdvScheme=4, tempVertAdvScheme=4)
            return g, p, s
        g, p, s = configs.advect_xy_ab3_c4()
        if case == "ab3_momentum":
            p["momStepping"] = 1
        elif case == "ab3_pickup":
            p["nIter0"] = 10
        elif case == "os7mp":
            p.update(useAB3=0, saltAdvScheme=7, saltVertAdvScheme=7)
        return g, p, s
    with pytest.raises(MgcmError) as e:
        configs.make_model(cfg)
    msg = str(e.value)
    want = {"ab3_momentum": "ADAMS_BASHFORTH3", "ab3_pickup": "ADAMS_BASHFORTH3", "c4_cube": "schemes 3 / 4",
            "os7mp": "saltAdvScheme 7"}[case]
    assert want in msg, msg
