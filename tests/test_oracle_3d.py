"""The oracle's 3-D path (DO_OCEANIC_PHYS + THERMODYNAMICS/GAD C2 + CALC_PHI_HYD
+ spherical metric terms + exactConserv) pinned against the reference's own
committed output: verification/tutorial_baroclinic_gyre/results/output.txt
(4 tiles of 31x31x15 on a spherical-polar grid), parsed into
tests/golden/tutorial_baroclinic_gyre/monitor.json."""
import json
import os

from conftest import digits


def _params(golden_dir):
    return json.load(open(os.path.join(golden_dir, "tutorial_baroclinic_gyre", "params.json")))


def test_baroclinic_params_pinned(golden_dir):
    """What configs.baroclinic_gyre assumes == the reference's resolved dump."""
    from mitgcm_amd import configs
    p = _params(golden_dir)
    g, params, state = configs.baroclinic_gyre()
    for name in ("deltaTMom", "deltaTFreeSurf", "abEps", "rhoConst", "rhoNil", "tAlpha", "sBeta", "ivdc_kappa",
                 "diffKhT", "sideDragFactor", "rSphere"):
        assert float(p[name]) == params[name], name
    assert float(p["viscAh"]) == params["viscAhD"] == params["viscAhZ"] and float(p["viscA4"]) == 0.0
    assert [float(x) for x in p["viscArNr"]] == [params["viscAr"]] * g.Nr
    assert [float(x) for x in p["diffKrNrT"]] == [params["diffKrT"]] * g.Nr
    assert [float(x.rstrip(",")) for x in p["tRef"]] == list(state["tRef"])
    assert [float(x) for x in p["dTtracerLev"]] == [params["deltaTtracer"]] * g.Nr
    assert int(p["tempAdvScheme"]) == 2 and int(p["tempVertAdvScheme"]) == 2
    assert int(p["selectCoriMap"][0]) == 2 and p["useNHMTerms"] == "F"
    for flag in ("implicitDiffusion", "exactConserv", "tempStepping", "tempForcing", "AdamsBashforthGt",
                 "no_slip_sides"):
        assert p[flag] == "T", flag
    for flag in ("saltStepping", "staggerTimeStep", "AdamsBashforth_T", "useRealFreshWaterFlux", "no_slip_bottom",
                 "implicitViscosity", "useCDscheme", "quasiHydrostatic", "nonHydrostatic", "vectorInvariantMomentum"):
        assert p[flag] == "F", flag
    assert int(p["nonlinFreeSurf"][0]) == 0 and int(p["select_rStar"]) == 0 and int(p["tracForcingOutAB"]) == 0
    assert float(p["tauThetaClimRelax"]) == 2592000.0
    assert abs(float(p["omega"]) - g.omega) <= 1e-15 * g.omega


def test_baroclinic_oracle_matches_reference_output(golden_dir):
    from mitgcm_amd import configs
    from oracle.harness import oracle_from_config
    gold = json.load(open(os.path.join(golden_dir, "tutorial_baroclinic_gyre", "monitor.json")))
    o, g = oracle_from_config(configs.baroclinic_gyre)
    worst = (99.0, None)
    for n in range(1, 11):
        o.forward_step()
        r = o.dynstat()
        gs = gold[n]
        assert r["cg2d_iters"] == gs["cg2d_iters"], n
        for k, v in r.items():
            if k in gs and k != "cg2d_iters":
                d = digits(v, gs[k])
                if d < worst[0]:
                    worst = (d, (n, k, v, gs[k]))
    # 14 printed significant digits: >= 13 is print precision
    assert worst[0] >= 13.0, worst
