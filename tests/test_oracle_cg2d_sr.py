"""The oracle's CG2D_SR (model/src/cg2d_sr.F, useSRCGSolver): the single-reduction
conjugate gradient against the standard CG2D on the same systems.  No reference output in the
tree uses useSRCGSolver with a configuration restated here (parity unpinned against the
reference); the checks are the algorithm's own: both converge to the tolerance, the
iteration counts agree within one, the solutions agree to the tolerance's scale, and in exact
arithmetic the two produce the same iterates (the first step is the standard one)."""
import numpy as np


def _solve(cfg, sr, nsteps=2):
    from oracle.harness import ocean90_oracle
    o, g = ocean90_oracle()
    o.set(useSRCGSolver=1 if sr else 0)
    for _ in range(nsteps):
        o.forward_step()
    return o, g


def test_cg2d_sr_matches_standard_cg2d_on_config2():
    o0, g = _solve(None, False)
    o1, _ = _solve(None, True)
    s0, s1 = o0.dynstat(), o1.dynstat()
    assert abs(s0["cg2d_iters"] - s1["cg2d_iters"]) <= 1, (s0["cg2d_iters"], s1["cg2d_iters"])
    assert s1["cg2d_last_res"] < 1e-6
    eta0, eta1 = np.array(o0.arr("etaN")), np.array(o1.arr("etaN"))
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    assert np.abs(eta0[inner] - eta1[inner]).max() <= 1e-9 * np.abs(eta0[inner]).max()


def test_cg2d_sr_direct_solve():
    from mitgcm_amd import configs
    from oracle.harness import oracle_from_config
    o, g = oracle_from_config(configs.baroclinic_gyre)
    rng = np.random.default_rng(5)
    b = np.zeros((g.nTiles, g.ny, g.nx))
    inner = g.sl(1, g.sNx, 1, g.sNy)
    for t in range(g.nTiles):
        b[t][inner] = rng.standard_normal((g.sNy, g.sNx)) * g.f["maskInC"][t][inner]
    x0 = np.zeros_like(b)
    xa, fa, _, la, ita, _ = o.cg2d(b, x0, 1000, -1)
    o.set(useSRCGSolver=1)
    xb, fb, _, lb, itb, _ = o.cg2d(b, x0, 1000, -1)
    assert fa == fb                    # same initial residual
    assert abs(ita - itb) <= 1, (ita, itb)
    sc = max(np.abs(xa[t][inner]).max() for t in range(g.nTiles))
    assert max(np.abs(xa[t][inner] - xb[t][inner]).max() for t in range(g.nTiles)) <= 1e-8 * sc
