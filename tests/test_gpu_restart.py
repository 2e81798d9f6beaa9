"""Restart parity on the GPU (verification/testreport's tst_2+2 check):
BASELINE config 2 (global_ocean.90x40x15) stepped 4 times from the reference's pickup,
against 2 steps -> WRITE_PICKUP (mitgcm_amd/pickup.py: the MDS pickup + pickup_cd of
write_pickup.F / cd_code_write_pickup.F, downloaded from the device) -> a new model read
from that pickup at nIter0 = 36002 -> 2 steps.  Bar: bit-identical interiors of the state
and the AB histories, identical CG2D records."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = ("uVel", "vVel", "wVel", "theta", "salt", "etaN", "etaH", "guNm1", "gvNm1", "gtNm1", "gsNm1",
          "totPhiHyd", "hFacC", "uVelD", "vVelD")


def test_ocean90_restart_2_plus_2_bit_identical(tmp_path):
    from mitgcm_amd import configs, pickup
    a = configs.make_model(configs.global_ocean_90x40x15)
    a.forward_step(4)
    a.sync()
    b = configs.make_model(configs.global_ocean_90x40x15)
    b.forward_step(2)
    it = pickup.write_pickup(b, str(tmp_path), simulation="global_ocean.90x40x15")
    b.close()
    assert it == 36002
    assert (tmp_path / "pickup.0000036002.meta").exists() and (tmp_path / "pickup_cd.0000036002.data").exists()
    c = configs.make_model(lambda: configs.global_ocean_90x40x15(pickup_dir=str(tmp_path), nIter0=36002))
    c.forward_step(2)
    c.sync()
    g = a.g
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    bad = []
    for n in FIELDS:
        x, y = a.get(n), c.get(n)
        if not np.array_equal(x[inner], y[inner]):
            bad.append((n, float(np.abs(x[inner] - y[inner]).max())))
    for back in (0, 1):
        sa, sc = a.solve_stats(back=back), c.solve_stats(back=back)
        if sa != sc:
            bad.append(("solve", back, sa, sc))
    assert c.my_iter() == a.my_iter() == 36004
    a.close()
    c.close()
    assert not bad, bad
