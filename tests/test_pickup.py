"""WRITE_PICKUP (mitgcm_amd/pickup.py) against the reference's own pickup: reading
verification/global_ocean.90x40x15/input/pickup.0000036000 (+ pickup_cd) into the tile
layout and writing it back reproduces the reference's bytes and its .meta text
(record order of write_pickup.F:107-322, MDS_WR_METAFILES format).  Host only."""
import os

import numpy as np


def test_pickup_round_trip_reproduces_reference_bytes(golden_dir, tmp_path):
    from mitgcm_amd import configs, pickup
    g, params, state, _ = configs.global_ocean_90x40x15()
    gd = os.path.join(golden_dir, "global_ocean.90x40x15")
    fields = dict(state)
    fields["etaHnm1"] = state["etaH"]   # READ_PICKUP puts the EtaH record in etaH
    cd = {n: state[n] for n in ("uVelD", "vVelD", "uNM1", "vNM1", "etaNm1")}
    pickup.write_pickup_fields(g, params, fields, str(tmp_path), 36000, 36000 * 86400.0,
                               simulation="global_ocean.90x40x15", cd=cd)
    mine = open(tmp_path / "pickup.0000036000.data", "rb").read()
    ref = open(os.path.join(gd, "pickup.0000036000"), "rb").read()
    assert len(mine) == len(ref) == 138 * 90 * 40 * 8
    assert mine == ref
    assert open(tmp_path / "pickup.0000036000.meta").read() == open(os.path.join(gd, "pickup.0000036000.meta")).read()
    mine_cd = np.fromfile(tmp_path / "pickup_cd.0000036000.data", dtype=">f8")
    ref_cd = np.fromfile(os.path.join(gd, "pickup_cd.0000036000"), dtype=">f8")
    # the reference file may carry records past CD_CODE_READ_PICKUP's 4*Nr+1
    assert np.array_equal(mine_cd, ref_cd[:mine_cd.size])


def test_pickup_records_follow_options():
    from mitgcm_amd.pickup import pickup_records
    names = [r[2] for r in pickup_records({"storePhiHyd4Phys": 1})]
    assert names == ["Uvel", "Vvel", "Theta", "Salt", "GuNm1", "GvNm1", "GtNm1", "GsNm1", "PhiHyd", "EtaN",
                     "dEtaHdt", "EtaH"]
    # DST3 flux-limited tracers step forward (no AB2 on the tendency): no GtNm1 / GsNm1
    names = [r[2] for r in pickup_records({"tempAdvScheme": 33, "saltAdvScheme": 33})]
    assert "GtNm1" not in names and "GsNm1" not in names and "PhiHyd" not in names
