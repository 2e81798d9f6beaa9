"""The cube's multi-dimensional advection on the device (kernels_thermo.hip k_advg_*: the
3-pass face-dependent split of gad_advection.F:339-367 with FILL_CS_CORNER_TR_RL /
FILL_CS_CORNER_UV_RS, GAD_MULTIDIM_COMPRESSIBLE) on verification/advect_cs through the
C-ABI.  Bars: theta bit-identical to the oracle after 24 steps; theta min/max/mean/sd
>= 13 digits against the reference's results/output.txt at every monitor step of the
first 96 steps."""
import json
import os

import numpy as np
import pytest

from conftest import digits

pytestmark = pytest.mark.gpu


def test_advect_cs_device_bitexact_vs_oracle():
    from mitgcm_amd import configs
    from oracle.harness import oracle_from_config
    m = configs.make_model(configs.advect_cs)
    o, g = oracle_from_config(configs.advect_cs)
    for _ in range(24):
        o.forward_step()
    m.forward_step(24)
    m.sync()
    dev = m.get("theta")
    ref = np.array(o.arr("theta")).reshape(dev.shape)
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    err = np.abs(dev[inner] - ref[inner]).max()
    m.close()
    assert np.array_equal(dev[inner], ref[inner]), err


def test_advect_cs_device_vs_reference_output(golden_dir):
    from mitgcm_amd import configs
    from mitgcm_amd.model import dynstat
    gold = json.load(open(os.path.join(golden_dir, "advect_cs", "monitor.json")))
    m = configs.make_model(configs.advect_cs)
    worst = (99.0, None)
    for n in range(8, 97, 8):
        m.forward_step(8)
        ds = dynstat(m)
        gs = gold[n // 8]
        for k in ("min", "max", "mean", "sd"):
            worst = min(worst, (digits(ds["dynstat_theta_" + k], gs["dynstat_theta_" + k]), (n, k)))
    m.close()
    print("advect_cs on the device, 96 steps: worst digits %.2f at %s" % worst)
    assert worst[0] >= 13.0, worst
