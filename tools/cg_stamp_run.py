"""Run a few eager steps with the stamped diagnostic library (tools/cg_stamps.sh):
MGCM_LIB=mitgcm_amd/_build/diag/libmitgcm_amd_stamps.so python tools/cg_stamp_run.py [config]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mitgcm_amd import configs  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "ocean90"
mk = {"ocean90": configs.global_ocean_90x40x15, "cs32x15": configs.global_ocean_cs32x15,
      "llc90": configs.llc_synthetic}[cfg]
m = configs.make_model(mk)
m.forward_step(3)
m.sync()
print("done")
