"""Write a refhost input case (refhost_in.bin) outside pytest, for diagnosis runs of the
reference-host harness: python tools/refhost_case.py ref|1t NSTEPS OUTDIR.  Uses the blob
writer of tests/test_gpu_refhost.py (config 2 on the reference's 9 x 4 tiles or one tile)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mitgcm_amd import configs  # noqa: E402
import test_gpu_refhost as T  # noqa: E402

layout, nsteps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
os.makedirs(out, exist_ok=True)
tiles = {"ref": (9, 4), "1t": (1, 1)}[layout]
m = configs.make_model(lambda: configs.global_ocean_90x40x15(nSx=tiles[0], nSy=tiles[1]))
T._write_blob(os.path.join(out, "refhost_in.bin"), m, nsteps, monitor_days=2, packages_off=True)
m.close()
print("wrote", os.path.join(out, "refhost_in.bin"))
