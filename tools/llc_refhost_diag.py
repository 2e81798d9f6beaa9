"""Diagnostic for test_refhost_llc30_exch2_bitexact: per-field differences after 1 and 2 steps
(eager and replayed) between refhost's drop-in path and the resident model.
  python tools/llc_refhost_diag.py <outdir>"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_refhost as T  # noqa: E402
from mitgcm_amd import configs  # noqa: E402

res = {}
for nsteps, eager in ((1, 1),):
    tmp = tempfile.mkdtemp()
    out3 = configs.llc_synthetic(n=30)
    g0, params, st0 = out3
    pdir = T._llc_namelists(os.path.join(tmp, "input"), params, st0["tRef"], st0["sRef"], configs.llc_delr(50), g0)
    m = configs.make_model(lambda: out3)
    w2 = m.g.topo.w2_arrays(ldNb=8, ldT=2 * m.g.nTiles)
    state = T._write_blob(os.path.join(tmp, "refhost_in.bin"), m, nsteps, monitor_days=2, w2=w2,
                          undef=("ALLOW_CD_CODE",))
    env = dict(os.environ, MGCM_AMD_MODELS="1", MGCM_AMD_EAGER=str(eager))
    r = subprocess.run([os.path.join(T.RH, "refhost_llc30"), tmp, pdir], capture_output=True, text=True, timeout=300,
                       env=env)
    if r.returncode != 0:
        print(r.stdout[-3000:], r.stderr[-3000:])
        sys.exit(1)
    out, st = T._read_out(os.path.join(tmp, "refhost_out.bin"), state, nsteps)
    m.forward_step(nsteps)
    m.sync()
    d = {}
    for n in out:
        if n == "phiRef":
            continue
        dev = m.get(n).reshape(-1)[:out[n].size]
        if not np.array_equal(out[n], dev):
            dd = np.abs(out[n] - dev)
            d[n] = [float(dd.max()), int((dd > 0).sum()), int(np.argmax(dd))]
    d["_solve"] = m.solve_stats()
    m.close()
    key = "steps%d_eager%d" % (nsteps, eager)
    res[key] = d
    print(key, json.dumps(d), flush=True)
    print(r.stdout[-1500:], flush=True)
    print([ln for ln in r.stderr.splitlines() if "cg2dNorm" in ln],
          "python: %.17e %.17e %.17e" % (m.g.cg2dNorm, m.g.cg2dTolerance_sq, getattr(m.g, "globalArea", 0.0)), flush=True)
if len(sys.argv) > 1:
    os.makedirs(sys.argv[1], exist_ok=True)
    json.dump(res, open(os.path.join(sys.argv[1], "llc_refhost_diag.json"), "w"), indent=1)
