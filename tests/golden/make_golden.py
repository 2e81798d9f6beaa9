"""Extract golden fixtures for the parity tests from the reference checkout.

Run in the build container only (it reads /root/reference, which does not exist
on the GPU box):  python tests/golden/make_golden.py

What it writes (data only -- inputs and expected outputs, no reference source):
  tests/golden/<exp>/*.bin            the experiment's own binary input fields, verbatim
  tests/golden/<exp>/monitor.json     per-step %MON / cg2d_* values parsed from the
                                      committed verification/<exp>/results/output.txt
  tests/golden/<exp>/params.json      resolved run-time parameters parsed from the
                                      "Model configuration" dump of the same output.txt
  tests/golden/<exp>/monitor.<tag>.json, params.<tag>.json
                                      the same from another committed output of the
                                      experiment (results/output.<tag>.txt)
  tests/golden/adjustment.cs-32x32x1/w2_topology.json
                                      the "W2 TILE TOPLOGY" lists (per tile, its neighbours'
                                      tile ids in W2's order) the reference printed for its
                                      default 6-face cube of 32 x 32 on 48 tiles of 16 x 8
                                      (results/output.txt) and 6 tiles of 32 x 32
                                      (results/output.nlfs.txt), with the tile sizes
"""
import json
import os
import re
import shutil
import sys

REF = "/root/reference/verification"
HERE = os.path.dirname(os.path.abspath(__file__))

EXPERIMENTS = {
    "tutorial_barotropic_gyre": {
        "inputs": ["input/bathy.bin", "input/windx_cosy.bin"],
        "output": "results/output.txt",
    },
    "advect_xy": {
        "inputs": [],
        "output": "results/output.txt",
        # input.ab3_c4: centred 4th-order advection (scheme 4) of theta and salt with
        # ADAMS_BASHFORTH3 (code/CPP_OPTIONS.h defines ALLOW_ADAMSBASHFORTH_3)
        "extra_outputs": {"ab3_c4": "results/output.ab3_c4.txt"},
    },
    "tutorial_baroclinic_gyre": {
        "inputs": ["input/bathy.bin", "input/windx_cosy.bin", "input/SST_relax.bin"],
        "output": "results/output.txt",
    },
    # 90x40x15 lat-lon ocean, cold start: JMD95Z, GM-Redi, CD scheme, monthly forcing.
    # lev_t/lev_s hold 12 monthly 3-D records; the run reads record 1 only, so only
    # that record is kept (90*40*15 fp32 = 216000 bytes).
    "tutorial_global_oce_latlon": {
        "inputs": ["input/bathymetry.bin", ("input/lev_t.bin", 216000), ("input/lev_s.bin", 216000),
                   "input/lev_sst.bin", "input/lev_sss.bin", "input/ncep_qnet.bin", "input/ncep_emp.bin",
                   "input/trenberth_taux.bin", "input/trenberth_tauy.bin"],
        "output": "results/output.txt",
    },
    # BASELINE config 2: same inputs (input/prepare_run links them from
    # tutorial_global_oce_latlon) + the pickups it restarts from at nIter0 = 36000
    "global_ocean.90x40x15": {
        "inputs": ["input/pickup.0000036000", "input/pickup.0000036000.meta", "input/pickup_cd.0000036000"],
        "namelists": ["input/data", "input/data.pkg", "input/data.gmredi"],
        "output": "results/output.txt",
    },
    # cubed sphere (pkg/exch2, 6 faces of 32x32, one tile each), 1 level, vector-invariant
    # momentum, passive salt: solid-body rotation (code/ini_vel.F, code/ini_psurf.F)
    "solid-body.cs-32x32x1": {
        "inputs": ["input/tile00%d.mitgrid" % f for f in range(1, 7)] + ["input/S_init.bin"],
        "output": "results/output.txt",
    },
    # cubed sphere (pkg/exch2, 6 faces of 32x32, OL=4), 1 level, momStepping=F: solid-body
    # rotation (code/ini_vel.F) advecting theta with DST3 flux-limited multi-dimensional
    # advection (tempAdvScheme=33, 3-pass cube split), GAD_MULTIDIM_COMPRESSIBLE; the grid is
    # global_ocean.cs32x15's grid_cs32 faces (input/prepare_run links the same files)
    "advect_cs": {
        "inputs": ["input/T.init", "input/S.init"],
        "output": "results/output.txt",
    },
    # BASELINE config 3 (cs32x15).  Its pickup.0000072000 is not in the checkout
    # (.MISSING_LARGE_BLOBS), so the run is a cold start from lev_T/lev_S: only the grid
    # statistics of output.txt pin it.  Grid files are linked by input/prepare_run.
    "global_ocean.cs32x15": {
        "inputs": ["input/bathy_Hmin50.bin", "input/lev_T_cs_15k.bin", "input/lev_S_cs_15k.bin",
                   "input/lev_surfT_cs_12m.bin", "input/lev_surfS_cs_12m.bin", "input/shiQnet_cs32.bin",
                   "input/shiEmPR_cs32.bin", "input/trenberth_taux.bin", "input/trenberth_tauy.bin"] +
                  ["../tutorial_held_suarez_cs/input/grid_cs32.face00%d.bin" % f for f in range(1, 7)],
        "namelists": ["input/data", "input/data.pkg", "input/data.gmredi"],
        "output": "results/output.txt",
    },
}

_num = r"[-+]?\d*\.?\d+(?:[EeDd][-+]?\d+)?"


def parse_grid_monitor(path):
    """%MON lines printed before the first time step (INI_GRID / INI_CORI grid
    statistics, model/src/ini_grid.F:128-145)."""
    grid = {}
    with open(path) as f:
        for line in f:
            m = re.search(r"%MON (\S+)\s*=\s*(" + _num + ")", line)
            if m:
                if m.group(1) == "time_tsnumber":
                    break
                grid[m.group(1)] = float(m.group(2).replace("D", "E"))
    return grid


def parse_monitor(path):
    """Return a list of per-step dicts: {'time_tsnumber': n, 'dynstat_eta_max': x, ...,
    'cg2d_init_res': ..., 'cg2d_iters': ..., 'cg2d_last_res': ...}.  The cg2d lines that
    precede a monitor block belong to the step that block reports."""
    steps, pending, cur = [], {}, None
    with open(path) as f:
        for line in f:
            m = re.search(r"%MON (\S+)\s*=\s*(" + _num + ")", line)
            if m:
                key, val = m.group(1), m.group(2).replace("D", "E")
                if key == "time_tsnumber":
                    cur = {"time_tsnumber": int(val)}
                    cur.update(pending)
                    pending = {}
                    steps.append(cur)
                elif cur is not None:
                    cur[key] = float(val)
                continue
            m = re.search(r"cg2d_init_res =\s*(" + _num + ")", line)
            if m:
                pending["cg2d_init_res"] = float(m.group(1))
                continue
            m = re.search(r"cg2d_iters\(min,last\) =\s*(-?\d+)\s+(\d+)", line)
            if m:
                pending["cg2d_iters_min"] = int(m.group(1))
                pending["cg2d_iters"] = int(m.group(2))
                continue
            m = re.search(r"cg2d_last_res =\s*(" + _num + ")", line)
            if m:
                pending["cg2d_last_res"] = float(m.group(1))
                continue
            m = re.search(r"cg2d: Sum\(rhs\),rhsMax =\s*(" + _num + r")\s+(" + _num + ")", line)
            if m:
                pending["cg2d_sum_rhs"] = float(m.group(1))
                pending["cg2d_rhs_max"] = float(m.group(2))
    return steps


def parse_params(path):
    """Parse the 'name = /* description */' + value lines of the configuration dump."""
    params = {}
    lines = open(path).read().splitlines()
    pref = "(PID.TID 0000.0001) "
    for n, line in enumerate(lines):
        if not line.startswith(pref):
            continue
        body = line[len(pref):]
        m = re.match(r"(\w+)\s*=\s*/\*", body)
        if not m or n + 1 >= len(lines):
            continue
        name, vals = m.group(1), []
        for nxt in lines[n + 1:n + 40]:
            v = nxt[len(pref):].strip() if nxt.startswith(pref) else ""
            if v.startswith(";") or not v:
                break
            tok = v.split("/*")[0].strip()
            mm = re.match(r"(\d+)\s*@\s*(" + _num + r"|[TF])", tok)
            if mm:
                vals += [mm.group(2)] * int(mm.group(1))
            else:
                vals.append(tok)
        if vals:
            params[name] = vals[0] if len(vals) == 1 else vals
    return params


W2_TOPOLOGY = ("adjustment.cs-32x32x1", ["results/output.txt", "results/output.nlfs.txt"])


def parse_w2_topology(path):
    """The tile sizes and, per tile, the neighbour tile ids of the 'W2 TILE TOPLOGY' print
    (pkg/exch2 w2_print_e2setup.F, W2_printMsg)."""
    txt = open(path).read()
    size = {k: int(re.search(r"\b%s =\s+(\d+) ;" % k, txt).group(1)) for k in ("sNx", "sNy", "nSx", "nSy", "OLx")}
    tiles = {}
    cur = None
    for line in txt.splitlines():
        m = re.search(r"^\(PID\.TID 0000\.0001\)\s+TILE:\s+(\d+)\s*$", line)
        if m:
            cur = int(m.group(1))
            tiles[cur] = []
            continue
        m = re.search(r"NEIGHBOUR\s+(\d+) = TILE\s+(\d+)", line)
        if m and cur is not None:
            assert int(m.group(1)) == len(tiles[cur]) + 1
            tiles[cur].append(int(m.group(2)))
    return dict(size, neighbours=[tiles[t] for t in sorted(tiles)])


def main():
    only = sys.argv[1:]   # optional: experiment names to (re)extract
    if not only or "w2" in only:
        exp, outs = W2_TOPOLOGY
        os.makedirs(os.path.join(HERE, exp), exist_ok=True)
        with open(os.path.join(HERE, exp, "w2_topology.json"), "w") as f:
            json.dump({o: parse_w2_topology(os.path.join(REF, exp, o)) for o in outs}, f)
        print("wrote", os.path.join(HERE, exp, "w2_topology.json"))
    for exp, spec in EXPERIMENTS.items():
        if only and exp not in only:
            continue
        out = os.path.join(HERE, exp)
        os.makedirs(out, exist_ok=True)
        for rel in spec["inputs"]:
            if isinstance(rel, tuple):   # (path, leading bytes kept)
                rel, nbytes = rel
                with open(os.path.join(REF, exp, rel), "rb") as fi, \
                        open(os.path.join(out, os.path.basename(rel)), "wb") as fo:
                    fo.write(fi.read(nbytes))
                continue
            shutil.copyfile(os.path.join(REF, exp, rel), os.path.join(out, os.path.basename(rel)))
        # the experiment's namelist files (data: the run-time parameters the reference-host
        # harness reads, refhost_parms.F), verbatim under <exp>/input/
        for rel in spec.get("namelists", []):
            os.makedirs(os.path.join(out, "input"), exist_ok=True)
            shutil.copyfile(os.path.join(REF, exp, rel), os.path.join(out, "input", os.path.basename(rel)))
        res = os.path.join(REF, exp, spec["output"])
        with open(os.path.join(out, "monitor.json"), "w") as f:
            json.dump(parse_monitor(res), f, indent=1)
        with open(os.path.join(out, "grid_monitor.json"), "w") as f:
            json.dump(parse_grid_monitor(res), f, indent=1)
        with open(os.path.join(out, "params.json"), "w") as f:
            json.dump(parse_params(res), f, indent=1, sort_keys=True)
        for tag, rel in spec.get("extra_outputs", {}).items():   # other runs of the same experiment
            res = os.path.join(REF, exp, rel)
            with open(os.path.join(out, "monitor.%s.json" % tag), "w") as f:
                json.dump(parse_monitor(res), f, indent=1)
            with open(os.path.join(out, "params.%s.json" % tag), "w") as f:
                json.dump(parse_params(res), f, indent=1, sort_keys=True)
        print("wrote", out)


if __name__ == "__main__":
    sys.exit(main())
