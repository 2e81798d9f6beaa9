"""Build the reference-host harness mitgcm_amd/fortran/refhost/refhost_<layout> (needs the
reference headers: the build container only; the binaries travel to the GPU box).

The MODS drop-ins (mitgcm_amd/fortran/mods/*.F), the harness main program
(refhost/refhost.F) and REFHOST_PARAM / REFHOST_FIELD -- generated here from the
parameters and arrays MGCM_AMD_MIRROR hands to the device, so the harness fills exactly
the COMMON-block names the mirror reads -- are preprocessed against the reference's own
headers (experiment code/ dir, model/inc, eesupp/inc, pkg/gmredi, pkg/cd_code; cpp
-traditional as genmake2 runs it, with its " _d " -> "D" constant rewrite), compiled with
amdflang and linked against libmitgcm_amd.so.  The preprocessed sources (which carry the
reference headers' text) are deleted after compiling; nothing of them is committed.

Layouts:
  ref   verification/global_ocean.90x40x15/code/SIZE.h as committed: 9 x 4 tiles of
        10 x 10, OL = 3 (the tiling results/output.txt was produced on)
  1t    the same experiment on one 90 x 40 tile, OL = 3 (the device's bench layout): a
        SIZE.h of that shape, as a user writes one in a code/ directory (refhost/SIZE.h.1t)
  cs32  verification/global_ocean.cs32x15/code/SIZE.h as committed: 12 tiles of 32 x 16,
        OL = 4, on pkg/exch2 (the cube's six 32 x 32 faces, two tiles each: W2's default
        topology, the experiment has no data.exch2), staggerTimeStep
  cs32_6t  the same experiment on six 32 x 32 tiles, one per face (the device's bench layout;
        refhost/SIZE.h.cs32_6t)
  llc30 BASELINE config 5's lat-lon-cap topology at n = 30 (13 tiles of 30 x 30, OL = 4, 50
        levels; refhost/SIZE.h.llc30) on global_ocean.cs32x15's code/ options and packages: the
        synthetic LLC workload has no reference experiment, its namelist is written by the test
        from mitgcm_amd/configs.py llc_synthetic
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
FC = "/opt/rocm/bin/amdflang"
MODS = os.path.join(HERE, "mods")
RH = os.path.join(HERE, "refhost")
# the package switches genmake2 derives from the experiment's packages.conf (the packages
# whose headers the drop-ins and the harness include)
OCEAN90 = ("global_ocean.90x40x15", "#define ALLOW_GMREDI\n#define ALLOW_CD_CODE\n")
CS32 = ("global_ocean.cs32x15", "#define ALLOW_GMREDI\n#define ALLOW_EXCH2\n")
# layout -> (experiment, PACKAGES_CONFIG.h, SIZE.h replacing the experiment's or None)
LAYOUTS = {"ref": OCEAN90 + (None,), "1t": OCEAN90 + (os.path.join(RH, "SIZE.h.1t"),), "cs32": CS32 + (None,),
           "cs32_6t": CS32 + (os.path.join(RH, "SIZE.h.cs32_6t"),),
           "llc30": CS32 + (os.path.join(RH, "SIZE.h.llc30"),)}


def available():
    return os.path.isdir(REF) and os.path.exists(FC) and shutil.which("cpp") is not None


def _calls(src):
    """(kind, name, arg[, bind kind]) of every MGCM_AMD_{R,L,I}PARAM and MGCM_AMD_BIND call
    of the mirror, with the #ifdef lines around them (kind '#' carries the line)."""
    lines, out, cur = open(src).read().splitlines(), [], ""
    for ln in lines:
        if ln.startswith("#") and not ln.startswith("#include"):
            out.append(("#", ln, None))
            continue
        if ln[:1] in ("C", "c", "!"):
            continue
        if len(ln) > 5 and ln[5] not in (" ", "0") and cur:
            cur += ln[6:].strip()
        else:
            cur = ln.strip()
        m = re.match(r"CALL MGCM_AMD_([RLI])PARAM\(\s*'(\w+)'\s*,\s*([\w()]+)\s*\)$", cur)
        if m:
            out.append((m.group(1), m.group(2), m.group(3)))
            cur = ""
            continue
        m = re.match(r"CALL MGCM_AMD_BIND\(\s*'(\w+)'\s*,\s*(\w+)\s*,\s*SIZE\(\w+\)\s*,\s*(\d)\s*\)$", cur)
        if m:
            out.append(("B", m.group(1), m.group(2), int(m.group(3))))
            cur = ""
    return out


def mirror_calls(undef=()):
    """The parameters [(R|L|I, name)] and bound arrays [(name, kind)] MGCM_AMD_MIRROR passes
    (every #ifdef branch of a config with GMREDI, CD_CODE, NONLIN_FRSURF, EXACT_CONSERV, but
    the #ifdef blocks of the macros in `undef`, e.g. ("ALLOW_CD_CODE",) for cs32)."""
    calls, skip = [], []
    for c in _calls(os.path.join(MODS, "mgcm_amd_mirror.F")):
        if c[0] == "#":
            w = c[1].lstrip("#").split()
            if w and w[0] in ("ifdef", "ifndef", "if"):
                skip.append(w[0] == "ifdef" and w[-1] in undef)
            elif w and w[0] in ("else", "elif"):
                raise ValueError("mirror_calls: #%s in the mirror is not handled" % w[0])
            elif w and w[0] == "endif":
                skip.pop()
            continue
        if not any(skip):
            calls.append(c)
    return [(c[0], c[1]) for c in calls if c[0] != "B"], [(c[1], c[3]) for c in calls if c[0] == "B"]


def generate_fill(path):
    """refhost_fill.F: REFHOST_PARAM(name, val, found) / REFHOST_FIELD(name, buf, n, dir, found)."""
    mirror = os.path.join(MODS, "mgcm_amd_mirror.F")
    src = open(mirror).read()
    body = src[src.index("      SUBROUTINE MGCM_AMD_MIRROR"):src.index("      INTEGER myIter, myThid")]
    incl = [ln for ln in body.splitlines() if ln.startswith("#") and "include" in ln or ln.startswith("# include")
            or ln.startswith("#ifdef") or ln.startswith("#endif")]
    calls = _calls(mirror)
    head = ['C refhost_fill.F -- GENERATED by mitgcm_amd/fortran/build_refhost.py from the calls of',
            'C MGCM_AMD_MIRROR (mods/mgcm_amd_mirror.F); do not edit.',
            '#include "PACKAGES_CONFIG.h"', '#include "CPP_OPTIONS.h"', '#ifdef ALLOW_GMREDI',
            '# include "GMREDI_OPTIONS.h"', '#endif', '']
    p = head + ['      SUBROUTINE REFHOST_PARAM( name, val, found )', '      IMPLICIT NONE'] + incl + [
        '      CHARACTER*(*) name', '      Real*8 val', '      LOGICAL found', '      INTEGER k', '      found = .TRUE.',
        "      IF ( name.EQ.'_none_' ) THEN", '        CONTINUE']
    for kind, name, arg, *_ in calls:
        if kind == "#":
            if name.startswith("#if") or name.startswith("#endif") or name.startswith("#else"):
                p.append(name)
            continue
        if kind == "B":
            continue
        p.append("      ELSEIF ( name.EQ.'%s' ) THEN" % name)
        if name == "eosType":      # the mirror's code: 0 LINEAR, 1 the JMD95 family
            p += ["        eosType = 'LINEAR'", "        IF ( val.NE.0.D0 ) eosType = 'JMD95Z'"]
        elif name == "periodicExternalForcing":
            p.append("        periodicExternalForcing = val.NE.0.D0")
        elif arg.endswith("(1)"):   # a per-level profile given by its (uniform) value
            a = arg[:-3]
            p += ["        DO k = 1, SIZE(%s)" % a, "          %s(k) = val" % a, "        ENDDO"]
        elif kind == "R":
            p.append("        %s = val" % arg)
        elif kind == "L":
            p.append("        %s = val.NE.0.D0" % arg)
        else:
            p.append("        %s = NINT(val)" % arg)
    p += ['      ELSE', '        found = .FALSE.', '      ENDIF',
          "C     set_parms.F:268-275 in reverse: the JMD95 family with the dynamic pressure is 'JMD95P'",
          "      IF ( eosType.EQ.'JMD95Z' .AND. selectP_inEOS_Zc.GE.2 )", "     &     eosType = 'JMD95P'",
          '      RETURN', '      END', '']
    # REFHOST_PARAM_GET(i, name, val, found): the i-th parameter the mirror passes and the value
    # it would pass (the COMMON variable it names; eosType as the mirror's code) -- the
    # harness's --params dump of what refhost_parms.F resolved
    pars = [c for c in calls if c[0] in ("R", "L", "I", "#")]
    p += ['      SUBROUTINE REFHOST_PARAM_GET( i, name, val, found )', '      IMPLICIT NONE'] + incl + [
        '      INTEGER i', '      CHARACTER*(*) name', '      Real*8 val', '      LOGICAL found', '      found = .TRUE.',
        "      name = ' '", '      val = 0.D0', '      IF ( i.LT.0 ) THEN', '        CONTINUE']
    idx = 0
    for kind, name, arg, *_ in pars:
        if kind == "#":
            if name.startswith("#if") or name.startswith("#endif") or name.startswith("#else"):
                p.append(name)
            continue
        idx += 1
        p.append("      ELSEIF ( i.EQ.%d ) THEN" % idx)
        p.append("        name = '%s'" % name)
        if name == "eosType":
            p += ["        val = 0.D0", "        IF ( eosType(1:5).EQ.'JMD95' ) val = 1.D0"]
        elif name == "periodicExternalForcing":
            p.append("        IF ( periodicExternalForcing ) val = 1.D0")
        elif kind == "R":
            p.append("        val = %s" % arg)
        elif kind == "L":
            p.append("        IF ( %s ) val = 1.D0" % arg)
        else:
            p.append("        val = DBLE( %s )" % arg)
    p += ['      ELSE', '        found = .FALSE.', '      ENDIF', '      RETURN', '      END', '']
    p += ['      SUBROUTINE REFHOST_FIELD( name, buf, n, dir, found )', '      IMPLICIT NONE'] + incl + [
        '      CHARACTER*(*) name', '      INTEGER n, dir', '      Real*8 buf(n)', '      LOGICAL found',
        '      found = .TRUE.', "      IF ( name.EQ.'_none_' ) THEN", '        CONTINUE']
    for kind, name, arg, *_ in calls:
        if kind == "#":
            if name.startswith("#if") or name.startswith("#endif") or name.startswith("#else"):
                p.append(name)
            continue
        if kind != "B":
            continue
        p.append("      ELSEIF ( name.EQ.'%s' ) THEN" % name)
        p.append("        CALL REFHOST_COPY( %s, SIZE(%s), buf, n, dir )" % (arg, arg))
    p += ['      ELSE', '        found = .FALSE.', '      ENDIF', '      RETURN', '      END', '']
    open(path, "w").write("\n".join(p) + "\n")


def _pre(src, tmp, incdirs):
    pre = subprocess.run(["cpp", "-traditional", "-P", "-DWORDLENGTH=4"] + ["-I" + d for d in incdirs] + [src],
                         check=True, capture_output=True, text=True).stdout
    base = os.path.basename(src)[:-2]
    f = os.path.join(tmp, base + ".f")
    open(f, "w").write(pre.replace(" _d ", "D"))
    return f


def build(layouts=("ref", "1t", "cs32", "cs32_6t", "llc30"), verbose=False):
    if not available():
        raise RuntimeError("build_refhost needs /root/reference (headers), amdflang and cpp")
    lib = os.path.join(ROOT, "mitgcm_amd", "libmitgcm_amd.so")
    if not os.path.exists(lib):
        sys.path.insert(0, ROOT)
        from mitgcm_amd import build as b
        b.build()
    out = []
    for lay in layouts:
        tmp = tempfile.mkdtemp(prefix="refhost_")
        try:
            exp, pkgs, size = LAYOUTS[lay]
            open(os.path.join(tmp, "PACKAGES_CONFIG.h"), "w").write(pkgs)
            if size:
                shutil.copy(size, os.path.join(tmp, "SIZE.h"))
            inc = [tmp] + [os.path.join(REF, p) for p in ("verification/%s/code" % exp, "model/inc", "eesupp/inc",
                                                          "pkg/gmredi", "pkg/cd_code", "pkg/exch2")]
            fill = os.path.join(tmp, "refhost_fill.F")
            generate_fill(fill)
            srcs = sorted(os.path.join(MODS, f) for f in os.listdir(MODS) if f.endswith(".F"))
            srcs += [os.path.join(RH, "refhost.F"), os.path.join(RH, "refhost_parms.F"), fill]
            objs = []
            for s in srcs:
                f = _pre(s, tmp, inc)
                o = f[:-2] + ".o"
                cmd = [FC, "-O2", "-ffp-contract=off", "-ffixed-form", "-ffixed-line-length=132", "-c", f, "-o", o]
                if verbose:
                    print(" ".join(cmd))
                subprocess.run(cmd, check=True, cwd=tmp)
                objs.append(o)
            exe = os.path.join(RH, "refhost_" + lay)
            cmd = [FC, "-o", exe + ".tmp"] + objs + ["-L" + os.path.dirname(lib), "-lmitgcm_amd",
                                                      "-Wl,-rpath,$ORIGIN/../.."]
            subprocess.run(cmd, check=True, cwd=tmp)
            os.replace(exe + ".tmp", exe)
            out.append(exe)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)   # the preprocessed text of the reference headers
    return out


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
