# s_sleep between the multi-workgroup CG2D's poll passes: 1 (default) against 2 and 4
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/mwsleep CONFIGS="global_ocean.cs32x15 llc90_synthetic" LIBS="default s2:mitgcm_amd/_variants/lib_s2.so s4:mitgcm_amd/_variants/lib_s4.so" bash tools/lib_ab.sh
for f in gpurun_out/mwsleep/b_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f'.split('/')[-1], round(d['ms_per_step'],4), round(d['roofline']['us_per_iteration'],3))"; done
