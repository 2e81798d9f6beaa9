#!/bin/bash
# Round-5 GPU call driver: runs the named steps in order; a step that fails its tests goes on
# to the next, one that times out, aborts or faults (124, 134, 137, 139) ends the call.
#   bash profiles/r5_steps.sh <out-tag> refhost_multi | parity | cg_lb | refhost_all | all_gpu ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
T=$1
shift
O=gpurun_out/$T
mkdir -p $O
PY="python -u -m pytest -v --timeout 300 --timeout-method thread"
worst=0
for s in "$@"; do
  case $s in
    refhost_multi) timeout -k 10 400 $PY tests/test_gpu_refhost.py -k "ref-0-4 or 6-0 or 3-1" > $O/refhost_multi.log 2>&1 ;;
    refhost_m4) timeout -k 10 300 $PY tests/test_gpu_refhost.py -k "ref-0-4-0-0-0 or 6-0-0" > $O/refhost_m4.log 2>&1 ;;
    refhost_tp) timeout -k 10 300 $PY tests/test_gpu_refhost.py -k "throughput" > $O/refhost_tp.log 2>&1 ;;
    refhost_all) timeout -k 10 600 $PY tests/test_gpu_refhost.py > $O/refhost_all.log 2>&1 ;;
    refhost_llc) timeout -k 10 300 $PY tests/test_gpu_refhost.py -k "llc30" > $O/refhost_llc.log 2>&1 ;;
    parity) timeout -k 10 500 $PY -x tests/test_gpu_llc.py tests/test_gpu_ocean90.py tests/test_gpu_cs32x15.py > $O/parity.log 2>&1 ;;
    auto_policy) timeout -k 10 400 $PY tests/test_gpu_parallel.py -k "auto" > $O/auto_policy.log 2>&1 ;;
    dist_cg) timeout -k 10 600 $PY tests/test_gpu_parallel.py -k "distributed_cg2d" > $O/dist_cg.log 2>&1 ;;
    march) bash profiles/march_ab.sh $T/march > $O/march.log 2>&1 ;;
    corr_sb) bash profiles/corr_sb.sh $T/corr_sb > $O/corr_sb.log 2>&1 ;;
    vlead) bash profiles/vlead_ab.sh $T/vlead > $O/vlead.log 2>&1 ;;
    phi_ab) bash profiles/env_ab2.sh $T/phi_ab MGCM_PHI_N50 > $O/phi_ab.log 2>&1 ;;
    libab) OUT=$O/libab CONFIGS="llc90_synthetic global_ocean.90x40x15 global_ocean.cs32x15" \
             LIBS="default flat:mitgcm_amd/_build/diag/libmitgcm_amd_flat.so" bash tools/lib_ab.sh > $O/libab.log 2>&1 ;;
    llc_par) timeout -k 10 500 $PY -x tests/test_gpu_llc.py > $O/llc_par.log 2>&1 ;;
    gm_ab) OUT=$O/gm_ab CONFIGS="global_ocean.90x40x15 global_ocean.cs32x15" \
             LIBS="default base:mitgcm_amd/_build/diag/libmitgcm_amd_base.so" bash tools/lib_ab.sh > $O/gm_ab.log 2>&1 ;;
    c23_par) timeout -k 10 800 $PY -x tests/test_gpu_ocean90.py tests/test_gpu_cs32x15.py tests/test_gpu_options.py \
               tests/test_gpu_3d.py tests/test_gpu_refpin.py > $O/c23_par.log 2>&1 ;;
    fver_ab) OUT=$O/fver_ab CONFIGS="global_ocean.90x40x15 global_ocean.cs32x15" \
             LIBS="default fver:mitgcm_amd/_build/diag/libmitgcm_amd_fver.so base:mitgcm_amd/_build/diag/libmitgcm_amd_base.so" \
             bash tools/lib_ab.sh > $O/fver_ab.log 2>&1 ;;
    fver_par) MGCM_LIB=mitgcm_amd/_build/diag/libmitgcm_amd_fver.so timeout -k 10 800 $PY -x tests/test_gpu_ocean90.py \
               tests/test_gpu_cs32x15.py tests/test_gpu_options.py tests/test_gpu_3d.py > $O/fver_par.log 2>&1 ;;
    tr_ab) OUT=$O/tr_ab CONFIGS="global_ocean.90x40x15 global_ocean.cs32x15 llc90_synthetic" \
             LIBS="default base:mitgcm_amd/_build/diag/libmitgcm_amd_base.so" bash tools/lib_ab.sh > $O/tr_ab.log 2>&1 ;;
    kc_ab) OUT=$O/kc_ab CONFIGS="llc90_synthetic" \
             LIBS="default kc3:mitgcm_amd/_build/diag/libmitgcm_amd_kc3.so kc4:mitgcm_amd/_build/diag/libmitgcm_amd_kc4.so" \
             bash tools/lib_ab.sh > $O/kc_ab.log 2>&1 ;;
    x_ab) OUT=$O/x_ab CONFIGS="llc90_synthetic global_ocean.cs32x15" \
             LIBS="default base:mitgcm_amd/_build/diag/libmitgcm_amd_base.so" bash tools/lib_ab.sh > $O/x_ab.log 2>&1 ;;
    vi_ab) OUT=$O/vi_ab CONFIGS="llc90_synthetic llc90_synthetic" \
             LIBS="default base:mitgcm_amd/_build/diag/libmitgcm_amd_base.so" bash tools/lib_ab.sh > $O/vi_ab.log 2>&1 ;;
    options) timeout -k 10 600 $PY tests/test_gpu_options.py > $O/options.log 2>&1 ;;
    rest) timeout -k 10 1000 $PY tests -m gpu --ignore=tests/test_gpu_refhost.py --ignore=tests/test_gpu_parallel.py \
            --ignore=tests/test_gpu_rccl.py > $O/rest.log 2>&1 ;;
    parallel) timeout -k 10 1000 $PY tests/test_gpu_parallel.py tests/test_gpu_rccl.py > $O/parallel.log 2>&1 ;;
    llc) timeout -k 10 500 $PY -x tests/test_gpu_llc.py > $O/llc.log 2>&1 ;;
    bench_llc) timeout -k 10 300 python bench.py --config llc90_synthetic --steps 30 --warmup 4 --no-cs32 --no-cpu-baseline > $O/bench_llc.json 2> $O/bench_llc.err; tail -c 300 $O/bench_llc.json ;;
    vi_gl) bash profiles/vi_gl.sh $T/vi_gl > $O/vi_gl.log 2>&1 ;;
    all_gpu) timeout -k 10 1000 $PY tests -m gpu > $O/all_gpu.log 2>&1 ;;
    cg_lb) bash profiles/cg_lb.sh $T/cg_lb > $O/cg_lb.log 2>&1 ;;
    bench) bash profiles/r5_check.sh $T/bench bench > $O/bench.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "step $s rc=$rc"
  f=$(ls -t $O/*.log 2>/dev/null | head -1)
  [ -n "$f" ] && tail -4 $f
  case $rc in 124|134|137|139) echo "stopping after $s (rc $rc)"; exit $rc ;; esac
  [ $rc -ne 0 ] && worst=$rc
done
exit $worst
