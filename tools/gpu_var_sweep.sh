# Compare kernel configurations at 512^3 with the probe library (make PROBES=1 OUT=../lib_probe): SWEEP is a list of
# env assignments, one bench each, base first (e.g. SWEEP="MVTV_CG3D_NZ=2 MVTV_CG3D_NZ=7"); prints the bench value,
# the PCG leg and its fused kernel's mean launch. Optional CHECK="tests/..." runs those GPU tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${SWEEP_OUT:-sweep}
mkdir -p $O
export MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_probe/libmvtv.so
if [ -n "$CHECK" ]; then
  timeout -k 10 400 python -u -m pytest $CHECK -q -m gpu -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for rep in $(seq 1 ${REPS:-1}); do
  i=0
  for v in NONE=0 ${SWEEP}; do
    env $v timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-10} --warmup 3 ${BENCH_EXTRA} > $O/s$i.$rep.json 2> $O/s$i.$rep.err || { echo "bench $v failed"; tail -5 $O/s$i.$rep.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); p=d.get('pcg_leg') or {}; print(sys.argv[2], d['value'], 'pcg_leg', p.get('value'), p.get('kernel_avg_ms'), {k: v['avg_ms'] for k, v in d.get('kernels', {}).items()})" $O/s$i.$rep.json "$v.$rep"
    i=$((i+1))
  done
done
