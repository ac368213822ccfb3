# Round 3: folded right-hand side: the changed-path GPU tests, then an A/B on one box (probe build:
# MVTV_FOLD_OFF=1 restores the 3-vector b).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3i
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    ${TESTS:-tests/test_gpu_fused3d.py tests/test_gpu_parity.py tests/test_gpu_spectral.py tests/test_gpu_configs.py} > gpurun_out/r3i/tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3i/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
export MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_probe/libmvtv.so
for rep in 1 2; do
  for e in base MVTV_FOLD_OFF=1; do
    if [ "$e" = base ]; then ev=""; else ev="$e"; fi
    for c in ${CASES:-3:512 3:256}; do
      d=${c%%:*}; n=${c##*:}
      env $ev timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 --steps ${STEPS:-30} --warmup 5 --dims $d --size $n ${BENCH_EXTRA} > gpurun_out/r3i/$n.$rep.${e%%=*}.json 2> gpurun_out/r3i/$n.$rep.${e%%=*}.err || { tail -5 gpurun_out/r3i/$n.$rep.${e%%=*}.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d.get('kernels',{}).items()})" gpurun_out/r3i/$n.$rep.${e%%=*}.json "$n $e.$rep"
    done
  done
done
