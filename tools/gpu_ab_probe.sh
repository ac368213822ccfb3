# Probe-build A/B on one box: the changed-path GPU tests with the probe library and AB_ENV set, then interleaved
# bench runs of the probe library without / with AB_ENV (CASES="dims:size ...", STEPS, BENCH_EXTRA).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${AB_OUT:-abp}
mkdir -p $OUT
export MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_probe/libmvtv.so
if [ -n "$TESTS" ]; then
  env $AB_ENV timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu $TESTS > $OUT/tests.log 2>&1
  rc=$?
  tail -3 $OUT/tests.log
  if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
for rep in 1 2; do
  for e in base $AB_ENV; do
    if [ "$e" = base ]; then ev=""; else ev="$e"; fi
    for c in ${CASES:-3:512}; do
      d=${c%%:*}; n=${c##*:}
      f=$OUT/$d.$n.$rep.${e%%=*}
      env $ev timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 --steps ${STEPS:-30} --warmup 5 --dims $d --size $n ${BENCH_EXTRA} > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d.get('kernels',{}).items()})" $f.json "$d:$n $e.$rep"
    done
  done
done
