# GPU box: A/B of environment switches on the 512^3 bench (same box, same binary, interleaved runs).
# usage: AB_ENVS="MVTV_DCT_FASTDIV=1 MVTV_EBUF3=1" bash tools/gpu_ab_env.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ab
cd $R
if [ -n "$AB_TESTS" ]; then
  env $AB_TEST_ENV timeout -k 10 300 python -u -m pytest $AB_TESTS -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 || { tail -20 gpurun_out/ab/tests.log; exit 1; }
  tail -2 gpurun_out/ab/tests.log
fi
for rep in $(seq 1 ${AB_REPS:-2}); do
  for e in base $AB_ENVS; do
    if [ "$e" = base ]; then ev=""; else ev="$e"; fi
    env $ev timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 --steps ${AB_STEPS:-30} --warmup 3 > gpurun_out/ab/$e.$rep.json 2> gpurun_out/ab/$e.$rep.err || { echo "bench $e failed"; tail -5 gpurun_out/ab/$e.$rep.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d['kernels'].items()})" gpurun_out/ab/$e.$rep.json "$e.$rep"
  done
done
