#!/bin/bash
# release library: spectral / config / parity GPU tests, then the 2-D config bench lines and 512^3
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/chk
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; return 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d['kernels'].items()})" $O/$n.json $n
}
run b1024 --dims 2 --size 1024 --steps 300 --pcg-steps 0 && run b2048 --dims 2 --size 2048 --steps 200 --pcg-steps 0 && \
run bcv --mode cv --steps 40 --warmup 5 && run b512 --pcg-steps 0
echo "rc=$?"
