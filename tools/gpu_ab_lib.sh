#!/bin/bash
# same-box A/B of two library builds (release lib vs multivartv_amd/lib_ab), interleaved bench runs
# usage: AB_ARGS="--pcg-steps 0" AB_REPS=3 bash tools/gpu_ab_lib.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ablib
mkdir -p $O
cd $R
for rep in $(seq 1 ${AB_REPS:-3}); do
  for v in new old; do
    if [ $v = old ]; then L=$R/multivartv_amd/lib_ab/libmvtv.so; else L=$R/multivartv_amd/lib/libmvtv.so; fi
    MVTV_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu ${AB_ARGS:---pcg-steps 0} > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail -5 $O/$v.$rep.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d['kernels'].items()})" $O/$v.$rep.json $v.$rep
  done
done
