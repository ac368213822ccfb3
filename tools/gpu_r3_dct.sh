#!/bin/bash
# DCT register-pairing: spectral parity tests, then same-box A/B (lib_ab = previous DCT) and a kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dct
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_slab.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  MVTV_LIB_PATH=$R/multivartv_amd/lib_ab/libmvtv.so timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 > $O/old_$i.json 2>> $O/err.log || exit 1
  timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 > $O/new_$i.json 2>> $O/err.log || exit 1
done
for f in $O/old_1.json $O/new_1.json $O/old_2.json $O/new_2.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps 10 --warmup 2 > $O/kt.log 2>&1
echo "rc=$?"
