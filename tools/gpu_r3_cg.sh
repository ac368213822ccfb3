#!/bin/bash
# fused CG tile height: PCG parity tests, then the 512^3 Jacobi-PCG leg with 8- and 16-wave tiles (probe
# build, same box, two rounds)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/cg
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spectral.py tests/test_gpu_fullsize.py -x -q --timeout 250 --timeout-method thread -k "pcg or PCG or 512 or rcpp or cpp or large" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
PL=$R/multivartv_amd/lib_probe/libmvtv.so
B="python bench.py --no-cpu --steps 4 --warmup 1 --pcg-steps 10"
for i in 1 2; do for nw in 8 16; do
  MVTV_LIB_PATH=$PL MVTV_CG3D_NW=$nw timeout -k 10 300 $B > $O/nw${nw}_$i.json 2>> $O/err.log || exit 1
done; done
for f in nw8_1 nw16_1 nw8_2 nw16_2; do python3 -c "import json; d=json.load(open('$O/$f.json')); p=d['pcg_leg']; print('$f', p['value'], p['kernel_avg_ms'], p['pcg_iters_mean'])"; done
cd /tmp && export TMPDIR=/tmp
for nw in 8 16; do
  MVTV_LIB_PATH=$PL MVTV_CG3D_NW=$nw timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch$nw -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 --pcg-steps 2 > $O/fetch$nw.log 2>&1 || exit 1
  MVTV_LIB_PATH=$PL MVTV_CG3D_NW=$nw timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write$nw -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 1 --warmup 0 --pcg-steps 2 > $O/write$nw.log 2>&1 || exit 1
done
echo rc=0
