#!/bin/bash
# tridiagonal last-dimension pass: spectral parity tests, then same-box A/B in the probe build
# (MVTV_DCT_TRI=0: FFT MID pass; MVTV_TRI_SEG=32: 32 rows per thread) and a kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tri
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_fullsize.py tests/test_gpu_slab.py tests/test_gpu_configs.py -x -q --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
PL=$R/multivartv_amd/lib_probe/libmvtv.so
for i in 1 2; do
  MVTV_LIB_PATH=$PL MVTV_DCT_TRI=0 timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 > $O/fft_$i.json 2>> $O/err.log || exit 1
  MVTV_LIB_PATH=$PL timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 > $O/tri16_$i.json 2>> $O/err.log || exit 1
  MVTV_LIB_PATH=$PL MVTV_TRI_SEG=32 timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 > $O/tri32_$i.json 2>> $O/err.log || exit 1
done
for f in fft_1 tri16_1 tri32_1 fft_2 tri16_2 tri32_2; do python -c "import json; d=json.load(open('$O/$f.json')); k=d['kernels']; print('$f', d['value'], d['ms_per_step'], k['dct']['avg_ms'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps 10 --warmup 2 > $O/kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt4 -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps 5 --warmup 1 --dims 4 --size 128 > $O/kt4.log 2>&1
echo "rc=$?"
