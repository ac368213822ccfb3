#!/bin/bash
# config 3 (256^3) and config 5 (128^4) kernel traces and FETCH_SIZE / WRITE_SIZE passes (own runs each)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3c
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused3d.py tests/test_gpu_parity.py \
  tests/test_gpu_slab.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --dims 3 --size 256 > $O/b256.json 2> $O/b256.err || exit 1
timeout -k 10 300 python bench.py --no-cpu > $O/b512.json 2> $O/b512.err || exit 1
timeout -k 10 300 python bench.py --mode cv --steps 40 --warmup 5 > $O/cv4.json 2> $O/cv4.err || exit 1
cd /tmp && export TMPDIR=/tmp
pmc() {  # name counter args...
  local n=$1 c=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d $O/${n}_$c -o run --output-format csv -- python3 $R/bench.py --no-cpu "$@" > $O/${n}_$c.log 2>&1
}
kt() {
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o run --output-format csv -- python3 $R/bench.py --no-cpu "$@" > $O/kt_$n.log 2>&1
}
kt b256 --dims 3 --size 256 --pcg-steps 0 --steps 20 --warmup 3 && \
pmc b256 FETCH_SIZE --dims 3 --size 256 --pcg-steps 0 --steps 3 --warmup 1 && \
pmc b256 WRITE_SIZE --dims 3 --size 256 --pcg-steps 0 --steps 3 --warmup 1 && \
kt b128_4d --dims 4 --size 128 --pcg-steps 0 --steps 6 --warmup 2 && \
pmc b128_4d FETCH_SIZE --dims 4 --size 128 --pcg-steps 0 --steps 2 --warmup 1 && \
pmc b128_4d WRITE_SIZE --dims 4 --size 128 --pcg-steps 0 --steps 2 --warmup 1 && \
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/calib_fetch -o run --output-format csv -- $R/tools/bin/pmc_calib > $O/calib_fetch.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/calib_write -o run --output-format csv -- $R/tools/bin/pmc_calib > $O/calib_write.log 2>&1
echo "rc=$?"
