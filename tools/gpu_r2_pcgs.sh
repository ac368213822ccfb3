#!/bin/bash
# scaled spectral-preconditioned PCG: parity tests, config-4 bench (AUTO -> PCG_SPECTRAL vs Jacobi), kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pcgs
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_config4_fold_path_2048_vs_c_oracle" -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode cv --steps 40 --warmup 5 > $O/bcv.json 2> $O/bcv.err || exit 1
timeout -k 10 300 python bench.py --mode cv --steps 40 --warmup 5 --solver pcg > $O/bcv_jacobi.json 2> $O/bcv_jacobi.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --mode cv --steps 20 --warmup 2 > $O/kt.log 2>&1
echo "rc=$?"
