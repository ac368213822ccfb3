#!/bin/bash
# aligned fused kernel only (63-column kernel removed): fused / parity tests, whole GPU suite, bench, kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused3d.py -x -v --timeout 200 --timeout-method thread > $O/fused.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_kt -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 10 --warmup 2 > $O/prof_kt.log 2>&1
echo "kt rc=$?"
