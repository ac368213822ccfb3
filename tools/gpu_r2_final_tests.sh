#!/bin/bash
# round-2: the new 128^4 eight-rank test, then the whole GPU suite and smoke
set -o pipefail
mkdir -p gpurun_out/r2f
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2f/full.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2f/gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2f/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r2f/full.log; tail -3 gpurun_out/r2f/gpu.log; echo rc=$rc
