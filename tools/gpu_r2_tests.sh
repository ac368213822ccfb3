#!/bin/bash
# round-2 GPU check: new full-size tests, whole GPU suite, smoke, bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_slab.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_full.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err
