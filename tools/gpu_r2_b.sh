#!/bin/bash
# round-2 boundary check: new C++/Python API tests, zpick identity, then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cxx_cpp.py tests/test_gpu_shims.py tests/test_gpu_zpick.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r2b_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2b_gpu.log 2>&1
