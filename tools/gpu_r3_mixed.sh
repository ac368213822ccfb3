#!/bin/bash
# mixed-radix spectral solve: the whole GPU suite (many fixtures now take k_dctg under AUTO)
set -o pipefail
O=gpurun_out/mixed
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/gpu.log 2>&1
rc=$?; tail -30 $O/gpu.log; echo rc=$rc; exit $rc
