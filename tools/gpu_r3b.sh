#!/bin/bash
# fused 3-D kernel: dim-2 chunking sweep (probe build in multivartv_amd/lib_p) at 256^3, 512^3, 512x512x64
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3b
mkdir -p $O
export MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_p/libmvtv.so
timeout -k 10 200 python tools/zchunk_probe.py 256 3952 1976 1520 1216 988 760 608 > $O/z256.txt 2>&1 && \
timeout -k 10 300 python tools/zchunk_probe.py 512 4736 2368 3848 7696 9472 1184 > $O/z512.txt 2>&1 && \
timeout -k 10 200 python tools/zchunk_probe.py 512x512x64 3848 2368 1184 592 > $O/z512x64.txt 2>&1
