#!/bin/bash
# spectral MID-pass placement probe (probe build): z (default) vs y as the forward/divide/inverse dimension
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mid
mkdir -p $O
cd $R
for i in 1 2; do
  for mid in 2 1; do
    MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so MVTV_DCT_MID=$mid timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 > $O/mid${mid}_$i.json 2>> $O/err.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so MVTV_DCT_MID=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt1 -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps 10 --warmup 2 > $O/kt1.log 2>&1
echo "rc=$?"
