#!/bin/bash
# aligned fused 3-D kernel: parity tests, bench, same-box A/B against the 63-column kernel (probe build),
# FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/al
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_strip.py tests/test_gpu_parity.py tests/test_gpu_spectral.py tests/test_gpu_configs.py tests/test_gpu_zpick.py "tests/test_gpu_fullsize.py::test_metric_config_512_cubed" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu > $O/bench.json 2> $O/bench.err || exit 1
for i in 1 2; do
  for al in 0 1; do
    MVTV_LIB_PATH=$R/multivartv_amd/lib_probe/libmvtv.so MVTV_F3D_ALIGN=$al timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 > $O/ab_align${al}_$i.json 2>> $O/ab.err || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/prof_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 2 --steps 2 --warmup 1 > $O/prof_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/prof_write -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 2 --steps 2 --warmup 1 > $O/prof_write.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/calib_fetch -o run --output-format csv -- $R/tools/bin/pmc_calib > $O/calib_fetch.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/calib_write -o run --output-format csv -- $R/tools/bin/pmc_calib > $O/calib_write.log 2>&1
echo "pmc rc=$?"
