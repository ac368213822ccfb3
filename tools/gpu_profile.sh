# GPU box: rocprofv3 kernel-trace stats of the bench, then PMC passes (FETCH_SIZE and WRITE_SIZE in
# separate runs, kernel-trace only beside them) for the bench and for the calibration copy kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --steps ${PROF_STEPS:-5} --warmup 2 ${PROF_ARGS}"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_kt -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/prof_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 2 --warmup 1 ${PROF_ARGS} > $R/gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/prof_write -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 2 --warmup 1 ${PROF_ARGS} > $R/gpurun_out/prof_write.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/calib_fetch -o run --output-format csv -- $R/tools/bin/pmc_calib > $R/gpurun_out/calib_fetch.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/calib_write -o run --output-format csv -- $R/tools/bin/pmc_calib > $R/gpurun_out/calib_write.log 2>&1
echo "exit $?"
