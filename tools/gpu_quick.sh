# GPU box: GPU test suite, then a kernel-trace profile of a short bench (steps via PROF_STEPS).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest ${TEST_ARGS:-tests} -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 60 $R/tools/bin/stream_bench > $R/gpurun_out/stream.txt 2>&1 && cat $R/gpurun_out/stream.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_q -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps ${PROF_STEPS:-10} --warmup 2 ${BENCH_ARGS} > $R/gpurun_out/bench_q.json 2> $R/gpurun_out/bench_q.err
rc2=$?
echo "tests rc=$rc prof rc=$rc2"
exit $rc2
