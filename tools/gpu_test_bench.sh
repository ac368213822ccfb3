# GPU box: parity tests, then the 512^3 bench. Each step time-limited; a test ASSERTION failure
# (pytest exit 1) still lets the bench run, anything else (fault, abort, timeout) stops here.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest ${TEST_ARGS:-tests} -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc2=$?
echo "tests rc=$rc bench rc=$rc2"
exit $rc2
