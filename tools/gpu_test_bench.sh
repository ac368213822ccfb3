# GPU box: parity tests, then the 512^3 bench (rank 0, N=1) — each step time-limited, chained with &&
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -3 gpurun_out/gpu_tests.log
echo "exit $rc"
