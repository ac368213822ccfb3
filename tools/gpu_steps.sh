# GPU box: pytest selection (TESTS), then optional probe commands (PROBE, one shell command), then the bench
# (BENCH_ARGS). Every GPU step is time-limited; a test assertion failure (pytest rc 1) lets the later steps run,
# anything else (fault, abort, timeout) stops the script there.
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
TAG=${TAG:-run}
if [ -n "$TESTS" ]; then
    timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest -v --maxfail=${MAXFAIL:-5} --timeout 300 --timeout-method thread \
        $TESTS > gpurun_out/${TAG}_tests.log 2>&1
    rc=$?
    tail -3 gpurun_out/${TAG}_tests.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
if [ -n "$PROBE" ]; then
    timeout -k 10 ${PROBE_TIMEOUT:-300} bash -c "$PROBE" > gpurun_out/${TAG}_probe.txt 2>&1 || { echo "probe failed"; exit 3; }
fi
if [ -n "$BENCH_ARGS" ]; then
    timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
    echo "bench rc=$?"
fi
