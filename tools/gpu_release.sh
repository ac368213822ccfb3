# GPU box, end-of-milestone evidence: full GPU test suite, the default bench (with cpu_baseline),
# a rocprofv3 kernel-trace of the bench, FETCH_SIZE / WRITE_SIZE passes (separate runs) and the
# PMC calibration copies. Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=${REL_OUT:-gpurun_out/rel}
mkdir -p $R/$O
cd $R
# SKIP_TESTS=1: the evidence steps only (the suite in a call of its own: gpurun's 20-minute cap)
rc=0
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -2 $O/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 60 tools/bin/stream_bench > $O/stream.txt 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_kt -o run --output-format csv -- python3 $R/bench.py --no-cpu --steps 10 --warmup 2 > $R/$O/prof_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/prof_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 2 --steps 2 --warmup 1 > $R/$O/prof_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$O/prof_write -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 2 --steps 2 --warmup 1 > $R/$O/prof_write.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/$O/calib_fetch -o run --output-format csv -- $R/tools/bin/pmc_calib > $R/$O/calib_fetch.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/$O/calib_write -o run --output-format csv -- $R/tools/bin/pmc_calib > $R/$O/calib_write.log 2>&1
rc2=$?; cd $R; [ $rc2 -eq 0 ] && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "tests rc=$rc release rc=$rc2 smoke rc=$?"
