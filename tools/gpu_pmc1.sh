# GPU box: one FETCH_SIZE pass over a short bench (kernel-trace beside --pmc only), then the summary.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_fetch
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/prof_fetch -o run --output-format csv -- python3 $R/bench.py --no-cpu --pcg-steps 0 --steps 2 --warmup 1 ${PROF_ARGS} > $R/gpurun_out/prof_fetch.log 2>&1
echo "pmc rc=$?"
