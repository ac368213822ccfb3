set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --size 256 --no-cpu > gpurun_out/bench256.json 2> gpurun_out/bench256.err && \
timeout -k 10 600 python bench.py > gpurun_out/bench512.json 2> gpurun_out/bench512.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
echo "exit $?"
