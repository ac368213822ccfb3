# round 5: the inter-process slab tests (verbose, progress to a file), the stream ceiling, the default bench and the
# 2-process slab line through bench.py's launcher on the one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 120 tools/bin/stream_bench > $O/stream.txt 2>&1 || { echo "stream failed"; exit 1; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_slab_ipc.py -v -s -x --timeout 280 --timeout-method thread > $O/ipc.log 2>&1
rc=$?; tail -12 $O/ipc.log
if [ $rc -ne 0 ]; then echo "ipc tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --mode slab --steps 10 --warmup 2 > $O/bench_slab2.json 2> $O/bench_slab2.err
echo "slab2 rc=$?"
