# round 5: env probe, the whole GPU suite with achieved parity errors logged, the default bench, and the slab
# loop across 2 rank processes on the one GPU (ipc transport) through bench.py's launcher
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a
mkdir -p $O
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'OMP', os.environ.get('OMP_NUM_THREADS'))" > $O/env.txt
cat /sys/fs/cgroup/cpu.max >> $O/env.txt 2>&1
MVTV_PARITY_LOG=$PWD/$O/parity.jsonl timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 tools/bin/stream_bench > $O/stream.txt 2>&1 || { echo "stream failed"; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --mode slab --steps 10 --warmup 2 > $O/bench_slab2.json 2> $O/bench_slab2.err
echo "slab2 rc=$?"
