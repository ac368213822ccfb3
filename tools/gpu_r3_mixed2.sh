#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mixed2
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_spectral.py tests/test_gpu_parity.py tests/test_gpu_cv.py tests/test_gpu_shims.py -x -q --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu --dims 3 --size 500 --steps 10 --warmup 2 --pcg-steps 5 > $O/b500.json 2> $O/err.log &&
timeout -k 10 300 python bench.py --no-cpu --dims 2 --size 1000 --steps 50 --warmup 5 --pcg-steps 20 > $O/b1000.json 2>> $O/err.log &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt500 -o run --output-format csv -- python3 $R/bench.py --no-cpu --dims 3 --size 500 --steps 5 --warmup 1 --pcg-steps 0 > $O/kt500.log 2>&1
rc=$?
for f in b500 b1000; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('pcg_leg',{}).get('value'), d['kernels'].get('dct',{}).get('avg_ms'))"; done
python3 - <<PY
import csv
for r in csv.DictReader(open('$O/kt500/run_kernel_stats.csv')):
    if float(r['Percentage'])>0.5: print('  ',r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
echo rc=$rc
