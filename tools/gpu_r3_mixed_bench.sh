#!/bin/bash
# mixed-radix spectral: non-power-of-two meshes in the bench (spectral vs the Jacobi-PCG leg)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mixedb
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --no-cpu --dims 3 --size 500 --steps 10 --warmup 2 --pcg-steps 5 > $O/b500.json 2> $O/err.log &&
timeout -k 10 300 python bench.py --no-cpu --dims 2 --size 1000 --steps 50 --warmup 5 --pcg-steps 20 > $O/b1000.json 2>> $O/err.log &&
timeout -k 10 300 python bench.py --no-cpu --dims 3 --size 480 --steps 10 --warmup 2 --pcg-steps 5 > $O/b480.json 2>> $O/err.log &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt500 -o run --output-format csv -- python3 $R/bench.py --no-cpu --dims 3 --size 500 --steps 5 --warmup 1 --pcg-steps 0 > $O/kt500.log 2>&1
rc=$?
for f in b500 b1000 b480; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('pcg_leg',{}).get('value'), d['kernels'].get('dct',{}).get('avg_ms'))"; done
echo rc=$rc
