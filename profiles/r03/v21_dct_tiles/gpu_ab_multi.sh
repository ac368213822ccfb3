set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/abm; mkdir -p $O
export MVTV_LIB_PATH=$GRAFT_REPO_ROOT/multivartv_amd/lib_probe/libmvtv.so
for rep in 1 2; do
  for e in base MVTV_DCT_T1=32 MVTV_DCT_T1=8 MVTV_DCT_T0=32 MVTV_DCT_T0=8; do
    if [ "$e" = base ]; then ev=""; else ev="$e"; fi
    env $ev timeout -k 10 200 python bench.py --no-cpu --pcg-steps 0 --steps 30 --warmup 5 > $O/$rep.$e.json 2> $O/$rep.$e.err || { tail -5 $O/$rep.$e.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],{k:v['avg_ms'] for k,v in d.get('kernels',{}).items()})" $O/$rep.$e.json "$e.$rep"
  done
done
