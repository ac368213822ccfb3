# round 5: measured per-rank time of the decomposed loop at G = 2 / 4 / 8 — one rank's share of the mesh (512^3:
# 256 / 128 / 64 planes; 128^4: 64 / 32 / 16) run at world 1 with MVTV_SLAB_DISTRIBUTED=1, so every kernel and
# collective call of a G-rank iteration runs (the collectives as RCCL transfers to the rank itself)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5h
mkdir -p $O
cd $R
for spec in "full3 0 512,512,512" "d3g1 1 512,512,512" "d3g2 1 512,512,256" "d3g4 1 512,512,128" "d3g8 1 512,512,64" \
            "full4 0 128,128,128,128" "d4g2 1 128,128,128,64" "d4g4 1 128,128,128,32" "d4g8 1 128,128,128,16"; do
  set -- $spec
  tag=$1; dist=$2; mesh=$3
  MVTV_SLAB_DISTRIBUTED=$dist timeout -k 10 300 python bench.py --mode slab --mesh $mesh --steps 20 --warmup 3 > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'],{k:v['avg_ms'] for k,v in d['kernels_rank0'].items()})" $O/$tag.json "$tag $mesh dist=$dist"
done
