# round 5: kernel trace of one G = 8 rank's share (512x512x64 and 128^3x16, world 1, distributed path) to see where the
# per-rank overhead of the decomposed loop goes (kernels, RCCL kernels, gaps)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
MVTV_SLAB_DISTRIBUTED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g8_3d -o run --output-format csv -- python3 $R/bench.py --mode slab --mesh 512,512,64 --steps 20 --warmup 3 > $O/g8_3d.log 2>&1 &&
MVTV_SLAB_DISTRIBUTED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g8_4d -o run --output-format csv -- python3 $R/bench.py --mode slab --mesh 128,128,128,16 --steps 20 --warmup 3 > $O/g8_4d.log 2>&1
echo "rc=$?"
