set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EDET_KERNEL_DETAIL=gpurun_out/detail.txt timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 > gpurun_out/detail_bench.json 2> gpurun_out/detail_bench.log
