set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/ka0.json 2> gpurun_out/ka0.log || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/ka1.json 2> gpurun_out/ka1.log || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/ka2.json 2> gpurun_out/ka2.log || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/ka3.json 2> gpurun_out/ka3.log || exit 1
