set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ktrace -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --cpu-baseline 0 --kernel-timing 0 > gpurun_out/ktrace.log 2>&1
