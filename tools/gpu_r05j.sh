set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=tensorflow2-machine-vision_amd/lib
O=gpurun_out/r05j; mkdir -p $O
VARIANTS="new:EDET_LIB=$L/libedet.so base:EDET_LIB=$L/libedet_base.so,EDET_ALLOW_MISSING=1" REPS=4 TAG=r05j_ab bash tools/ab_bench.sh &&
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/ktrace -o run --output-format csv \
    -- python bench.py --steps 6 --warmup 2 --cpu-baseline 0 --kernel-timing 0 > $O/ktrace.log 2>&1 &&
python scripts/trace_sum.py $O/ktrace 40 > $O/trace_sum.txt && cat $O/trace_sum.txt | head -60
find $O -name "*.db" -delete 2>/dev/null; true
