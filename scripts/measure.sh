#!/bin/bash
# Round measurement on the GPU box: PMC traffic (two passes), the default bench line, and the
# rocprofv3 kernel-trace summary of the same bench command.  Every GPU step has its own time
# limit and the steps are chained: the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
TAG=${TAG:-r01}
BENCH="--steps ${STEPS:-20} --warmup ${WARMUP:-5}"
make -C tensorflow2-machine-vision_amd -j16 > $O/build.log 2>&1 || { echo "build failed"; exit 10; }
rm -rf $O/pmc_fetch $O/pmc_write $O/ktrace
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv \
    -- python bench.py --steps 3 --warmup 1 --graph 0 --cpu-baseline 0 --kernel-timing 0 > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv \
    -- python bench.py --steps 3 --warmup 1 --graph 0 --cpu-baseline 0 --kernel-timing 0 > $O/pmc_write.log 2>&1 &&
python scripts/pmc_traffic.py --fetch $O/pmc_fetch --write $O/pmc_write --out $O/pmc_traffic.json > $O/pmc_traffic.txt &&
cp $O/pmc_traffic.json profiles/pmc_traffic.json &&
timeout -k 10 900 python bench.py $BENCH > $O/bench_$TAG.json 2> $O/bench_$TAG.log &&
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv \
    -- python bench.py $BENCH --cpu-baseline 0 > $O/ktrace.log 2>&1
rc=$?
echo "measure rc=$rc"
cat $O/pmc_traffic.txt 2>/dev/null | head -12
tail -4 $O/bench_$TAG.log 2>/dev/null
cat $O/bench_$TAG.json 2>/dev/null
exit $rc
