#!/bin/bash
# Round measurement on the GPU box (TAG=r03x bash scripts/measure.sh):
#   1. PMC traffic, two passes (FETCH_SIZE, WRITE_SIZE)      -> pmc_traffic.json / _pmc_traffic.txt
#   2. PMC MFMA utilisation (SQ_VALU_MFMA_BUSY_CYCLES)       -> pmc_mfma.json / _pmc_mfma.txt
#   2b. PMC wave-time breakdown + instruction mix, two passes -> pmc_limiter.json / _pmc_limiter.txt
#   3. the default bench line, with the JSONs of 1-2 in profiles/ so its table reads them
#   4. rocprofv3 --kernel-trace --stats of the same bench command
#   5. scripts/kbench.py per-launch replay table
# Every GPU step has its own time limit and the steps are chained: the first failure ends it.
# Results land in gpurun_out/$TAG/; copy them to profiles/ (named by TAG) to commit them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/$TAG
rm -rf $O/pmc_fetch $O/pmc_write $O/pmc_mfma $O/pmc_lima $O/pmc_limb $O/ktrace && mkdir -p $O
BENCH="--steps ${STEPS:-20} --warmup ${WARMUP:-5}"
EAGER="python bench.py --steps 3 --warmup 1 --graph 0 --cpu-baseline 0 --kernel-timing 0"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o run --output-format csv \
    -- $EAGER > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o run --output-format csv \
    -- $EAGER > $O/pmc_write.log 2>&1 &&
python scripts/pmc_traffic.py --fetch $O/pmc_fetch --write $O/pmc_write --steps 6 --tag $TAG \
    --out $O/pmc_traffic.json > $O/${TAG}_pmc_traffic.txt &&
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma -o run \
    --output-format csv -- $EAGER > $O/pmc_mfma.log 2>&1 &&
python scripts/pmc_mfma.py --dir $O/pmc_mfma --steps 6 --tag $TAG --out $O/pmc_mfma.json > $O/${TAG}_pmc_mfma.txt &&
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_lima -o run \
    --output-format csv -- $EAGER > $O/pmc_lima.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_limb -o run \
    --output-format csv -- $EAGER > $O/pmc_limb.log 2>&1 &&
python scripts/pmc_limiter.py --a $O/pmc_lima --b $O/pmc_limb --steps 6 --tag $TAG --out $O/pmc_limiter.json \
    > $O/${TAG}_pmc_limiter.txt &&
cp $O/pmc_traffic.json $O/pmc_mfma.json $O/pmc_limiter.json profiles/ &&
timeout -k 10 900 python bench.py $BENCH > $O/${TAG}_bench.json 2> $O/${TAG}_bench.log &&
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/ktrace -o run --output-format csv \
    -- python bench.py $BENCH --cpu-baseline 0 > $O/ktrace.log 2>&1 &&
cp $(find $O/ktrace -name "*kernel_stats.csv" | head -1) $O/${TAG}_kernel_stats.csv &&
timeout -k 10 300 python scripts/kbench.py --top 400 --out $O/${TAG}_kbench.txt > /dev/null 2> $O/kbench.err
rc=$?
# counter databases are large and not needed once summarised
find $O -name "*.db" -delete 2>/dev/null
echo "measure rc=$rc"
head -12 $O/${TAG}_pmc_traffic.txt 2>/dev/null
head -12 $O/${TAG}_pmc_mfma.txt 2>/dev/null
head -16 $O/${TAG}_pmc_limiter.txt 2>/dev/null
tail -4 $O/${TAG}_bench.log 2>/dev/null
cut -c1-400 $O/${TAG}_bench.json 2>/dev/null
exit $rc
