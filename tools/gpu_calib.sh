#!/bin/bash
# GPU box: FETCH_SIZE / WRITE_SIZE calibration (tools/pmc_calib.hip) and the counter list.
# Every GPU step has its own limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/calib
rm -rf $O && mkdir -p $O
timeout -k 10 120 tools/bin/pmc_calib > $O/plain.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o run --output-format csv \
    -- tools/bin/pmc_calib > $O/fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o run --output-format csv \
    -- tools/bin/pmc_calib > $O/write.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/hit -o run --output-format csv \
    -- tools/bin/pmc_calib > $O/hit.log 2>&1
rc=$?
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
cat $O/plain.txt
echo "calib rc=$rc"
exit $rc
