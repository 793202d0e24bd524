#!/bin/bash
# r03g: configs 2 and 5 re-measured on the current tree (bench lines with roofline tables),
# then the full GPU suite with parity reports.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03g
rm -rf $O && mkdir -p $O
timeout -k 10 400 python bench.py --workload backbone --batch 64 --steps 20 --warmup 5 --cpu-baseline 0 \
    > $O/r03g_config2_backbone_b64_bench.json 2> $O/config2.log &&
timeout -k 10 600 python bench.py --model efficientdet-d4 --batch 8 --steps 10 --warmup 3 --cpu-baseline 0 \
    > $O/r03g_config5_d4_b8_1gpu_bench.json 2> $O/config5.log
rc=$?
echo "bench rc=$rc"
cut -c1-400 $O/r03g_config2_backbone_b64_bench.json $O/r03g_config5_d4_b8_1gpu_bench.json
[ $rc -eq 0 ] || { tail -20 $O/config2.log $O/config5.log; exit $rc; }
EDET_REPORT_DIR=$O/parity timeout -k 10 1100 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/pytest_all.log 2>&1
rc=$?
tail -8 $O/pytest_all.log
echo "r03g rc=$rc"
exit $rc
