#!/bin/bash
# r03 round-end measurement: full GPU suite with parity reports, smoke, scripts/measure.sh
# (TAG=r03s: PMC traffic + MFMA passes, bench, rocprof kernel stats, kbench), configs 2 and 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03sfinal
rm -rf $O && mkdir -p $O
EDET_REPORT_DIR=$O/parity timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests \
    > $O/pytest_all.log 2>&1
rc=$?
tail -3 $O/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=r03s bash scripts/measure.sh > $O/measure.log 2>&1
rc=$?
tail -8 $O/measure.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload backbone --batch 64 --steps 20 --warmup 5 --cpu-baseline 0 \
    > $O/r03s_config2_backbone_b64_bench.json 2> $O/config2.log &&
timeout -k 10 600 python bench.py --model efficientdet-d4 --batch 8 --steps 10 --warmup 3 --cpu-baseline 0 \
    > $O/r03s_config5_d4_b8_1gpu_bench.json 2> $O/config5.log
rc=$?
cut -c1-160 $O/r03s_config2_backbone_b64_bench.json $O/r03s_config5_d4_b8_1gpu_bench.json
exit $rc
