#!/bin/bash
# r03d: fused backward after the load-order fix; k_gemm with the LDS-staged epilogue.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03d
rm -rf $O && mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_kernels_gpu.py -k "dwconv or conv1x1" > $O/pytest_k.log 2>&1 &&
EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so timeout -k 10 400 python tools/dw_bwd_probe.py \
    "16=0,17=2,16=2048" "6=0" > $O/dw_probe.txt 2> $O/dw_probe.err &&
timeout -k 10 300 python scripts/kbench.py --filter conv1x1,dwconv --top 200 --out $O/kb.txt > /dev/null 2> $O/kb.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench.json 2> $O/bench.log
rc=$?
tail -2 $O/pytest_k.log; cat $O/dw_probe.txt; head -12 $O/kb.txt; cut -c1-200 $O/bench.json
echo "r03d rc=$rc"
exit $rc
