#!/bin/bash
# r03i: LDS-DMA fused depthwise backward (k_dwg), unconditional loader loads -- kernel tests,
# probe against the register ring (slot 21 = 1) and ring depths (slot 22), then the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03i
rm -rf $O && mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_kernels_large_gpu.py > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so timeout -k 10 300 python tools/dw_bwd_probe.py \
    "16=0,21=1,22=2,22=4,16=512,16=2048" "6=0" > $O/probe.txt 2> $O/probe.err
rc=$?
cat $O/probe.txt; tail -3 $O/probe.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench.json 2> $O/bench.log
rc=$?
tail -16 $O/bench.log
exit $rc
