#!/bin/bash
# r03l: per-shape depthwise backward plan (two rows per step), SE weight-gradient tiles -- kernel
# and model tests, probe, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03l
rm -rf $O && mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_kernels_large_gpu.py tests/test_model_gpu.py > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so timeout -k 10 300 python tools/dw_bwd_probe.py \
    "16=0,25=1" "6=0" > $O/probe.txt 2> $O/probe.err
rc=$?
tail -1 $O/probe.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench.json 2> $O/bench.log
rc=$?
tail -16 $O/bench.log
exit $rc
