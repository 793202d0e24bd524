#!/bin/bash
# r03u: GEMM tests (D4 K = 224 shapes on the B-resident form) and config 5 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03u
rm -rf $O && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "conv1x1" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py --model efficientdet-d4 --batch 8 --steps 10 --warmup 3 --cpu-baseline 0 \
    > $O/r03u_config5_d4_b8_1gpu_bench.json 2> $O/config5.log
rc=$?
cut -c1-200 $O/r03u_config5_d4_b8_1gpu_bench.json
exit $rc
