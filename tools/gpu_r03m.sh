#!/bin/bash
# r03m: SE tiles per (32 c, 8 r), GEMM register staging back to 4 vectors -- SE/GEMM tests,
# bench, kbench of the whole step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03m
rm -rf $O && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "squeeze or gate_bn or conv1x1" > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench.json 2> $O/bench.log &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-timing 0 > $O/bench2.json 2> $O/bench2.log &&
timeout -k 10 300 python scripts/kbench.py --top 400 --out $O/kbench.txt > /dev/null 2> $O/kbench.err
rc=$?
grep "img/s" $O/bench.log $O/bench2.log
head -30 $O/kbench.txt
exit $rc
