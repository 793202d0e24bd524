#!/bin/bash
# r03s: D4 (config 5) per-launch table of the conv and depthwise entry points; GEMM tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03s
rm -rf $O && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "conv1x1" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/kbench.py --model efficientdet-d4 --batch 8 --top 300 --out $O/kb_d4.txt > /dev/null 2> $O/kb.err
rc=$?
head -60 $O/kb_d4.txt
exit $rc
