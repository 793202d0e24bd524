#!/bin/bash
# r03p: K-loop GEMM tiles for the wide lazy expand convs (slot 23), and the depthwise tests for the
# two-steps-in-flight forward default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03p
rm -rf $O && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "dwconv" > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for v in "" "23=1" "23=2" "23=3" ""; do
  EDET_LIB=$DEV timeout -k 10 200 python scripts/kbench.py --filter conv1x1_fwd --top 12 \
      ${v:+--dev $v} --out $O/kb_${v:-base}.txt > /dev/null 2> $O/kb.err || exit 1
  echo "== $v"; head -2 $O/kb_${v:-base}.txt | tail -1; grep "N=1152 bn\|N=672 bn\|N=480 bn" $O/kb_${v:-base}.txt | head -4
done
