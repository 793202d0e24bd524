#!/bin/bash
# r03j: A-resident GEMM for the lazy expand convs (slot 23) with B prefetch to K = 256 (slot 24);
# depthwise backward block targets at k5; SE weight-gradient tiles (tests).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03j
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "squeeze or gate_bn or conv1x1 or dwconv" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in "" "23=1" "23=1,24=1" "24=1"; do
  EDET_LIB=$DEV timeout -k 10 200 python scripts/kbench.py --filter conv1x1_fwd,conv1x1_dgrad --top 40 \
      ${v:+--dev $v} --out $O/kb_${v:-base}.txt > /dev/null 2> $O/kb_${v:-base}.err || exit 1
  echo "== $v"; head -3 $O/kb_${v:-base}.txt
done
EDET_LIB=$DEV timeout -k 10 300 python tools/dw_bwd_probe.py "16=0,21=1,16=512,22=3+16=512" "6=0" > $O/probe.txt 2> $O/probe.err
rc=$?
cat $O/probe.txt
exit $rc
