#!/bin/bash
# r03y: GEMM route sweep (development slot 26: 1 wave-streaming, 2 B-resident, 3 A-resident,
# 4 K loop) over every conv1x1 fwd / dgrad launch of the D0 step, each table twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03y
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for rep in 1 2; do
for v in 0 1 2 3 4; do
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --filter conv1x1_fwd,conv1x1_dgrad --top 400 --dev 26=$v \
      --out $O/kb_${v}_$rep.txt > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  echo "== route $v rep $rep"; head -3 $O/kb_${v}_$rep.txt
done
done
