#!/bin/bash
# r03r: batched in-place B chunk loads in the A-resident GEMM (slot 24 = 1) on D4 (config 5) and D0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03r
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for m in "--model efficientdet-d4 --batch 8" "--model efficientdet-d0 --batch 32"; do
  for v in "" "24=1" ""; do
    EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py $m --filter conv1x1 --top 20 ${v:+--dev $v} \
        --out $O/kb.txt > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
    echo "== $m $v"; head -4 $O/kb.txt
  done
done
