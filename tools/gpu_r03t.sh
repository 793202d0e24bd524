#!/bin/bash
# r03t: B-resident GEMM (k_pwb) for the D4 K = 224 convs (slot 23 = 2) and everywhere it fits
# (23 = 1), on D4 and D0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03t
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for m in "--model efficientdet-d4 --batch 8" "--model efficientdet-d0 --batch 32"; do
  for v in "" "23=2" "23=1"; do
    EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py $m --filter conv1x1 --top 30 ${v:+--dev $v} \
        --out $O/kb.txt > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
    echo "== $m $v"; head -4 $O/kb.txt; grep "K=224 N=224" $O/kb.txt | head -2
  done
done
