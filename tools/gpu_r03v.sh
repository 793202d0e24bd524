#!/bin/bash
# r03v: wave-streaming GEMM grid (slot 7) on D0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03v
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for v in "" "7=2048" "7=4096" "7=256" ""; do
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --filter conv1x1 --top 400 ${v:+--dev $v} \
      --out $O/kb_${v:-base}.txt > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  echo "== $v"; head -4 $O/kb_${v:-base}.txt; grep "M=2097152" $O/kb_${v:-base}.txt | head -4
done
