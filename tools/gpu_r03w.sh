#!/bin/bash
# r03w: wave-streaming GEMM for narrow outputs over K <= 160 plain A (slot 23 = 1) on D0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03w
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for v in "" "23=1" "" "23=1"; do
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --filter conv1x1 --top 400 ${v:+--dev $v} \
      --out $O/kb_${v:-base}.txt > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  echo "== $v"; head -4 $O/kb_${v:-base}.txt; grep "N=96 K=16\|N=144 K=24\|K=96 N=24\|K=144 N=24" $O/kb_${v:-base}.txt | head -6
done
