#!/bin/bash
# r03aa: depthwise form sweep (development slot 27: 1 TILE, 2 DW3, 3 DIRECT, 4 DW4, 5 ROWS) over the
# D0 step's depthwise forward / dgrad / wgrad launches (the fused stride-1 backward is not routed
# by the form), each table twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03aa
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for rep in 1 2; do
for v in 0 1 2 3 4 5; do
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --filter dwconv_fwd,dwconv_dgrad,dwconv_wgrad --top 400 \
      --dev 27=$v --out $O/kb_${v}_$rep.txt > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  echo "== form $v rep $rep"; head -4 $O/kb_${v}_$rep.txt
done
done
