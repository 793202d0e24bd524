#!/bin/bash
# r03af: launch-size sweep (development slots 7 = wave-streaming GEMM grid cap, 6 = row-streaming
# depthwise forward / filter-gradient block target, 16 = fused depthwise backward block target,
# 14 = stride-2 depthwise dgrad block cap; 31 = unused, the production plan) over every D0 launch
# of the 1x1 forward / dgrad and depthwise entry points, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03af
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
F=conv1x1_fwd,conv1x1_dgrad,dwconv_fwd,dwconv_bwd,dwconv_dgrad,dwconv_wgrad
for rep in 1 2; do
for v in "31=0" "7=256" "7=1024" "7=2048" "6=512" "6=2048" "6=4096" "16=256" "16=512" "16=1024" "16=2048" "16=4096" \
         "14=1024" "14=2048" "14=8192"; do
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --filter $F --top 400 --dev $v \
      --out "$O/kb_${v}_$rep.txt" > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  echo "== $v rep $rep"; head -1 "$O/kb_${v}_$rep.txt"
done
done
