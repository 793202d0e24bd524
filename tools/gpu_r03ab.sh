#!/bin/bash
# r03ab: 1x1 weight-gradient plan sweep (development slots 0 = block target, 1 = min stages,
# 2 = partials (1 on, 2 off), 3 = wide wave-streaming tiles) over every D0 wgrad launch, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ab
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
i=0
for rep in 1 2; do
for v in "9=0" "0=1024" "0=4096" "1=4" "1=32" "2=1" "2=2" "3=1" "0=8192,1=2"; do
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --filter conv1x1_wgrad --top 400 --dev $v \
      --out "$O/kb_${v}_$rep.txt" > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  echo "== $v rep $rep"; head -2 "$O/kb_${v}_$rep.txt" | tail -1
done
done
