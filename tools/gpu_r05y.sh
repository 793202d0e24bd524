#!/bin/bash
# stem weight gradient: rows per strip (dev slot 48) and block cap (49), kbench replays
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for d in 0=0 48=1 48=1,49=1024 48=1,49=1280 48=1,49=2048 49=256 49=1024 48=4 48=4,49=256; do
  timeout -k 10 300 python scripts/kbench.py --top 400 --filter stem --dev $d --out $O/kb_$d.txt > $O/kb_$d.log 2>&1 || exit 1
done
