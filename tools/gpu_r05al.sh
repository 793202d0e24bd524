#!/bin/bash
# stem forward: output rows per block (dev slot 51), kbench replays
set -o pipefail
O=gpurun_out/r05al
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for d in 0=0 51=1 51=2 51=8 0=0; do
  timeout -k 10 300 python scripts/kbench.py --top 400 --filter stem_fwd --dev $d --out $O/kb_$d.txt > $O/kb_$d.log 2>&1 || exit 1
done
