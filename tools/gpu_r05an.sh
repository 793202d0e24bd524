#!/bin/bash
# BN-backward apply with nontemporal row loads / stores (dev slot 53 = 1, from slot 54 rows):
# all applies, and only those over >= 524288 rows; kbench replays
set -o pipefail
O=gpurun_out/r05an
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for d in 0=0 53=1 53=1,54=524288 0=0 53=1 53=1,54=524288; do
  timeout -k 10 300 python scripts/kbench.py --top 400 --filter lazy_bwd_apply --dev $d --out $O/kb.txt > $O/kb.log 2>&1 || exit 1
  mv $O/kb.txt $O/kb_${d}_$(date +%s%N).txt
done
