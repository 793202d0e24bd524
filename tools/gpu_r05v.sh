#!/bin/bash
# k_gate_bn_reduce slice width (dev slot 47 = vectors per slice; 46 = 2: unsliced), kbench replays
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for d in 0=0 46=2 47=4 47=16 47=32 0=0; do
  timeout -k 10 300 python scripts/kbench.py --top 400 --filter gate_bn_reduce --dev $d --out $O/kb_$d.txt > $O/kb_$d.log 2>&1 || exit 1
done
