#!/bin/bash
# BN row kernels at C = 1152: two vectors per thread (dev slot 52 = 1), kbench replays
set -o pipefail
O=gpurun_out/r05am
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for d in 0=0 52=1 0=0 52=1; do
  timeout -k 10 300 python scripts/kbench.py --top 400 --filter lazy_bwd,lazy_materialize,gate_bn_reduce,se_squeeze --dev $d --out $O/kb_$d.txt > $O/kb_$d.log 2>&1 || exit 1
  mv $O/kb_$d.txt $O/kb_${d}_$(date +%s%N).txt
done
