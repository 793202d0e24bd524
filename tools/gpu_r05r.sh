#!/bin/bash
# 1x1 weight-gradient plan sweep per D0 shape on the current kernels: stage form (slot 21),
# min stages (slot 1), target blocks (slot 0); plain and lazy A (scripts/wg_probe.py)
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for cfg in none 21=1 21=3 21=4 1=4 1=8 1=32 21=3,1=4 21=3,1=8 0=4096 21=3,0=4096,1=4 2=1; do
  if [ "$cfg" = none ]; then unset EDET_DEV_SLOTS; else export EDET_DEV_SLOTS=$cfg; fi
  echo "### $cfg" >> $O/plain.txt
  timeout -k 10 150 python -u scripts/wg_probe.py >> $O/plain.txt 2>&1 || exit 1
  echo "### $cfg" >> $O/lazy.txt
  timeout -k 10 150 python -u scripts/wg_probe.py --lazy >> $O/lazy.txt 2>&1 || exit 1
done
