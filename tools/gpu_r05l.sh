#!/bin/bash
# K-loop GEMM tile sweep (dev slots 26 = 4 K loop, 42 / 43 = BM / BN) over the mid-size D0
# conv1x1 shapes that run at 0.4-1.6 TB/s in kbench (scripts/gemm_probe.py, all variants)
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
SHAPES="8192x192x1152 8192x1152x320 8192x1152x192 8192x672x192 8192x320x64 32768x112x672 32768x80x480 32768x672x112 32768x480x112 32768x480x80 131072x40x240 32768x112x64"
for cfg in none 26=4 26=4,42=32,43=64 26=4,42=32,43=128 26=4,42=32,43=256 26=4,42=64,43=64 26=4,42=64,43=128 26=4,42=64,43=256 26=4,42=128,43=64 26=4,42=128,43=128; do
  if [ "$cfg" = none ]; then unset EDET_DEV_SLOTS; else export EDET_DEV_SLOTS=$cfg; fi
  echo "### $cfg" >> $O/sweep.txt
  timeout -k 10 150 python -u scripts/gemm_probe.py $SHAPES >> $O/sweep.txt 2>&1 || exit 1
done
