#!/bin/bash
# class predict (174592 x 64 -> 729, plain, no statistics) and the other big plain products:
# production route vs the K loop at forced tiles (dev slots 26 = 4, 42 / 43 = BM / BN)
set -o pipefail
O=gpurun_out/r05ac
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
export ONLY="fwd plain"
SHAPES="174592x64x729 174592x64x36 174592x64x64"
for cfg in none 26=4 26=4,42=64,43=64 26=4,42=64,43=128 26=4,42=64,43=256 26=4,42=128,43=64 26=4,42=128,43=128 26=4,42=32,43=256 26=2 26=3; do
  if [ "$cfg" = none ]; then unset EDET_DEV_SLOTS; else export EDET_DEV_SLOTS=$cfg; fi
  echo "### $cfg" >> $O/sweep.txt
  timeout -k 10 150 python -u scripts/gemm_probe.py $SHAPES >> $O/sweep.txt 2>&1 || exit 1
done
