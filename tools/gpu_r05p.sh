#!/bin/bash
# wave-streaming GEMM with the lazy activation as a compile-time case (dev slot 45 = 1)
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
SHAPES="2097152x16x96 524288x24x144 131072x40x64 2097152x32x16 32768x16x96"
for rep in 1 2; do
for cfg in none 45=1; do
  if [ "$cfg" = none ]; then unset EDET_DEV_SLOTS; else export EDET_DEV_SLOTS=$cfg; fi
  echo "### $cfg" >> $O/sweep.txt
  timeout -k 10 150 python -u scripts/gemm_probe.py $SHAPES >> $O/sweep.txt 2>&1 || exit 1
done
done
