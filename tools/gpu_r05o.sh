#!/bin/bash
# wave-streaming GEMM grid (dev slot 7 = blocks) over the large D0 expand / narrow convs
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
SHAPES="2097152x16x96 524288x24x144 2097152x32x16 524288x144x24 524288x96x24 131072x40x64 174592x64x64"
for cfg in none 7=256 7=512 7=1024 7=2048 7=4096; do
  if [ "$cfg" = none ]; then unset EDET_DEV_SLOTS; else export EDET_DEV_SLOTS=$cfg; fi
  echo "### $cfg" >> $O/sweep.txt
  timeout -k 10 150 python -u scripts/gemm_probe.py $SHAPES >> $O/sweep.txt 2>&1 || exit 1
done
