#!/bin/bash
# wave-streaming GEMM at three waves per SIMD (dev slot 50 = 1) for the lazy KS = 1 instances
set -o pipefail
O=gpurun_out/r05ad
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
SHAPES="2097152x16x96 524288x24x144 32768x16x96 131072x24x144"
for rep in 1 2; do
for cfg in none 50=1; do
  if [ "$cfg" = none ]; then unset EDET_DEV_SLOTS; else export EDET_DEV_SLOTS=$cfg; fi
  echo "### $cfg" >> $O/sweep.txt
  ONLY="fwd bn" timeout -k 10 150 python -u scripts/gemm_probe.py $SHAPES >> $O/sweep.txt 2>&1 || exit 1
done
done
