#!/bin/bash
# k_dwt plan with chunks spanning images: tiles per block (dev slot 31) and block floor (30)
# against the production plan, tools/dwt_ab.py per D0 stride-1 shape
set -o pipefail
O=gpurun_out/r05ai
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for b in 31=2 31=4 31=8 31=16 30=384 30=1536; do
  DWT_A=29=1 DWT_B=29=1,$b timeout -k 10 240 python -u tools/dwt_ab.py bf16 > $O/ab_$b.txt 2>&1 || exit 1
done
