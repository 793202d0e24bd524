#!/bin/bash
# k_dwt next-tile register prefetch (dev slot 41 = 2) against the production tiled form
set -o pipefail
mkdir -p gpurun_out/r05ab
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
DWT_A=29=1 DWT_B=29=1,41=2 timeout -k 10 240 python -u tools/dwt_ab.py bf16 > gpurun_out/r05ab/dwt_pf_ab.txt 2>&1
