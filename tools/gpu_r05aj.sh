#!/bin/bash
# depthwise forward: form (dev slot 27: 1 tile, 2 dw3, 3 direct, 5 rows) and row-streaming block
# target (slot 6) over the step's launches, kbench replays
set -o pipefail
O=gpurun_out/r05aj
mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for d in 0=0 27=1 27=2 27=5 6=512 6=1024 6=4096 6=8192; do
  timeout -k 10 300 python scripts/kbench.py --top 400 --filter dwconv_fwd --dev $d --out $O/kb_$d.txt > $O/kb_$d.log 2>&1 || exit 1
done
