#!/bin/bash
# r03o: row-streaming depthwise forward: two steps in flight (slot 18 = 2), block targets (slot 6).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03o
rm -rf $O && mkdir -p $O
EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so timeout -k 10 300 python tools/dw_bwd_probe.py \
    "16=0" "6=0,18=2,6=2048,6=2048+18=2,6=4096+18=2" > $O/probe.txt 2> $O/probe.err
rc=$?
cat $O/probe.txt; tail -2 $O/probe.err
exit $rc
