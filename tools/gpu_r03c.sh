#!/bin/bash
# r03c: two-rows-in-flight variants of the fused depthwise backward and the row-streaming forward.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03c
rm -rf $O && mkdir -p $O
EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so timeout -k 10 400 python tools/dw_bwd_probe.py \
    "16=0,17=2,16=2048+17=2,16=512+17=2" "6=0,18=2,6=2048+18=2,6=512+18=2" > $O/dw_probe.txt 2> $O/dw_probe.err
rc=$?
cat $O/dw_probe.txt; tail -3 $O/dw_probe.err
echo "r03c rc=$rc"
exit $rc
