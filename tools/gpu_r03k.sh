#!/bin/bash
# r03k: two output rows per step in the register-ring depthwise backward (slot 25 = 2) against the
# production plan (k3 register ring, k5 DMA rings) and the register ring everywhere (21 = 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03k
rm -rf $O && mkdir -p $O
EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so timeout -k 10 300 python tools/dw_bwd_probe.py \
    "16=0,21=1,21=1+25=2,21=1+25=2+16=512,21=1+25=2+16=2048" "6=0" > $O/probe.txt 2> $O/probe.err
rc=$?
cat $O/probe.txt; tail -3 $O/probe.err
exit $rc
