#!/bin/bash
# r03f: fused depthwise backward columns-per-thread sweep (development slot 20).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03f
EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so timeout -k 10 400 python tools/dw_bwd_probe.py \
    "16=0,20=2,20=1,20=2+16=2048,20=1+16=2048" "6=0" > gpurun_out/r03f/probe.txt 2> gpurun_out/r03f/probe.err
rc=$?
cat gpurun_out/r03f/probe.txt; tail -3 gpurun_out/r03f/probe.err
exit $rc
