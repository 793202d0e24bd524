#!/bin/bash
# r03e: the round measurement (scripts/measure.sh) then the forward depthwise variants probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r03e bash scripts/measure.sh > gpurun_out/r03e_measure.log 2>&1
rc=$?
echo "measure rc=$rc"
[ $rc -eq 0 ] || exit $rc
EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so timeout -k 10 400 python tools/dw_bwd_probe.py \
    "16=0" "6=0,19=1,6=2048+19=1,6=512+19=1" > gpurun_out/r03e/dw_probe_fwd.txt 2> gpurun_out/r03e/dw_probe_fwd.err
rc=$?
tail -20 gpurun_out/r03e_measure.log
cat gpurun_out/r03e/dw_probe_fwd.txt
exit $rc
