#!/bin/bash
# r03b: fused depthwise backward / forward block-target sweep; full GPU suite with parity reports.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03b
rm -rf $O && mkdir -p $O
DEVLIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
EDET_LIB=$DEVLIB timeout -k 10 300 python tools/dw_bwd_probe.py 0,256,512,2048,4096 > $O/dw_probe.txt 2> $O/dw_probe.err
echo "probe rc=$?"
EDET_REPORT_DIR=$O/parity timeout -k 10 1500 python -u -m pytest -q --timeout 900 --timeout-method thread -m gpu tests \
    > $O/pytest_all.log 2>&1
rc=$?
cat $O/dw_probe.txt
tail -6 $O/pytest_all.log
echo "r03b rc=$rc"
exit $rc
