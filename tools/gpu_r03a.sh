#!/bin/bash
# r03a: counter calibration, depthwise parity (incl. the fused backward), GPU test suite,
# block-order and fused-backward A/B (kbench), PMC traffic of the step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03a
rm -rf $O && mkdir -p $O
DEVLIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash tools/gpu_calib.sh > $O/calib.log 2>&1
echo "calib rc=$?"
timeout -k 10 300 $PYT tests/test_kernels_gpu.py -k dwconv > $O/pytest_dw.log 2>&1 &&
timeout -k 10 240 python scripts/kbench.py --filter dwconv --top 150 --out $O/kb_fused.txt > /dev/null 2> $O/kb_fused.err &&
EDET_FUSED_DW=0 timeout -k 10 240 python scripts/kbench.py --filter dwconv,lazy_bwd --top 150 --out $O/kb_inner.txt > /dev/null 2> $O/kb_inner.err &&
EDET_FUSED_DW=0 EDET_LIB=$DEVLIB timeout -k 10 240 python scripts/kbench.py --filter dwconv --top 150 --dev 15=2 --out $O/kb_outer.txt \
    > /dev/null 2> $O/kb_outer.err &&
timeout -k 10 240 python scripts/kbench.py --filter lazy_bwd --top 80 --out $O/kb_fused_bn.txt > /dev/null 2> $O/kb_fused_bn.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench.json 2> $O/bench.log &&
EDET_FUSED_DW=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench_nofuse.json 2> $O/bench_nofuse.log &&
timeout -k 10 900 $PYT -m gpu tests > $O/pytest_all.log 2>&1
rc=$?
tail -3 $O/pytest_dw.log; head -8 $O/kb_fused.txt; head -8 $O/kb_inner.txt; head -8 $O/kb_outer.txt
tail -4 $O/pytest_all.log; cat $O/bench.json $O/bench_nofuse.json | cut -c1-300
echo "r03a rc=$rc"
exit $rc
