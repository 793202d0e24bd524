#!/bin/bash
# r03ag: depthwise launch-size rules from the r03af sweep -- depthwise tests, then same-box A/B of the
# previous library (lib/libedet_prev.so) against the new one on D0 and D4 (ABBA), depthwise only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ag
rm -rf $O && mkdir -p $O/d0 $O/d4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "dwconv" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
PREV=tensorflow2-machine-vision_amd/lib/libedet_prev.so
for m in d0 d4; do
  if [ $m = d0 ]; then MA="--model efficientdet-d0 --batch 32"; else MA="--model efficientdet-d4 --batch 8"; fi
  i=0
  for lib in old new new old; do
    i=$((i+1))
    if [ $lib = old ]; then L=$PREV; else L=tensorflow2-machine-vision_amd/lib/libedet.so; fi
    EDET_LIB=$L timeout -k 10 300 python scripts/kbench.py $MA --filter dwconv_fwd,dwconv_bwd,dwconv_dgrad,dwconv_wgrad --top 2000 --out $O/$m/kb_${i}_$lib.txt > /dev/null 2> $O/kb.err \
        || { tail -5 $O/kb.err; exit 1; }
  done
  python tools/ab_kbench.py $O/$m | head -12
done
