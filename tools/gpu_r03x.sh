#!/bin/bash
# r03x: narrow-output wave-streaming GEMM route -- tests, and the K <= 256 / N <= 48 extension
# (slot 23 = 1) against the production route.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03x
rm -rf $O && mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "conv1x1" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for v in "" "23=1" "23=2" ""; do
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --filter conv1x1 --top 400 ${v:+--dev $v} \
      --out $O/kb_${v:-base}.txt > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  echo "== $v"; head -4 $O/kb_${v:-base}.txt; grep "K=240 N=40\|N=240 K=40\|K=144 N=40\|N=40 K=240" $O/kb_${v:-base}.txt | head -4
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-timing 0 > $O/bench.json 2> $O/bench.log
grep img/s $O/bench.log
