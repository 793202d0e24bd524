#!/bin/bash
# r03ah: BiFPN fusion forward grid cap (development slot 28; 31 = unused, the uncapped plan) over
# every D0 and D4 fusion-forward launch, after the fusion tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ah
rm -rf $O && mkdir -p $O/d0 $O/d4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "fuse" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for rep in 1 2; do
for v in "31=0" "28=128" "28=256" "28=512" "28=1024" "28=2048"; do
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --filter bifpn_fuse_fwd --top 400 --dev $v \
      --out "$O/d0/kb_${v}_$rep.txt" > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --model efficientdet-d4 --batch 8 --filter bifpn_fuse_fwd --top 400 --dev $v \
      --out "$O/d4/kb_${v}_$rep.txt" > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  echo "== $v rep $rep"; head -1 "$O/d0/kb_${v}_$rep.txt"; head -1 "$O/d4/kb_${v}_$rep.txt"
done
done
