#!/bin/bash
# Round-6 re-sweep of the tiled depthwise backward's launch plan (development build, kbench
# replays): slot 30 = block floor, slot 31 = tiles per block.  (libedet_dev.so un-ignored)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06ak}; mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so EDET_ALLOW_MISSING=1
run() {  # variant dev
  for rep in 1 2; do
    D=""; [ -n "$2" ] && D="--dev $2"
    timeout -k 10 300 python scripts/kbench.py --top 600 --reps 5 --filter edet_dwconv_bwd $D --out $O/kb_$1_$rep.txt > $O/kb_$1.log 2>&1 \
      || { tail -5 $O/kb_$1.log; return 1; }
  done
}
if [ "${SWEEP:-plan}" = gemm ]; then
  F=edet_conv1x1_fwd,edet_conv1x1_dgrad
  runf() { for rep in 1 2; do D=""; [ -n "$2" ] && D="--dev $2"
    timeout -k 10 300 python scripts/kbench.py --top 600 --reps 5 --filter $F $D --out $O/kb_$1_$rep.txt > $O/kb_$1.log 2>&1 \
      || { tail -5 $O/kb_$1.log; return 1; }; done; }
  runf base ""
  runf m64n64 42=64,43=64
  runf m128n64 42=128,43=64
  runf m64n128 42=64,43=128
  runf m32n64 42=32,43=64
  runf m32n128 42=32,43=128
  runf m128n128 42=128,43=128
elif [ "${SWEEP:-plan}" = dwform ]; then
  F=edet_dwconv_fwd,edet_dwconv_wgrad
  runf() { for rep in 1 2; do D=""; [ -n "$2" ] && D="--dev $2"
    timeout -k 10 300 python scripts/kbench.py --top 600 --reps 5 --filter $F $D --out $O/kb_$1_$rep.txt > $O/kb_$1.log 2>&1 \
      || { tail -5 $O/kb_$1.log; return 1; }; done; }
  runf base ""
  runf tile 27=1
  runf dw3 27=2
  runf rows 27=5
elif [ "${SWEEP:-plan}" = form ]; then
  run base ""
  run rows 29=2
  run rows512 29=2,16=512
  run rows2048 29=2,16=2048
else
  run base ""
  run f384 30=384
  run f1536 30=1536
  run f3072 30=3072
  run t1 31=1
  run t2 31=2
  run t4 31=4
fi
python tools/sweep_table.py $O base x 0.0 > $O/sweep.txt
head -40 $O/sweep.txt
