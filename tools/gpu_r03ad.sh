#!/bin/bash
# r03ad: BN row-kernel plan sweep (development slots 8/9 = apply passes per chunk / grid cap,
# 10/11 = reduce passes / cap, 12 = SE-fused reduce passes, 13 = materialize passes; 31 = unused,
# the production plan) over every D0 launch of those entry points, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ad
rm -rf $O && mkdir -p $O
DEV=tensorflow2-machine-vision_amd/lib/libedet_dev.so
F=lazy_bwd_apply,lazy_bwd_reduce,gate_bn_reduce,lazy_materialize
for rep in 1 2; do
for v in "31=0" "8=2" "8=4" "8=8" "8=16" "9=1024" "9=4096" "10=8" "10=16" "10=32" "10=64" "11=256" "11=1024" \
         "12=16" "12=64" "13=2" "13=4" "13=8" "13=16"; do
  EDET_LIB=$DEV timeout -k 10 300 python scripts/kbench.py --filter $F --top 400 --dev $v \
      --out "$O/kb_${v}_$rep.txt" > /dev/null 2> $O/kb.err || { tail -5 $O/kb.err; exit 1; }
  echo "== $v rep $rep"; head -1 "$O/kb_${v}_$rep.txt"
done
done
