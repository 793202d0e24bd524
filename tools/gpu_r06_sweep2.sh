#!/bin/bash
# Round-6 plan re-sweep under replicated statistics (the block caps of the statistics producers
# were set when every block's flush hit one fp64 vector): kbench replays of the development build,
# two repetitions per setting, then tools/sweep_table.py.  gpurun -- 'bash tools/gpu_r06_sweep2.sh'
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06v}; mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
run() {  # variant filter dev
  for rep in 1 2; do
    D=""; [ -n "$3" ] && D="--dev $3"
    timeout -k 10 300 python scripts/kbench.py --top 600 --reps 5 --filter $2 $D --out $O/kb_$1_$rep.txt > $O/kb_$1.log 2>&1 \
      || { tail -5 $O/kb_$1.log; return 1; }
  done
}
F=edet_lazy_bwd_reduce,edet_conv1x1_fwd,edet_dwconv_fwd,edet_lazy_materialize,edet_gate_bn_reduce
run base $F ""
run r1024 edet_lazy_bwd_reduce 11=1024
run r2048 edet_lazy_bwd_reduce 11=2048
run p8 edet_lazy_bwd_reduce 10=8
run g512 edet_conv1x1_fwd 7=512
run g1024 edet_conv1x1_fwd 7=1024
run g2048 edet_conv1x1_fwd 7=2048
run d2048 edet_dwconv_fwd 6=2048
run d1024 edet_dwconv_fwd 6=1024
run d4096 edet_dwconv_fwd 6=4096
python tools/sweep_table.py $O base x 0.03 > $O/sweep.txt
head -80 $O/sweep.txt
# whole-step A/B of the Python-side materialise policies (production library)
P=tensorflow2-machine-vision_amd/lib/libedet.so
STEPS=30 TAG=${TAG:-r06v}/ab REPS=3 VARIANTS="base:EDET_LIB=$P ms48:EDET_LIB=$P,EDET_MATERIALIZE_SE_MIN_N=48 ms1k:EDET_LIB=$P,EDET_MATERIALIZE_SE_MIN_N=1000 wm128:EDET_LIB=$P,EDET_WGRAD_MATERIALIZE_N=128 wm1k:EDET_LIB=$P,EDET_WGRAD_MATERIALIZE_N=100000" bash tools/ab_bench.sh
