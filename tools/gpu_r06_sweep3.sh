#!/bin/bash
# Round-6 plan re-sweep of the BN-backward apply and materialize (development build, kbench
# replays, two repetitions per setting): slot 8 = apply passes, 9 = apply block cap, 13 =
# materialize passes.   gpurun -- 'bash tools/gpu_r06_sweep3.sh'  (libedet_dev.so un-ignored)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06ae}; mkdir -p $O
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
run() {  # variant filter dev
  for rep in 1 2; do
    D=""; [ -n "$3" ] && D="--dev $3"
    timeout -k 10 300 python scripts/kbench.py --top 600 --reps 5 --filter $2 $D --out $O/kb_$1_$rep.txt > $O/kb_$1.log 2>&1 \
      || { tail -5 $O/kb_$1.log; return 1; }
  done
}
run base edet_lazy_bwd_apply,edet_lazy_materialize ""
run a2 edet_lazy_bwd_apply 8=2
run a8 edet_lazy_bwd_apply 8=8
run a16 edet_lazy_bwd_apply 8=16
run c1024 edet_lazy_bwd_apply 9=1024
run c4096 edet_lazy_bwd_apply 9=4096
run m2 edet_lazy_materialize 13=2
run m8 edet_lazy_materialize 13=8
run m16 edet_lazy_materialize 13=16
python tools/sweep_table.py $O base x 0.03 > $O/sweep.txt
head -60 $O/sweep.txt
