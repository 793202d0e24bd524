set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=tensorflow2-machine-vision_amd/lib
O=gpurun_out/r05i; mkdir -p $O
OLD=$L/libedet_base.so NEW=$L/libedet.so OLDENV="EDET_ALLOW_MISSING=1" REPS=2 TAG=r05i_abk HEADN=45 bash tools/ab_kbench.sh || exit 1
F=edet_lazy_bwd_apply,edet_lazy_materialize,edet_gate_bn_reduce,edet_lazy_bwd_reduce
for d in "" 8=2 8=4 8=8 8=16 8=32 13=4 13=8 13=16 12=8 12=16 10=8 10=16 10=32 9=512 9=1024; do
  tag=${d:-default}; tag=${tag//=/_}
  EDET_LIB=$L/libedet_dev.so timeout -k 10 300 python scripts/kbench.py --top 400 --filter $F ${d:+--dev $d} \
      --out $O/sweep_$tag.txt > $O/sweep_$tag.log 2>&1 || { echo "sweep $d failed"; tail -3 $O/sweep_$tag.log; exit 1; }
  head -6 $O/sweep_$tag.txt | sed "s/^/[$tag] /"
done
