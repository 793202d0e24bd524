set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_dw
mkdir -p $O
CTR="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS"
for shape in "32 32 32 672 5 1" "32 128 128 144 3 1"; do
  tag=$(echo $shape | tr ' ' '_')
  for op in fwd wgrad dgrad; do
    ONLY=$op timeout -s KILL 60 rocprofv3 --pmc $CTR --kernel-trace -d $O/${tag}_$op -o run --output-format csv -- python scripts/dw_probe.py $shape > $O/${tag}_$op.log 2>&1 || exit 1
  done
done
python scripts/dw_probe.py 32 32 32 672 5 1 > $O/time.txt 2>&1
python scripts/dw_probe.py 32 128 128 144 3 1 >> $O/time.txt 2>&1
