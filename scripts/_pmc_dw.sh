set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_dw2
mkdir -p $O
EXP=$PWD/tensorflow2-machine-vision_amd/lib_exp/libedet.so
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
P2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
for shape in "32 32 32 672 5 1" "32 64 64 240 5 1"; do
  tag=$(echo $shape | tr ' ' '_')
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    ONLY=fwd EDET_LIB=$EXP timeout -s KILL 60 rocprofv3 --pmc $P --kernel-trace -d $O/${tag}_p$i -o run --output-format csv -- python scripts/dw_probe.py $shape > $O/${tag}_p$i.log 2>&1 || exit 1
    ONLY=dgrad timeout -s KILL 60 rocprofv3 --pmc $P --kernel-trace -d $O/${tag}_dg_p$i -o run --output-format csv -- python scripts/dw_probe.py $shape > $O/${tag}_dg_p$i.log 2>&1 || exit 1
  done
done
