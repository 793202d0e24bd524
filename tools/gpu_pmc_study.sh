#!/bin/bash
# SQ / TCC counter study of single launches (tools/one_launch.py), one rocprofv3 pass per
# counter group; each pass under its own time limit, the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_study
rm -rf $O && mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1
want() {  # keep the counters this box lists
  local out=""
  for c in "$@"; do grep -qw "$c" $O/counters.txt && out="$out $c"; done
  echo $out
}
PA=$(want SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS)
PB=$(want SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM)
echo "A: $PA" > $O/groups.txt; echo "B: $PB" >> $O/groups.txt
i=0
while read -r CASE; do
  i=$((i+1))
  for P in A B F W; do
    case $P in A) C="$PA";; B) C="$PB";; F) C="FETCH_SIZE";; W) C="WRITE_SIZE";; esac
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d $O/c${i}_$P -o run --output-format csv \
        -- python tools/one_launch.py $CASE > $O/c${i}_$P.log 2>&1 || { echo "case $i pass $P failed"; exit 1; }
  done
  echo "== case $i: $CASE" >> $O/table.txt
  grep "us/launch" $O/c${i}_A.log >> $O/table.txt
  python tools/pmc_table.py $O/c${i}_A $O/c${i}_B $O/c${i}_F $O/c${i}_W >> $O/table.txt
done <<'CASES'
dwfwd 32 128 128 144 3 1
dwbwd 32 128 128 144 3
dwfwd 32 16 16 1152 5 1
dwbwd 32 16 16 1152 5
gemm 8192 192 1152
wgrad 8192 1152 192
CASES
find $O -name "*.db" -delete
cat $O/groups.txt $O/table.txt
