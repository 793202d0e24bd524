#!/bin/bash
# r03n: same-box A/B of the whole step's launches: the r03e library (tree 231107d) against the
# current one, each kbench run twice (order ABBA).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03n
rm -rf $O && mkdir -p $O
OLD=tensorflow2-machine-vision_amd/lib/libedet_r03e.so
i=0
for lib in old new new old; do
  i=$((i+1))
  if [ $lib = old ]; then
    EDET_LIB=$OLD timeout -k 10 300 python scripts/kbench.py --abi-any --top 637 --out $O/kb_${i}_$lib.txt > /dev/null 2> $O/kb_${i}.err || exit 1
  else
    timeout -k 10 300 python scripts/kbench.py --top 637 --out $O/kb_${i}_$lib.txt > /dev/null 2> $O/kb_${i}.err || exit 1
  fi
  echo "== $i $lib"; head -1 $O/kb_${i}_$lib.txt
done
