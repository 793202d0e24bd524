#!/bin/bash
# Same-box A/B of whole-step throughput: alternates bench.py runs under environment settings.
#   VARIANTS="A:EDET_FOLD_GEMM_BN=1 B:EDET_FOLD_GEMM_BN=0" REPS=3 bash tools/ab_bench.sh
# One line per run: <variant> <images/s> <ms/step>; results in gpurun_out/${TAG:-ab}/ab.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
: > $O/ab.txt
for rep in $(seq 1 ${REPS:-3}); do
  for v in $VARIANTS; do
    name=${v%%:*}; envs=${v#*:}
    env $(echo $envs | tr ',' ' ') timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --cpu-baseline 0 \
        --kernel-timing 0 ${BENCH_ARGS:-} > $O/ab_$name.json 2> $O/ab_$name.log || { echo "$name failed"; tail -3 $O/ab_$name.log; exit 1; }
    python -c "import json;d=json.load(open('$O/ab_$name.json'));print('$name', d['value'], d['ms_per_step'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
