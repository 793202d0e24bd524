#!/bin/bash
# Same-box per-launch A/B of two libraries (kbench replay tables), then tools/ab_kbench.py:
#   OLD=lib/libedet_base.so NEW=lib/libedet.so REPS=2 TAG=r04r bash tools/ab_kbench.sh
# OLDENV / NEWENV: extra environment per side, ';'-separated VAR=VALUE (commas stay inside a value:
# EDET_DEV_SLOTS=29=2,30=1024;EDET_LAZY_DY=0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-abk}
mkdir -p $O
L=tensorflow2-machine-vision_amd
for rep in $(seq 1 ${REPS:-2}); do
  for side in old new; do
    lib=$([ $side = old ] && echo ${OLD:-$L/lib/libedet_base.so} || echo ${NEW:-$L/lib/libedet.so})
    xenv=$([ $side = old ] && echo ${OLDENV:-} || echo ${NEWENV:-})
    env EDET_LIB=$lib $(echo $xenv | tr ';' ' ') timeout -k 10 400 python scripts/kbench.py --top 400 ${KB_ARGS:-} --out $O/kb_${rep}_$side.txt \
        > $O/kb_${rep}_$side.log 2>&1 || { echo "kbench $side failed"; tail -3 $O/kb_${rep}_$side.log; exit 1; }
  done
done
python tools/ab_kbench.py $O > $O/ab_kbench.txt
head -${HEADN:-60} $O/ab_kbench.txt
