set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=tensorflow2-machine-vision_amd/lib
OLD=$L/libedet_base.so NEW=$L/libedet.so OLDENV="EDET_ALLOW_MISSING=1;EDET_LAZY_DY=0;EDET_SESUM_DGRAD=0" \
  NEWENV="EDET_LAZY_DY=0;EDET_SESUM_DGRAD=0" REPS=2 TAG=r05c_abk HEADN=80 bash tools/ab_kbench.sh
