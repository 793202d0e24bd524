set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=tensorflow2-machine-vision_amd/lib
VARIANTS="fixed:EDET_LIB=$L/libedet.so base:EDET_LIB=$L/libedet_base.so,EDET_ALLOW_MISSING=1" REPS=4 TAG=r05g_ab bash tools/ab_bench.sh
