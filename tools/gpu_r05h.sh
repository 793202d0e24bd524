set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=tensorflow2-machine-vision_amd/lib
VARIANTS="nostats:EDET_LIB=$L/libedet_nostats.so base:EDET_LIB=$L/libedet_base.so,EDET_ALLOW_MISSING=1 fixed:EDET_LIB=$L/libedet.so" REPS=4 TAG=r05h_ab bash tools/ab_bench.sh
