set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=tensorflow2-machine-vision_amd/lib
VARIANTS="base:EDET_LIB=$L/libedet_base.so,EDET_ALLOW_MISSING=1,EDET_LAZY_DY=0,EDET_SESUM_DGRAD=0 patches:EDET_LIB=$L/libedet.so,EDET_LAZY_DY=0,EDET_SESUM_DGRAD=0 lazy:EDET_LIB=$L/libedet.so,EDET_SESUM_DGRAD=0 new:EDET_LIB=$L/libedet.so" REPS=3 TAG=r05b_ab bash tools/ab_bench.sh &&
timeout -k 10 400 python scripts/kbench.py --top 400 --out gpurun_out/r05b_ab/r05b_kbench.txt > gpurun_out/r05b_ab/kbench.log 2>&1
