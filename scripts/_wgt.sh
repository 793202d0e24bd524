set -u
cd $GRAFT_REPO_ROOT
P=$PWD/tensorflow2-machine-vision_amd
: > gpurun_out/wg_sweep.txt
for v in lib lib_a lib_b lib_c lib_d; do
  echo "== $v" >> gpurun_out/wg_sweep.txt
  EDET_LIB=$P/$v/libedet.so timeout -k 10 120 python scripts/wg_probe.py >> gpurun_out/wg_sweep.txt 2>&1 || exit 1
done
