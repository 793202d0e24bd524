set -u
cd $GRAFT_REPO_ROOT
P=$PWD/tensorflow2-machine-vision_amd
true
true
: > gpurun_out/g_probe.txt
for v in lib lib_exp; do
  echo "== $v" >> gpurun_out/g_probe.txt
  EDET_LIB=$P/$v/libedet.so timeout -k 10 200 python scripts/gemm_probe.py 32768x112x672 32768x80x480 8192x192x1152 32768x672x112 8192x1152x192 32768x480x112 131072x40x240 >> gpurun_out/g_probe.txt 2>&1 || exit 1
done
