#!/bin/bash
# kbench per-launch sweep of development plan slots (lib/libedet_devx.so = `make dev` output
# under another name, so it travels): SWEEP="base 9=256 9=512" FILTER=lazy_bwd_apply
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06s}
mkdir -p $O
for v in ${SWEEP:-base}; do
  dev=$([ "$v" = base ] && echo "" || echo "--dev $v")
  EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_devx.so timeout -k 10 300 python scripts/kbench.py --top 400 \
      --filter ${FILTER:-lazy} $dev --out $O/kb_${v//[=,]/_}.txt > $O/kb_${v//[=,]/_}.log 2>&1 || { echo "$v failed"; tail -3 $O/kb_${v//[=,]/_}.log; exit 1; }
  echo "$v: $(head -1 $O/kb_${v//[=,]/_}.txt)"
done
