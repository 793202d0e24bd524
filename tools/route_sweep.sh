set -u
O=gpurun_out/r04ad; mkdir -p $O/d0 $O/d4
export EDET_LIB=tensorflow2-machine-vision_amd/lib/libedet_dev.so
for m in d0 d4; do
  if [ $m = d0 ]; then MA="--model efficientdet-d0 --batch 32"; else MA="--model efficientdet-d4 --batch 8"; fi
  for r in 0 2 3 4; do
    D=""; [ $r != 0 ] && D="--dev 26=$r"
    timeout -k 10 300 python scripts/kbench.py $MA --top 600 --reps 5 --filter edet_conv1x1_fwd,edet_conv1x1_dgrad $D --out $O/$m/kb_r${r}_1.txt > $O/kb_${m}_$r.log 2>&1 || { mkdir -p $O/$m; timeout -k 10 300 python scripts/kbench.py $MA --top 600 --reps 5 --filter edet_conv1x1_fwd,edet_conv1x1_dgrad $D --out $O/$m/kb_r${r}_1.txt > $O/kb_${m}_$r.log 2>&1 || exit 1; }
  done
done
echo swept
