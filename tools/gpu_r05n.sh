#!/bin/bash
# lazy_bwd_apply table build: TU = 8 / 4 channels per thread for the wide rows (dev slot 44)
# against TU = 2, per launch (kbench replay, dev library on both sides)
set -o pipefail
L=tensorflow2-machine-vision_amd/lib
export KB_ARGS="--filter lazy_bwd_apply"
TAG=r05n_tu8 OLD=$L/libedet_dev.so NEW=$L/libedet_dev.so NEWENV="EDET_DEV_SLOTS=44=8" REPS=2 HEADN=30 bash tools/ab_kbench.sh &&
TAG=r05n_tu4 OLD=$L/libedet_dev.so NEW=$L/libedet_dev.so NEWENV="EDET_DEV_SLOTS=44=4" REPS=2 HEADN=30 bash tools/ab_kbench.sh
