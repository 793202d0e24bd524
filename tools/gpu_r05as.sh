#!/bin/bash
# nontemporal apply rows from 131072 rows (dev slots 53 = 1, 54) against the production 524288,
# dev library both sides, kbench replays of the applies
set -o pipefail
L=tensorflow2-machine-vision_amd/lib
TAG=r05as OLD=$L/libedet_dev.so NEW=$L/libedet_dev.so OLDENV="EDET_DEV_SLOTS=53=1,54=524288" \
  NEWENV="EDET_DEV_SLOTS=53=1,54=131072" REPS=2 KB_ARGS="--filter lazy_bwd_apply" HEADN=30 bash tools/ab_kbench.sh
