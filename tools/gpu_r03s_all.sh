#!/bin/bash
# depthwise A/B (tools/gpu_r03ag.sh), then the round measurement (tools/gpu_r03sfinal.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r03ag.sh 2>/dev/null && bash tools/gpu_r03sfinal.sh
