#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_abx.sh ab15 2 2 "" "HCU_CONV8_G=4" "HCU_CONV8_G=2" "HCU_NO_CONV8=1"
