#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_abx.sh ab21 3 2 "" "HCU_BW_ZHALF=160" "HCU_BW_ZHALF=640"
