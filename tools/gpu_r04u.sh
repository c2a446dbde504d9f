#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_abx.sh ab18 3 2 "" "HCU_BW_ZSPLIT=1"
