#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_abx.sh ab17 2 3 "" "HCU_W3_TILES=3" "HCU_W3_TILES=1"
