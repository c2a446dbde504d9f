#!/usr/bin/env bash
# bwgrad grid size for the non-first layers, with the first layer at 256 CUs (config 3)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_abx.sh bwc 3 2 'HCU_BW_CUS=224' 'HCU_BW_CUS=208' 'HCU_BW_CUS=240'
