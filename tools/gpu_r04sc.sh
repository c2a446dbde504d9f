#!/usr/bin/env bash
# side_cus() (generic / wgrad2 weight-gradient grids) re-checked on config 2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_abx.sh sc2 2 3 'HCU_SIDE_CUS=224' 'HCU_SIDE_CUS=192' 'HCU_SIDE_CUS=256'
