#!/usr/bin/env bash
# Parameter sweep (interleaved A/B): bf16 weight-gradient tiling knobs on
# config 3, grid sizing / K-split knobs on config 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_abx.sh ab8 3 2 "" "HCU_BW_TILE=1" "HCU_BW_OCC=1" "HCU_BW_CKA=16" "HCU_BW_CUS=240" "HCU_BCONV_LDS_KB=96" || exit 1
bash tools/gpu_abx.sh ab9 2 2 "" "HCU_SIDE_CUS=240" "HCU_SIDE_CUS=224" "HCU_BCONV_KS_TARGET=512" "HCU_BCONV_LDS_KB=96" "HCU_WGF_TILED=0"
