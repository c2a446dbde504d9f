#!/usr/bin/env bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r04cus0.sh && bash tools/gpu_r04ph3.sh
