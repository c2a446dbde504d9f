#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04z_gpu_tests.log 2>&1 && tail -2 gpurun_out/r04z_gpu_tests.log &&
bash tools/gpu_abx.sh ab32 3 2 "" && bash tools/gpu_abx.sh ab33 2 2 ""
