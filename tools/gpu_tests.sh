#!/usr/bin/env bash
# GPU parity tests only (optionally a subset): bash tools/gpu_tests.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-t}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ARGS=${*:-tests}
timeout -k 10 900 python -u -m pytest $ARGS -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
