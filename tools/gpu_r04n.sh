#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/r04n_tests.log 2>&1 || { tail -40 $O/r04n_tests.log; exit 1; }
tail -1 $O/r04n_tests.log
bash tools/gpu_abx.sh ab12 2 3 "" "HCU_WGRAD3=0"
