#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_modes.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "bf16" > $O/r04p_tests.log 2>&1 || { tail -50 $O/r04p_tests.log; exit 1; }
tail -1 $O/r04p_tests.log
bash tools/gpu_abx.sh ab14 3 2 "" "HCU_BW_T44=0"
