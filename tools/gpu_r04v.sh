#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
HCU_CONV8_NPF16=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/r04v_tests.log 2>&1 || { tail -40 $O/r04v_tests.log; exit 1; }
tail -1 $O/r04v_tests.log
bash tools/gpu_abx.sh ab19 2 3 "" "HCU_CONV8_NPF16=1"
