#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/r04y_tests.log 2>&1 || { tail -40 $O/r04y_tests.log; exit 1; }
tail -1 $O/r04y_tests.log
bash tools/gpu_abx.sh ab22 2 3 "" "HCU_LIB_PATH=$PWD/hcunet_amd/libhcunet_old.so" || exit 1
bash tools/gpu_abx.sh ab23 3 2 "" "HCU_LIB_PATH=$PWD/hcunet_amd/libhcunet_old.so"
