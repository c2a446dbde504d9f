#!/usr/bin/env bash
# kernel-family switch test + first-layer bwgrad grid A/B (config 3)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_modes.py -x -q --timeout 500 --timeout-method thread \
  -k "kernel_family" > $O/fb_tests.log 2>&1 || { tail -40 $O/fb_tests.log; exit 1; }
tail -1 $O/fb_tests.log
bash tools/gpu_abx.sh cus0 3 3 'HCU_BW_CUS0=0' 'HCU_BW_CUS0=256'
