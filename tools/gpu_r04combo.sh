#!/usr/bin/env bash
# A/Bs first (first-layer bwgrad grid, config 3; phase-form wgrad2, config 2), then the switch test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
bash tools/gpu_abx.sh cus0 3 3 'HCU_BW_CUS0=0' 'HCU_BW_CUS0=256' || exit 1
bash tools/gpu_r04ph3.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_modes.py -q --timeout 500 --timeout-method thread \
  -k "kernel_family" > $O/fb_tests.log 2>&1
rc=$?; tail -3 $O/fb_tests.log; grep -E '^E ' $O/fb_tests.log | cut -c1-1500 | head -6; exit $rc
