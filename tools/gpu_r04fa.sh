#!/usr/bin/env bash
# switch test, then the measurement pass part a (GPU tests, config 2/3 profiles, PMC, SQ)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_modes.py -q --timeout 500 --timeout-method thread \
  -k "kernel_family" > $O/fb_tests.log 2>&1
rc=$?; tail -2 $O/fb_tests.log; grep -E '^E ' $O/fb_tests.log | cut -c1-1500 | head -4
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_final_a.sh r04 1
