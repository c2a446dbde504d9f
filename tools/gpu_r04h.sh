#!/usr/bin/env bash
# Full GPU test suite, then A/B of the defaults against HCU_AP=0, a graphed
# backward and weight-gradient grids sized for fewer CUs (HCU_SIDE_CUS).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/r04h_tests.log 2>&1 || { tail -40 $O/r04h_tests.log; exit 1; }
tail -1 $O/r04h_tests.log
bash tools/gpu_abx.sh ab5 2 2 "" "HCU_AP=0" "HCU_GRAPHS=1" "HCU_SIDE_CUS=192" "HCU_SIDE_CUS=128" "HIP_FORCE_DEV_KERNARG=1" || exit 1
bash tools/gpu_abx.sh ab6 3 1 "" "HCU_GRAPHS=1" "HCU_SIDE_CUS=192" "HCU_SIDE_CUS=128"
