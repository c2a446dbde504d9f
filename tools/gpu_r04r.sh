#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_modes.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/r04r_tests.log 2>&1 || { tail -50 $O/r04r_tests.log; exit 1; }
tail -1 $O/r04r_tests.log
bash tools/gpu_abx.sh ab16 2 3 "" "HCU_CONVT_PHASE_WG=0" || exit 1
timeout -k 10 200 python -u tools/layer_profile.py --config 2 --steps 5 > $O/r04r_layers_config2.txt 2>&1 || exit 1
grep -E "\.up\.|total|finalize" $O/r04r_layers_config2.txt | head -20
