#!/usr/bin/env bash
# wgrad3 (output-split deep fp32 weight gradient) and the deeper bconv fragment
# prefetch: parity tests, then interleaved A/B on config 2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_modes.py tests/test_gpu_unet.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "wgrad2 or split_graphed or unet" > $O/r04l_tests.log 2>&1 || { tail -50 $O/r04l_tests.log; exit 1; }
tail -1 $O/r04l_tests.log
bash tools/gpu_abx.sh ab10 2 2 "" "HCU_WGRAD3=0" "HCU_LIB_PATH=$PWD/hcunet_amd/libhcunet_pf0.so" || exit 1
timeout -k 10 200 python -u tools/layer_profile.py --config 2 --steps 5 > $O/r04l_layers_config2.txt 2>&1 || exit 1
grep -E "wgrad3|total" $O/r04l_layers_config2.txt | head -20
