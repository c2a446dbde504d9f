#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_modes.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "wgrad2" > $O/r04m_tests.log 2>&1 || { tail -50 $O/r04m_tests.log; exit 1; }
tail -1 $O/r04m_tests.log
timeout -k 10 200 python -u tools/layer_profile.py --config 2 --steps 5 > $O/r04m_layers_config2.txt 2>&1 || exit 1
grep -E "wgrad3|total" $O/r04m_layers_config2.txt | head -20
bash tools/gpu_abx.sh ab11 2 2 "" "HCU_WGRAD3=0"
