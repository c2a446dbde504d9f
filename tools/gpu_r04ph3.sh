#!/usr/bin/env bash
# ConvTranspose3d phase-form weight gradient on wgrad2 for u2.up / u3.up (HCU_CONVT_PHASE_WG=3): parity, A/B, layers
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
HCU_CONVT_PHASE_WG=3 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "unet and not bf16" > $O/ph3_tests.log 2>&1 || { tail -40 $O/ph3_tests.log; exit 1; }
tail -1 $O/ph3_tests.log
HCU_CONVT_PHASE_WG=3 timeout -k 10 200 python -u tools/layer_profile.py --steps 5 > $O/ph3_layers.txt 2>&1 || { tail -30 $O/ph3_layers.txt; exit 1; }
grep -E 'up\.wgrad|chansum' $O/ph3_layers.txt
bash tools/gpu_abx.sh ph3 2 3 'HCU_CONVT_PHASE_WG=2' 'HCU_CONVT_PHASE_WG=3'
