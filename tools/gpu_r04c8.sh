#!/usr/bin/env bash
# conv8 fused-BN-backward y prefetch (G <= 4): parity under the knob, A/B, per-layer times.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
HCU_C8_DGRAD_G=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "unet or ops or modes" > $O/c8_tests.log 2>&1 || { tail -40 $O/c8_tests.log; exit 1; }
tail -1 $O/c8_tests.log
HCU_C8_DGRAD_G=4 timeout -k 10 200 python -u tools/layer_profile.py --steps 5 > $O/c8_layers.txt 2>&1 || { tail -30 $O/c8_layers.txt; exit 1; }
grep -E 'dgrad' $O/c8_layers.txt | grep conv8
bash tools/gpu_abx.sh c8ab 2 3 'HCU_C8_DGRAD_G=0' 'HCU_C8_DGRAD_G=4'
