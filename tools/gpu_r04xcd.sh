#!/usr/bin/env bash
# XCD-contiguous bconv tile ranges (HCU_XCD_REMAP, default on): parity, A/B configs 2 and 3, layers
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "unet or ops or bf16 or modes" > $O/xcd_tests.log 2>&1 || { tail -40 $O/xcd_tests.log; exit 1; }
tail -1 $O/xcd_tests.log
bash tools/gpu_abx.sh xcd3 3 2 'HCU_XCD_REMAP=0' 'HCU_XCD_REMAP=1' || exit 1
bash tools/gpu_abx.sh xcd2 2 3 'HCU_XCD_REMAP=0' 'HCU_XCD_REMAP=1' || exit 1
timeout -k 10 200 python -u tools/layer_profile.py --config 3 --steps 5 > $O/xcd_layers3.txt 2>&1 || exit 1
head -14 $O/xcd_layers3.txt
