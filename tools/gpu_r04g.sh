#!/usr/bin/env bash
# bf16 run-to-run determinism per feature, then per-feature A/B on configs 2 and 3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
OFF="HCU_AP=0 HCU_BNB_TAIL=0 HCU_CONVT_PHASE_WG=0 HCU_PREP_TILED=0 HCU_SPLIT_LAST=0"
timeout -k 10 500 python -u tools/det_check.py --bf16 "$OFF" "" "HCU_AP=0" "HCU_BNB_TAIL=0" "HCU_SPLIT_LAST=0" > $O/det_bf16.txt 2>&1 || { tail -20 $O/det_bf16.txt; exit 1; }
cat $O/det_bf16.txt
bash tools/gpu_abx.sh ab3 2 2 "$OFF" \
  "HCU_AP=0 HCU_CONVT_PHASE_WG=0 HCU_PREP_TILED=0 HCU_SPLIT_LAST=0" \
  "HCU_AP=0 HCU_BNB_TAIL=0 HCU_PREP_TILED=0 HCU_SPLIT_LAST=0" \
  "HCU_BNB_TAIL=0 HCU_CONVT_PHASE_WG=0 HCU_PREP_TILED=0 HCU_SPLIT_LAST=0" || exit 1
bash tools/gpu_abx.sh ab4 3 1 "$OFF" "HCU_AP=0 HCU_BNB_TAIL=0 HCU_CONVT_PHASE_WG=0 HCU_SPLIT_LAST=0" \
  "HCU_BNB_TAIL=0 HCU_CONVT_PHASE_WG=0 HCU_PREP_TILED=0 HCU_SPLIT_LAST=0"
