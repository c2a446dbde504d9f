#!/usr/bin/env bash
# Kernel-trace timelines (rocpd databases kept under gpurun_out/) of the
# bench step for each environment setting given, config CONFIG.
#   bash tools/gpu_tl.sh TAG CONFIG 'ENV_A' ['ENV_B' ...]
set -o pipefail
TAG=$1; CFG=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
k=0
for arm in "$@"; do
  k=$((k + 1))
  # (rocprofv3 must start the program itself: the arm's settings are exported first)
  for kv in $arm; do export "$kv"; done
  timeout -k 10 240 rocprofv3 --kernel-trace -d $O/${TAG}_tl$k -o run -- python3 bench.py --config "$CFG" \
    --steps 8 --warmup 4 --no-cpu-baseline --no-kernel-timing > $O/${TAG}_tl$k.log 2>&1 \
    || { tail -20 $O/${TAG}_tl$k.log; exit 1; }
  for kv in $arm; do unset "${kv%%=*}"; done
  db=$(find $O/${TAG}_tl$k -name '*.db' | head -1)
  python3 tools/timeline.py "$db" --all > $O/${TAG}_timeline$k.txt 2>&1 || true
  echo "arm $k [$arm]: $(head -1 $O/${TAG}_timeline$k.txt)"
done
