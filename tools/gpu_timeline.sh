#!/usr/bin/env bash
# Step timeline + kernel audit only (the timeline part of gpu_final.sh):
#   bash tools/gpu_timeline.sh TAG [CONFIGS="2 3"]
set -o pipefail
TAG=${1:-tl}
CONFIGS=${2-"2 3"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
for C in $CONFIGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${TAG}_tl$C \
    -- python3 bench.py --config $C --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
    > $O/${TAG}_tl$C.log 2>&1 || { tail -30 $O/${TAG}_tl$C.log; exit 1; }
  db=$(find $O/${TAG}_tl$C -name '*.db' | head -1)
  python3 tools/timeline.py "$db" > $O/${TAG}_timeline_config$C.txt 2>&1 || true
  python3 tools/kernel_audit.py "$db" > $O/${TAG}_kernel_audit_config$C.txt 2>&1 || true
  head -14 $O/${TAG}_timeline_config$C.txt
  grep -i "branch\|adam" $O/${TAG}_timeline_config$C.txt | head -5
  find $O/${TAG}_tl$C -name '*.db' -delete 2>/dev/null
done
echo done
