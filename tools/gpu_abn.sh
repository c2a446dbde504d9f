#!/usr/bin/env bash
# Interleaved A/B of several environment settings on the bench (noise control:
# base, arm1, arm2, ..., repeated R times).   bash tools/gpu_abn.sh TAG R CONFIGS "ENV1" "ENV2" ...
set -o pipefail
TAG=$1; R=$2; CFGS=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
for C in $CFGS; do
  for r in $(seq 1 $R); do
    i=0
    for E in "X_BASE=1" "$@"; do
      env $E timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing \
        > $O/${TAG}_${C}_${i}.json 2> $O/${TAG}_${C}_${i}.err || { tail -20 $O/${TAG}_${C}_${i}.err; exit 1; }
      python3 -c "import json;d=json.loads(open('$O/${TAG}_${C}_${i}.json').read().strip().splitlines()[-1]);print('config $C run $r [$E] ms/step',round(d['ms_per_step'],4),'host',round(d['config']['host_enqueue_ms_per_step'],3))"
      i=$((i+1))
    done
  done
done
echo done
