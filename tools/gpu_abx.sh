#!/usr/bin/env bash
# Interleaved A/B of environment settings on ONE box (via gpurun): each arm
# runs bench.py (no CPU baseline, no per-kernel timing pass) REPS times,
# alternating arms, and the ms/step of every run is printed.
#   bash tools/gpu_abx.sh TAG CONFIG REPS 'ENV_A' 'ENV_B' ['ENV_C' ...]
# e.g. bash tools/gpu_abx.sh ab1 2 3 'HCU_WGRAD3=0' 'HCU_WGRAD3=1'
set -o pipefail
TAG=$1; CFG=$2; REPS=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
for r in $(seq 1 "$REPS"); do
  k=0
  for arm in "$@"; do
    k=$((k + 1))
    env $arm timeout -k 10 200 python -u bench.py --config "$CFG" --steps 30 --warmup 5 --no-cpu-baseline \
      --no-kernel-timing > $O/${TAG}_${k}_${r}.json 2> $O/${TAG}_${k}_${r}.err \
      || { tail -20 $O/${TAG}_${k}_${r}.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('$O/${TAG}_${k}_${r}.json').read().strip().splitlines()[-1]);print('rep $r arm $k [$arm]: %.4f ms/step host %.3f' % (d['ms_per_step'], d['config'].get('host_enqueue_ms_per_step') or -1))"
  done
done
