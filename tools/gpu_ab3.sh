#!/usr/bin/env bash
# config-2 bench, N repeats of several environments interleaved:  bash tools/gpu_ab3.sh N "ENV1" "ENV2" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
N=$1; shift
for i in $(seq $N); do
  for E in "$@"; do
    env $E timeout -k 10 200 python -u bench.py --config 2 --steps 30 --warmup 3 --no-cpu-baseline --no-kernel-timing \
      > $O/ab3.json 2> $O/ab3.err || { tail -20 $O/ab3.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/ab3.json').read().strip().splitlines()[-1]);print('$E', round(d['ms_per_step'],4), 'host', round(d['config']['host_enqueue_ms_per_step'],3))"
  done
done
