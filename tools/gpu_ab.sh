#!/usr/bin/env bash
# A/B of an environment switch on the bench:  bash tools/gpu_ab.sh TAG "ENV=VAL ..." [configs]
set -o pipefail
TAG=$1; ENVS=$2; CFGS=${3:-"2 3"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
for C in $CFGS; do
  for arm in base test; do
    if [ $arm = test ]; then E="$ENVS"; else E=""; fi
    env $E timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing \
      > $O/${TAG}_${arm}$C.json 2> $O/${TAG}_${arm}$C.err || { tail -20 $O/${TAG}_${arm}$C.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/${TAG}_${arm}$C.json').read().strip().splitlines()[-1]);print('config $C $arm ms/step',round(d['ms_per_step'],4))"
  done
done
