#!/usr/bin/env bash
# Quick GPU iteration (via gpurun): parity tests, short bench, per-layer profile.
#   bash tools/gpu_quick.sh TAG [extra command run first]
set -o pipefail
TAG=${1:-q}
EXTRA=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
mkdir -p $O
if [ -n "$EXTRA" ]; then
  timeout -k 10 120 bash -c "$EXTRA" > $O/${TAG}_extra.log 2>&1 || { tail -30 $O/${TAG}_extra.log; exit 1; }
  cat $O/${TAG}_extra.log | head -90
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
tail -2 $O/${TAG}_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err \
  || { tail -30 $O/${TAG}_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]);print('ms/step',d['ms_per_step'],'value',d['value'],'kernel ms',d['kernels']['kernel_ms_per_step'])"
timeout -k 10 200 python -u tools/layer_profile.py --steps 5 --json $O/${TAG}_layers.json \
  > $O/${TAG}_layers.txt 2>&1 || { tail -30 $O/${TAG}_layers.txt; exit 1; }
head -30 $O/${TAG}_layers.txt
