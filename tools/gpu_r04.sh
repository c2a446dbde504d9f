#!/usr/bin/env bash
# Round-4 iteration pass (via gpurun): optional tests, bench lines for
# config 2 / 3, per-layer tables.  Every GPU step has its own limit.
#   bash tools/gpu_r04.sh TAG [TESTS=0] [LAYERS=1]
set -o pipefail
TAG=${1:-r04}
TESTS=${2:-0}
LAYERS=${3:-1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
  tail -1 $O/${TAG}_tests.log
fi
for C in 2 3; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline \
    > $O/${TAG}_bench_config$C.json 2> $O/${TAG}_bench_config$C.err \
    || { tail -30 $O/${TAG}_bench_config$C.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/${TAG}_bench_config$C.json').read().strip().splitlines()[-1]);print('config $C ms/step',d['ms_per_step'],'value',d['value'],'launches',d['config'].get('launches_per_step'),'host',d['config'].get('host_enqueue_ms_per_step'))"
done
if [ "$LAYERS" = 1 ]; then
  for C in 2 3; do
    timeout -k 10 200 python -u tools/layer_profile.py --config $C --steps 5 > $O/${TAG}_layers_config$C.txt 2>&1 || exit 1
    head -3 $O/${TAG}_layers_config$C.txt
  done
fi
echo done
