#!/usr/bin/env bash
# Round-3 iteration pass (via gpurun): parity tests, bench lines for config 2
# and 3, per-layer profiles.  Every GPU step has its own limit; stops at the
# first failure.     bash tools/gpu_r03.sh TAG [TESTS=1] [EXTRA command run first]
set -o pipefail
TAG=${1:-r03}
TESTS=${2:-1}
EXTRA=${3:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
mkdir -p $O
if [ -n "$EXTRA" ]; then
  timeout -k 10 300 bash -c "$EXTRA" > $O/${TAG}_extra.log 2>&1 || { tail -40 $O/${TAG}_extra.log; exit 1; }
  tail -60 $O/${TAG}_extra.log
fi
if [ "$TESTS" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
  tail -2 $O/${TAG}_tests.log
fi
for C in 2 3; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline \
    > $O/${TAG}_bench$C.json 2> $O/${TAG}_bench$C.err || { tail -30 $O/${TAG}_bench$C.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/${TAG}_bench$C.json').read().strip().splitlines()[-1]);print('config $C ms/step',round(d['ms_per_step'],3),'value %.4g'%d['value'],'kernel ms',round(d['kernels']['kernel_ms_per_step'],3), 'host', round(d['config']['host_enqueue_ms_per_step'],3))"
  timeout -k 10 200 python -u tools/layer_profile.py --config $C --steps 5 \
    > $O/${TAG}_layers$C.txt 2>&1 || { tail -30 $O/${TAG}_layers$C.txt; exit 1; }
done
echo done
