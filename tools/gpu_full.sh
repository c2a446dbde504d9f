#!/usr/bin/env bash
# Round-3 pass (via gpurun): full -m gpu suite, bench lines for configs 2, 3
# and 5 (r_unet), per-layer profiles.   bash tools/gpu_full.sh TAG [TESTS=1]
set -o pipefail
TAG=${1:-r03}
TESTS=${2:-1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
mkdir -p $O
if [ "$TESTS" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1
  rc=$?
  grep -E "FAILED|passed|failed" $O/${TAG}_tests.log | tail -8
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
for C in 2 3; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline \
    > $O/${TAG}_bench$C.json 2> $O/${TAG}_bench$C.err || { tail -30 $O/${TAG}_bench$C.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/${TAG}_bench$C.json').read().strip().splitlines()[-1]);print('config $C ms/step',round(d['ms_per_step'],3),'value %.4g'%d['value'],'kernel ms',round(d['kernels']['kernel_ms_per_step'],3), 'host', round(d['config']['host_enqueue_ms_per_step'],3), 'tiling', d['tiling'])"
done
timeout -k 10 300 python -u bench.py --runet --steps 5 --warmup 2 --no-cpu-baseline > $O/${TAG}_bench5.json 2> $O/${TAG}_bench5.err \
  || { tail -30 $O/${TAG}_bench5.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/${TAG}_bench5.json').read().strip().splitlines()[-1]);print('config 5 ms/step',round(d['ms_per_step'],3),'value %.4g'%d['value']);[print(r) for r in d['kernels']['top'][:6]]"
echo done
