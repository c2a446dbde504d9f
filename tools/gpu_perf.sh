#!/usr/bin/env bash
# Parity tests + bench (configs 2 and 3) + per-layer profiles:  bash tools/gpu_perf.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-p}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
if [ -z "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1 || { tail -60 $O/${TAG}_tests.log; exit 1; }
  tail -2 $O/${TAG}_tests.log
fi
for C in 2 3; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline > $O/${TAG}_b$C.json 2> $O/${TAG}_b$C.err \
    || { tail -30 $O/${TAG}_b$C.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/${TAG}_b$C.json').read().strip().splitlines()[-1]);print('config $C ms/step',round(d['ms_per_step'],4),'value',round(d['value']/1e6,1),'Mvox/s')"
  timeout -k 10 200 python -u tools/layer_profile.py --config $C --steps 5 --json $O/${TAG}_l$C.json \
    > $O/${TAG}_l$C.txt 2>&1 || { tail -30 $O/${TAG}_l$C.txt; exit 1; }
done
grep -E "pool|apply|to_cl|prep|total|phase" $O/${TAG}_l2.txt | head -20
grep -E "pool|apply|to_cl|prep|total|phase" $O/${TAG}_l3.txt | head -20
