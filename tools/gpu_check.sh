#!/usr/bin/env bash
# Iteration pass (via gpurun): the GPU parity suite, the config-2 (and
# optionally config-3) bench line without the kernel-timing pass, and the
# per-layer HIP-event table.  Every GPU step has its own limit; the script
# stops at the first failure.
#   bash tools/gpu_check.sh TAG [TESTS=1] [CONFIGS="2"] [LAYERS=1]
set -o pipefail
TAG=${1:-chk}
TESTS=${2:-1}
CONFIGS=${3:-2}
LAYERS=${4:-1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
  tail -1 $O/${TAG}_tests.log
fi
for C in $CONFIGS; do
  for R in 1 2; do
    timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing \
      > $O/${TAG}_b${C}_$R.json 2> $O/${TAG}_b${C}_$R.err || { tail -20 $O/${TAG}_b${C}_$R.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('config', sys.argv[2], 'run', sys.argv[3], '%.4f ms/step' % d['ms_per_step'], 'host %.3f' % d['config']['host_enqueue_ms_per_step'])" $O/${TAG}_b${C}_$R.json $C $R
  done
  if [ "$LAYERS" = 1 ]; then
    timeout -k 10 200 python -u tools/layer_profile.py --config $C --steps 5 > $O/${TAG}_layers_config$C.txt 2>&1 || { tail -20 $O/${TAG}_layers_config$C.txt; exit 1; }
    head -30 $O/${TAG}_layers_config$C.txt
  fi
done
