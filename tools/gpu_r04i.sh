#!/usr/bin/env bash
# RDCNet full-tile oracle test, the --runet bench line with its per-layer
# table, then config-3 A/B of the bf16 weight-gradient grid size.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_runet.py -m gpu -x -v -s --timeout 360 --timeout-method thread \
  -k full_tile > $O/r04i_runet_test.log 2>&1 || { tail -40 $O/r04i_runet_test.log; exit 1; }
grep -E "ok |FAIL|passed|failed" $O/r04i_runet_test.log | tail -20
timeout -k 10 300 python -u bench.py --runet --steps 5 --warmup 2 --no-cpu-baseline > $O/r04i_runet.json 2> $O/r04i_runet.err \
  || { tail -30 $O/r04i_runet.err; exit 1; }
cut -c1-600 $O/r04i_runet.json
bash tools/gpu_abx.sh ab7 3 2 "" "HCU_BW_CUS=224" "HCU_BW_CUS=192" "HCU_BW_CUS=160"
