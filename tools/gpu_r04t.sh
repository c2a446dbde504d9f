#!/usr/bin/env bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/r04t_tests.log 2>&1 || { tail -40 $O/r04t_tests.log; exit 1; }
tail -1 $O/r04t_tests.log
for C in 2 3; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing \
    > $O/r04t_bench$C.json 2> $O/r04t_bench$C.err || { tail -20 $O/r04t_bench$C.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/r04t_bench$C.json').read().strip().splitlines()[-1]);print('config $C', d['ms_per_step'])"
done
