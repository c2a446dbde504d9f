#!/usr/bin/env bash
# end-of-session check of the committed tree: GPU suite, smoke(), one bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/end_tests.log 2>&1 \
  || { tail -40 $O/end_tests.log; exit 1; }
tail -1 $O/end_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/end_smoke.log 2>&1 || { tail -20 $O/end_smoke.log; exit 1; }
tail -1 $O/end_smoke.log
timeout -k 10 300 python -u bench.py > $O/end_bench.json 2> $O/end_bench.err || { tail -20 $O/end_bench.err; exit 1; }
cut -c1-300 $O/end_bench.json
