#!/usr/bin/env bash
# Full GPU measurement pass (run via gpurun from the repo root):
#   bash tools/gpu_round.sh TAG [skip-tests]
# 1. parity tests (-m gpu), 2. bench.py JSON line, 3. per-layer kernel profile,
# 4. rocprofv3 --kernel-trace --stats of the bench, 5. FETCH_SIZE / WRITE_SIZE
# PMC passes (separate runs, no tracing domains) -> per-kernel HBM traffic.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-r01}
SKIP_TESTS=${2:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
  tail -3 $O/${TAG}_tests.log
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err \
  || { tail -30 $O/${TAG}_bench.err; exit 1; }
cut -c1-700 $O/${TAG}_bench.json
timeout -k 10 200 python -u tools/layer_profile.py --steps 5 --json $O/${TAG}_layers.json \
  > $O/${TAG}_layers.txt 2>&1 || { tail -30 $O/${TAG}_layers.txt; exit 1; }
head -45 $O/${TAG}_layers.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof \
  -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing \
  > $O/${TAG}_prof.log 2>&1 || { tail -30 $O/${TAG}_prof.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_pmc_fetch \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing \
  > $O/${TAG}_pmc_fetch.log 2>&1 || { tail -20 $O/${TAG}_pmc_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_pmc_write \
  -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing \
  > $O/${TAG}_pmc_write.log 2>&1 || { tail -20 $O/${TAG}_pmc_write.log; exit 1; }
python3 tools/pmc_traffic.py $O/${TAG}_pmc_fetch $O/${TAG}_pmc_write --out $O/${TAG}_traffic.json | head -20
# drop the bulky per-dispatch PMC CSVs, keep the summaries
find $O/${TAG}_pmc_fetch $O/${TAG}_pmc_write -name '*.csv' -size +20M -delete 2>/dev/null
echo done
