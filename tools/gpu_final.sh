#!/usr/bin/env bash
# Round measurement pass (via gpurun): parity tests, bench lines (config 2, 3,
# tiled inference), rocprofv3 kernel stats of the graphed step per config,
# FETCH/WRITE PMC traffic and SQ counter passes.  Every GPU step has its own
# limit; the script stops at the first failure.   bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
tail -1 $O/${TAG}_tests.log
for C in 2 3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof$C \
    -- python3 bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing \
    > $O/${TAG}_prof$C.log 2>&1 || { tail -30 $O/${TAG}_prof$C.log; exit 1; }
  f=$(find $O/${TAG}_prof$C -name '*kernel_stats.csv' | head -1); cp "$f" $O/${TAG}_kernel_stats_config$C.csv
  echo "rocprof config $C: $(head -3 $O/${TAG}_kernel_stats_config$C.csv | tail -2 | cut -c1-120)"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_fetch$C \
    -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing \
    > $O/${TAG}_fetch$C.log 2>&1 || { tail -20 $O/${TAG}_fetch$C.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_write$C \
    -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing \
    > $O/${TAG}_write$C.log 2>&1 || { tail -20 $O/${TAG}_write$C.log; exit 1; }
  python3 tools/pmc_traffic.py $O/${TAG}_fetch$C $O/${TAG}_write$C --out $O/${TAG}_traffic_config$C.json > /dev/null
  echo "traffic config $C done"
  bash tools/pmc_sq.sh ${TAG}_sq$C $C > $O/${TAG}_sq$C.log 2>&1 || { tail -20 $O/${TAG}_sq$C.log; exit 1; }
  echo "sq counters config $C done"
  find $O/${TAG}_fetch$C $O/${TAG}_write$C $O/${TAG}_prof$C -name '*.csv' -size +20M -delete 2>/dev/null
done
cp $O/${TAG}_kernel_stats_config2.csv profiles/r02_kernel_stats_config2.csv
cp $O/${TAG}_kernel_stats_config3.csv profiles/r02_kernel_stats_config3.csv
cp $O/${TAG}_traffic_config2.json profiles/traffic.json
cp $O/${TAG}_traffic_config3.json profiles/traffic_config3.json
for C in 2 3; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 > $O/${TAG}_bench_config$C.json 2> $O/${TAG}_bench_config$C.err \
    || { tail -30 $O/${TAG}_bench_config$C.err; exit 1; }
  cut -c1-400 $O/${TAG}_bench_config$C.json
done
timeout -k 10 300 python -u bench.py --infer --steps 3 --warmup 1 > $O/${TAG}_bench_infer.json 2> $O/${TAG}_bench_infer.err \
  || { tail -30 $O/${TAG}_bench_infer.err; exit 1; }
cut -c1-300 $O/${TAG}_bench_infer.json
timeout -k 10 200 python -u tools/layer_profile.py --config 2 --steps 5 > $O/${TAG}_layers_config2.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/layer_profile.py --config 3 --steps 5 > $O/${TAG}_layers_config3.txt 2>&1 || exit 1
echo done
