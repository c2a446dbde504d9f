#!/usr/bin/env bash
# Round measurement pass, part b (via gpurun; part a: gpu_final_a.sh): parity tests, bench lines (config 2, 3,
# tiled inference, r_unet), rocprofv3 kernel stats of the step per config
# (tiling from the persistent table: no plan-time timing dispatches), the step
# timeline per stream, FETCH/WRITE PMC traffic and SQ counter passes.  Every
# GPU step has its own limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-r04}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1   # table + cost model on a miss: never time candidates inside a profile
# config 5 (RDCNet, --runet): kernel stats of its step
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_profrunet \
  -- python3 bench.py --runet --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing \
  > $O/${TAG}_profrunet.log 2>&1 || { tail -30 $O/${TAG}_profrunet.log; exit 1; }
f=$(find $O/${TAG}_profrunet -name '*kernel_stats.csv' | head -1); cp "$f" $O/${TAG}_kernel_stats_runet.csv
find $O/${TAG}_profrunet -name '*.csv' -size +20M -delete 2>/dev/null
# the bench lines cite profiles/<TAG>_* (bench.py PROFILE_TAG): install this
# pass's summaries there first (in the box's copy; the results come back via
# gpurun_out/ and are committed from there)
for C in 2 3; do
  # (part a's summaries were installed under profiles/ before this call)
  [ -f $O/${TAG}_kernel_stats_config$C.csv ] && cp $O/${TAG}_kernel_stats_config$C.csv profiles/${TAG}_kernel_stats_config$C.csv
  [ -f $O/${TAG}_kernel_stats_serial_config$C.csv ] && cp $O/${TAG}_kernel_stats_serial_config$C.csv profiles/${TAG}_kernel_stats_serial_config$C.csv
  [ -s $O/${TAG}_traffic_config$C.json ] && cp $O/${TAG}_traffic_config$C.json profiles/${TAG}_traffic_config$C.json
done
cp $O/${TAG}_kernel_stats_runet.csv profiles/${TAG}_kernel_stats_runet.csv
for C in 2 3; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 > $O/${TAG}_bench_config$C.json 2> $O/${TAG}_bench_config$C.err \
    || { tail -30 $O/${TAG}_bench_config$C.err; exit 1; }
  cut -c1-400 $O/${TAG}_bench_config$C.json
done
timeout -k 10 300 python -u bench.py --infer --steps 3 --warmup 1 > $O/${TAG}_bench_infer.json 2> $O/${TAG}_bench_infer.err \
  || { tail -30 $O/${TAG}_bench_infer.err; exit 1; }
cut -c1-300 $O/${TAG}_bench_infer.json
timeout -k 10 300 python -u bench.py --runet --steps 5 --warmup 2 > $O/${TAG}_bench_runet.json 2> $O/${TAG}_bench_runet.err \
  || { tail -30 $O/${TAG}_bench_runet.err; exit 1; }
cut -c1-300 $O/${TAG}_bench_runet.json
timeout -k 10 200 python -u tools/layer_profile.py --config 2 --steps 5 > $O/${TAG}_layers_config2.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/layer_profile.py --config 3 --steps 5 > $O/${TAG}_layers_config3.txt 2>&1 || exit 1
echo done
