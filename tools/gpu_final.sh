#!/usr/bin/env bash
# Round measurement pass (via gpurun): parity tests, bench lines (config 2, 3,
# tiled inference, r_unet), rocprofv3 kernel stats of the step per config
# (tiling from the persistent table: no plan-time timing dispatches), the step
# timeline per stream, FETCH/WRITE PMC traffic and SQ counter passes.  Every
# GPU step has its own limit; the script stops at the first failure.
#   bash tools/gpu_final.sh TAG [TESTS=1] [CONFIGS="2 3"] [PARTS="runet install bench layers"]
# (gpurun's 20-minute limit: run it as several calls, e.g. TESTS + config 2,
# then config 3, then the runet / install / bench parts)
set -o pipefail
TAG=${1:-r05}
TESTS=${2:-1}
CONFIGS=${3-"2 3"}
PARTS=${4-"runet install bench layers"}
has() { case " $PARTS " in *" $1 "*) return 0;; *) return 1;; esac; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1   # table + cost model on a miss: never time candidates inside a profile
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
  tail -1 $O/${TAG}_tests.log
fi
for C in $CONFIGS; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof$C \
    -- python3 bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
    > $O/${TAG}_prof$C.log 2>&1 || { tail -30 $O/${TAG}_prof$C.log; exit 1; }
  f=$(find $O/${TAG}_prof$C -name '*kernel_stats.csv' | head -1); cp "$f" $O/${TAG}_kernel_stats_config$C.csv
  echo "rocprof config $C: $(head -3 $O/${TAG}_kernel_stats_config$C.csv | tail -2 | cut -c1-120)"
  # the same bench with the backward on one stream: kernel durations under the
  # conditions of bench.py's serialized HIP-event timing pass
  HCU_SIDE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_profs$C \
    -- python3 bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
    > $O/${TAG}_profs$C.log 2>&1 || { tail -30 $O/${TAG}_profs$C.log; exit 1; }
  f=$(find $O/${TAG}_profs$C -name '*kernel_stats.csv' | head -1); cp "$f" $O/${TAG}_kernel_stats_serial_config$C.csv
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${TAG}_tl$C \
    -- python3 bench.py --config $C --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
    > $O/${TAG}_tl$C.log 2>&1 || { tail -30 $O/${TAG}_tl$C.log; exit 1; }
  db=$(find $O/${TAG}_tl$C -name '*.db' | head -1)
  python3 tools/timeline.py "$db" > $O/${TAG}_timeline_config$C.txt 2>&1 || true
  python3 tools/kernel_audit.py "$db" > $O/${TAG}_kernel_audit_config$C.txt 2>&1 || true
  head -12 $O/${TAG}_timeline_config$C.txt
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_fetch$C \
    -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
    > $O/${TAG}_fetch$C.log 2>&1 || { tail -20 $O/${TAG}_fetch$C.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_write$C \
    -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
    > $O/${TAG}_write$C.log 2>&1 || { tail -20 $O/${TAG}_write$C.log; exit 1; }
  CB=$([ $C = 2 ] && echo 1.342e9 || echo 5.29e9)
  python3 tools/pmc_traffic.py $O/${TAG}_fetch$C $O/${TAG}_write$C --steps 4 --compulsory $CB \
    --out $O/${TAG}_traffic_config$C.json > $O/${TAG}_traffic_config$C.txt 2>&1 || true
  tail -4 $O/${TAG}_traffic_config$C.txt
  bash tools/pmc_sq.sh ${TAG}_sq$C $C > $O/${TAG}_sq$C.log 2>&1 || { tail -20 $O/${TAG}_sq$C.log; exit 1; }
  cp $O/${TAG}_sq${C}_summary.txt $O/${TAG}_sq_counters_config$C.txt
  echo "sq counters config $C done"
  find $O/${TAG}_fetch$C $O/${TAG}_write$C $O/${TAG}_prof$C $O/${TAG}_profs$C $O/${TAG}_tl$C -name '*.csv' -size +20M -delete 2>/dev/null
  find $O/${TAG}_tl$C -name '*.db' -delete 2>/dev/null
done
if has runet; then
# config 5 (RDCNet, --runet): kernel stats of its step
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_profrunet \
  -- python3 bench.py --runet --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
  > $O/${TAG}_profrunet.log 2>&1 || { tail -30 $O/${TAG}_profrunet.log; exit 1; }
f=$(find $O/${TAG}_profrunet -name '*kernel_stats.csv' | head -1); cp "$f" $O/${TAG}_kernel_stats_runet.csv
find $O/${TAG}_profrunet -name '*.csv' -size +20M -delete 2>/dev/null
# its HBM traffic (FETCH_SIZE / WRITE_SIZE, one pass each; 3 steps profiled)
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_fetchrunet \
  -- python3 bench.py --runet --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
  > $O/${TAG}_fetchrunet.log 2>&1 || { tail -20 $O/${TAG}_fetchrunet.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_writerunet \
  -- python3 bench.py --runet --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
  > $O/${TAG}_writerunet.log 2>&1 || { tail -20 $O/${TAG}_writerunet.log; exit 1; }
python3 tools/pmc_traffic.py $O/${TAG}_fetchrunet $O/${TAG}_writerunet --steps 3 \
  --out $O/${TAG}_traffic_runet.json > $O/${TAG}_traffic_runet.txt 2>&1 || true
tail -2 $O/${TAG}_traffic_runet.txt
find $O/${TAG}_fetchrunet $O/${TAG}_writerunet -name '*.csv' -size +20M -delete 2>/dev/null
fi
# the bench lines cite profiles/<TAG>_* (bench.py PROFILE_TAG): install this
# pass's summaries there first (in the box's copy; the results come back via
# gpurun_out/ and are committed from there; a later call of this script finds
# them in profiles/ once committed)
if has install; then
for C in 2 3; do
  [ -s $O/${TAG}_kernel_stats_config$C.csv ] && cp $O/${TAG}_kernel_stats_config$C.csv profiles/${TAG}_kernel_stats_config$C.csv
  [ -s $O/${TAG}_kernel_stats_serial_config$C.csv ] && cp $O/${TAG}_kernel_stats_serial_config$C.csv profiles/${TAG}_kernel_stats_serial_config$C.csv
  [ -s $O/${TAG}_traffic_config$C.json ] && cp $O/${TAG}_traffic_config$C.json profiles/${TAG}_traffic_config$C.json
done
[ -s $O/${TAG}_kernel_stats_runet.csv ] && cp $O/${TAG}_kernel_stats_runet.csv profiles/${TAG}_kernel_stats_runet.csv
[ -s $O/${TAG}_traffic_runet.json ] && cp $O/${TAG}_traffic_runet.json profiles/${TAG}_traffic_runet.json
fi
if has bench; then
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
fi
if has layers; then
timeout -k 10 200 python -u tools/layer_profile.py --config 2 --steps 5 > $O/${TAG}_layers_config2.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/layer_profile.py --config 3 --steps 5 > $O/${TAG}_layers_config3.txt 2>&1 || exit 1
fi
echo done
