#!/usr/bin/env bash
# tests + bench/layers (gpu_perf.sh) + timeline of both configs
set -o pipefail
TAG=${1:-p}
bash tools/gpu_perf.sh $TAG $2 || exit 1
bash tools/gpu_timeline.sh > gpurun_out/${TAG}_tl.log 2>&1 || { tail -20 gpurun_out/${TAG}_tl.log; exit 1; }
grep -E "step wall|backward from" gpurun_out/tl2_timeline.txt gpurun_out/tl3_timeline.txt
