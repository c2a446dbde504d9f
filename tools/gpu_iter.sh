#!/usr/bin/env bash
# One GPU iteration: parity tests, per-layer profile, short bench.  Usage (via gpurun):
#   bash tools/gpu_iter.sh TAG
set -o pipefail
TAG=${1:-iter}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python tools/layer_profile.py --steps 5 --json gpurun_out/${TAG}_layers.json > gpurun_out/${TAG}_layers.txt 2>&1 || { tail -30 gpurun_out/${TAG}_layers.txt; exit 1; }
head -40 gpurun_out/${TAG}_layers.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
