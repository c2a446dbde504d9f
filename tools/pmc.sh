#!/usr/bin/env bash
# PMC counters for the training step (separate passes; no tracing domains mixed in).
# Usage (via gpurun): bash tools/pmc.sh TAG "COUNTERS..." [extra rocprofv3 args]
set -o pipefail
TAG=$1; shift
CTRS=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc_$TAG "$@" -- python3 tools/layer_profile.py --steps 2 > gpurun_out/pmc_$TAG.log 2>&1
