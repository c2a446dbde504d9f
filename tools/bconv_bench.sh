#!/usr/bin/env bash
# Builds tools/bconv_bench (one bf16 conv launch with phase timing) (stand-alone: bconv.hip
# compiled in with HCU_BCONV_PHASES).
set -euo pipefail
cd "$(dirname "$0")/.."
CV=${1:-4}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ihcunet_amd/csrc -DBENCH_CV=$CV \
  tools/bconv_bench.hip hcunet_amd/csrc/timing.cpp -o tools/bconv_bench_cv$CV
echo "built tools/bconv_bench_cv$CV"
