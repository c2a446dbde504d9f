#!/usr/bin/env bash
# Per-phase cycle counts of single bconv launches (tools/bconv_bench_cv*,
# built by tools/bconv_bench.sh CV) for representative layers of config 2
# (fp32) and config 3 (bf16).  Every run has its own limit.
#   bash tools/gpu_bb.sh TAG
set -o pipefail
TAG=${1:-bb}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
run() {   # CV ES args...
  local cv=$1 es=$2; shift 2
  BCONV_ES=$es timeout -k 10 60 tools/bconv_bench_cv$cv "$@" 200 >> $O/${TAG}.txt 2>&1 || { tail -5 $O/${TAG}.txt; exit 1; }
}
: > $O/${TAG}.txt
# config 3 (bf16)
run 4 2 f 4 254 254 15 32 32 3 3 1 1     # d0.c2 fwd
run 4 2 f 4 124 124 14 64 64 3 3 1 1     # d1.c2 fwd
run 4 2 db 4 252 252 15 32 32 3 3 1 1    # d0.c2 dgrad (+ BN backward)
# config 2 (fp32)
run 2 4 f 2 126 126 15 8 16 3 3 2 0      # d1.c1 fwd (pooled input, no act)
run 4 4 f 2 124 124 14 16 16 3 3 1 1     # d1.c2 fwd
run 4 4 f 2 59 59 13 32 32 3 3 1 1       # d2.c2 fwd
run 4 4 f 2 28 28 13 32 64 3 3 2 0       # d3.c1 fwd
run 4 4 f 2 12 12 12 64 128 3 3 2 0      # d4.c1 fwd

# variants of config 3 d0.c2 fwd: direct staging (no register prefetch), fewer subtiles
HCU_BCONV_FORCE=32,2,4,0 run 4 2 f 4 254 254 15 32 32 3 3 1 1
HCU_BCONV_FORCE=32,2,2 run 4 2 f 4 254 254 15 32 32 3 3 1 1
HCU_BCONV_FORCE=32,1,4 run 4 2 f 4 254 254 15 32 32 3 3 1 1
tail -12 $O/${TAG}.txt
