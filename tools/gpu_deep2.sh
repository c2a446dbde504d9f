#!/usr/bin/env bash
# Deep-level bconv launches: bench-loop time vs the kernels' own durations (rocprofv3).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export BCONV_ES=4
B=tools/bconv_bench
for S in "f 2 12 12 12 64 128 3 3 2 1" "f 2 14 14 11 64 64 3 3 1 1" "f 2 26 26 12 64 64 3 3 1 1" "db 2 8 8 11 128 128 3 3 1 0"; do
  timeout -k 5 60 $B $S 200 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/deep_prof -- $B f 2 14 14 11 64 64 3 3 1 1 200 > $O/deep_prof.log 2>&1 || { tail -20 $O/deep_prof.log; exit 1; }
f=$(find $O/deep_prof -name '*kernel_stats.csv' | head -1); cut -c1-200 "$f"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/deep_prof2 -- $B f 2 12 12 12 64 128 3 3 2 1 200 > $O/deep_prof2.log 2>&1 || { tail -20 $O/deep_prof2.log; exit 1; }
f=$(find $O/deep_prof2 -name '*kernel_stats.csv' | head -1); cut -c1-200 "$f"
find $O/deep_prof $O/deep_prof2 -name '*.csv' -size +5M -delete
