#!/usr/bin/env bash
# bconv per-block phase probe on deep-level shapes (tools/bconv_bench).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export BCONV_ES=4
B=tools/bconv_bench
for S in "f 2 12 12 12 64 128 3 3 2 1" "f 2 14 14 11 64 64 3 3 1 1" "f 2 26 26 12 64 64 3 3 1 1" "db 2 8 8 11 128 128 3 3 1 0" "f 2 124 124 14 16 16 3 3 1 1"; do
  timeout -k 5 60 $B $S 200 || exit 1
done
