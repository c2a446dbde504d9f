#!/usr/bin/env bash
# Deep-level (d3/d4/u0) convolution shapes of config 2 through tools/bconv_bench:
# launch time and per-phase cycles, tuned tiling vs forced ones and K-split targets.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B=tools/bconv_bench
export BCONV_ES=4
run() { timeout -k 5 60 $B "$@" 200 || { echo "FAILED $*"; exit 1; }; }
for KS in 256 512 1024 2048; do
  export HCU_BCONV_KS_TARGET=$KS
  echo "== KS_TARGET $KS"
  run f 2 12 12 12 64 128 3 3 2 1
  run f 2 10 10 11 128 128 3 3 1 1
  run db 2 10 10 11 128 64 3 3 2 0
  run db 2 8 8 11 128 128 3 3 1 0
  run f 2 28 28 13 32 64 3 3 2 1
  run f 2 26 26 12 64 64 3 3 1 1
  run f 2 16 16 12 64 64 3 3 2 0
  run f 2 14 14 11 64 64 3 3 1 1
done
unset HCU_BCONV_KS_TARGET
for F in 16,1,1,4 16,1,2,4 16,2,1,4 16,2,2,4 16,4,1,4 8,1,1,4 8,2,1,4 4,1,1,4; do
  echo "== force $F"
  HCU_BCONV_FORCE=$F run f 2 12 12 12 64 128 3 3 2 1
  HCU_BCONV_FORCE=$F run f 2 10 10 11 128 128 3 3 1 1
done
echo done
