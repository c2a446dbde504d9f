#!/usr/bin/env bash
# GPU sweep of tools/bconv_bench (fp32 kernels) over config-2 layer shapes (experiments).
B=tools/bconv_bench
export BCONV_ES=4
run() { timeout -k 5 30 $B "$@" || { echo "FAILED $*"; exit 1; }; }
run f 2 256 256 16 4 8 3 3 2 0
run f 2 254 254 15 8 8 3 3 1 1
run db 2 252 252 15 8 8 3 3 1 0
run f 2 126 126 15 8 16 3 3 2 1
run f 2 124 124 14 16 16 3 3 1 1
run f 2 59 59 13 32 32 3 3 1 1
run f 2 26 26 12 64 64 3 3 1 1
run f 2 10 10 11 128 128 3 3 1 1
for F in ${FORCES:-4,1,4,8 4,1,2,8 4,1,1,4 8,1,4,8}; do
  echo "force $F"; HCU_BCONV_FORCE=$F run f 2 254 254 15 8 8 3 3 1 1
done
