#!/usr/bin/env bash
# GPU sweep of tools/bconv_bench over the config-3 layer shapes (experiments).
B=tools/bconv_bench
run() { timeout -k 5 30 $B "$@" || { echo "FAILED $*"; exit 1; }; }
run f 4 254 254 15 32 32 3 3 1 1
run db 4 252 252 15 32 32 3 3 1 0
run f 4 256 256 16 8 32 3 3 2 0
run f 4 124 124 14 64 64 3 3 1 1
run f 4 26 26 12 256 256 3 3 1 1
run f 4 10 10 11 512 512 3 3 1 1
for F in ${FORCES:-32,2,4,0 32,2,4,8 32,2,2,8 32,2,2,0 32,1,4,12 32,2,1,4}; do
  echo "force $F"; HCU_BCONV_FORCE=$F run f 4 254 254 15 32 32 3 3 1 1
done
