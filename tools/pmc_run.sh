#!/usr/bin/env bash
# SQ counter passes (one rocprofv3 run per pass, counters only) over any python command.
#   bash tools/pmc_run.sh TAG python3 tools/wgrad_bench.py --only d0.c1
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/${TAG}_p$i -- "$@" \
    > $O/${TAG}_p$i.log 2>&1 || { tail -20 $O/${TAG}_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O/${TAG}_p1 $O/${TAG}_p2 --top 30 > $O/${TAG}_summary.txt 2>&1
echo done
