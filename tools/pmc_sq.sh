#!/usr/bin/env bash
# SQ counter passes over a short bench run (one rocprofv3 run per pass, counters only).
#   bash tools/pmc_sq.sh TAG [CONFIG|runet]
set -o pipefail
TAG=${1:-sq}
CFG=${2:-2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/${TAG}_counters.txt 2>&1 || true
grep -oE '\bSQ_[A-Z0-9_]+' $O/${TAG}_counters.txt | sort -u > $O/${TAG}_sq_names.txt || true
wc -l $O/${TAG}_sq_names.txt
if [ "$CFG" = runet ]; then BARGS="--runet --steps 1 --warmup 1"; else BARGS="--config $CFG --steps 2 --warmup 1"; fi
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  ok=1
  for c in $P; do grep -qx "$c" $O/${TAG}_sq_names.txt || { echo "missing counter $c"; ok=0; }; done
  [ $ok = 1 ] || continue
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/${TAG}_p$i \
    -- python3 bench.py $BARGS --no-cpu-baseline --no-kernel-timing --idle-steps 0 \
    > $O/${TAG}_p$i.log 2>&1 || { tail -20 $O/${TAG}_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O/${TAG}_p1 $O/${TAG}_p2 --top 30 > $O/${TAG}_summary.txt 2>&1
cat $O/${TAG}_summary.txt | cut -c1-250
find $O/${TAG}_p1 $O/${TAG}_p2 -name '*.csv' -size +20M -delete 2>/dev/null
echo done
