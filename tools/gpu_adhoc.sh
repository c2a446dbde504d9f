set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
S=d2.c2,d3.c1,d3.c2,d4.c1,d4.c2,u1.c1
for PF in 1 0; do
HCU_W3_PF=$PF HCU_CONV2_LOG=1 timeout -k 10 120 python -u tools/wgrad_bench.py --only $S > $O/wb_$PF.txt 2>&1 || { tail -20 $O/wb_$PF.txt; exit 1; }
echo "PF=$PF"; grep -v "^$" $O/wb_$PF.txt | grep -v amdgpu.ids
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
for PF in 1 0; do
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  HCU_W3_PF=$PF timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/wsq${PF}_p$i \
    -- python3 tools/wgrad_bench.py --only d2.c2 --reps 5 > $O/wsq${PF}_p$i.log 2>&1 || { tail -20 $O/wsq${PF}_p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O/wsq${PF}_p1 $O/wsq${PF}_p2 --top 5 > $O/wsq${PF}_summary.txt 2>&1
echo "PF=$PF"; cut -c1-400 $O/wsq${PF}_summary.txt
done
