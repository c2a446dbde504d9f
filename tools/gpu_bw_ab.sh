cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/bw_ab.log; : > $O
for V in "" "HCU_BWGRAD_SERIAL=1" "HCU_BW_OCC=1" "HCU_BW_OCC=4" "HCU_BW_CKA=16" "HCU_BW_CKA=16 HCU_BW_OCC=4" "HCU_BW_TILE=1"; do
  echo "== $V" >> $O
  env $V HCU_CONV2_LOG=1 timeout -k 10 120 python -u tools/wgrad_bench.py --bf16 --only c3.d0.c2,c3.d1.c2,c3.d1.c1 --reps 10 >> $O 2>&1 || { tail -20 $O; exit 1; }
done
grep -E "==|bwgrad|finalize" $O | grep -v "^bwgrad plan" | head -80
grep "bwgrad plan" $O | sort -u | head -20
