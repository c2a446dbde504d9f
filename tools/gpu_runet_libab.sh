# RDCNet bench A/B of two library builds (HCU_LIB_PATH), interleaved, plus
# each arm's plan log (HCU_CONV2_LOG) and wall time of the whole process.
#   bash tools/gpu_runet_libab.sh TAG REPS LIB_A LIB_B
set -o pipefail
TAG=$1; REPS=$2; A=$3; B=$4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
for r in $(seq 1 "$REPS"); do
  k=0
  for L in "$A" "$B"; do
    k=$((k + 1))
    t0=$(date +%s.%N)
    HCU_LIB_PATH=$L HCU_CONV2_LOG=1 timeout -k 10 300 python -u bench.py --runet --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing \
      > $O/${TAG}_${k}_${r}.json 2> $O/${TAG}_${k}_${r}.err || { tail -20 $O/${TAG}_${k}_${r}.err; exit 1; }
    t1=$(date +%s.%N)
    python3 -c "import json;d=json.loads(open('$O/${TAG}_${k}_${r}.json').read().strip().splitlines()[-1]);print('rep $r arm $k [$L]: %.3f ms/step loss %r process %.1f s' % (d['ms_per_step'], d['config']['final_loss'], $t1 - $t0))"
  done
done
