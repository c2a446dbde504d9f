# Times the top bconv tilings of RDCNet's convolutions (plan-time timing,
# HCU_BCONV_TUNE=2) into a copy of the committed table, then an interleaved
# A/B of that table against the committed one (cost-model choice on a miss).
#   bash tools/gpu_runet_retune.sh REPS [TOP]
set -o pipefail
REPS=${1:-2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
NEW=$PWD/$O/tune_runet.txt
cp hcunet_amd/tuning/bconv_gfx950.txt $NEW
HCU_TUNE_FILE=$NEW HCU_BCONV_TUNE=2 HCU_BCONV_TUNE_TOP=${2:-6} HCU_TUNE_SAVE=$NEW HCU_CONV2_LOG=1 timeout -k 10 400 \
  python -u bench.py --runet --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing \
  > $O/retune_runet.json 2> $O/retune_runet.err || { tail -30 $O/retune_runet.err; exit 1; }
cp $NEW $O/tune_runet_saved.txt
bash tools/gpu_runet_ab.sh rrt $REPS - "" "HCU_TUNE_FILE=$NEW"
