# Old-vs-new library builds on one box: bitwise comparison (fp32 and bf16
# training steps, tools/cmp_libs.py), then interleaved bench A/B on configs 2
# and 3.  Build the old library first, e.g. from a git worktree of the base
# commit: OUT=$PWD/hcunet_amd/libhcunet_old.so BDIR=/tmp/oldbuild ./build.sh
#   bash tools/gpu_lib_ab.sh TAG [OLD_LIB]
set -o pipefail
TAG=$1; OLD=${2:-hcunet_amd/libhcunet_old.so}; NEW=hcunet_amd/libhcunet.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 200 python -u tools/cmp_libs.py $OLD $NEW > $O/${TAG}_cmp32.log 2>&1 && tail -1 $O/${TAG}_cmp32.log &&
timeout -k 10 200 python -u tools/cmp_libs.py $OLD $NEW --bf16 > $O/${TAG}_cmp16.log 2>&1 && tail -1 $O/${TAG}_cmp16.log &&
bash tools/gpu_abx.sh ${TAG}c2 2 3 HCU_LIB_PATH=$OLD HCU_LIB_PATH=$NEW &&
bash tools/gpu_abx.sh ${TAG}c3 3 2 HCU_LIB_PATH=$OLD HCU_LIB_PATH=$NEW
