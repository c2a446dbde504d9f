set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
for arm in HCU_X=0 HCU_C8_NPF16=1; do
  echo "== $arm"
  env $arm timeout -k 10 120 python -u tools/conv_bench.py --reps 20 --only d1.c1,d0.c2 2>&1 | grep -v amdgpu.ids
done
bash tools/gpu_abx.sh ab7 2 3 HCU_X=0 HCU_C8_NPF16=1
