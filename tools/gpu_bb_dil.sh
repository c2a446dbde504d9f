# Phase counts of RDCNet's 5x5x5 bf16 convolution shapes (tools/bconv_bench, CV = 1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export HCU_BCONV_TUNE=0
for force in "" "8,1,4,8" "8,1,2,8" "8,1,1,4" "8,1,4,4"; do
  HCU_BCONV_FORCE=$force timeout -k 5 60 tools/bbench_cv1 f 1 260 260 12 16 16 5 5 5 0 20 2>&1 | grep -v amdgpu.ids | head -3 || true
  HCU_BCONV_FORCE=$force timeout -k 5 60 tools/bbench_cv1 f 1 68 68 7 16 16 5 5 5 0 20 2>&1 | grep -v amdgpu.ids | head -3 || true
done
