# Phase counts of config 2's deep-level fp32 convolutions (tools/bconv_bench, CV = 4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export BCONV_ES=4 HCU_BCONV_TUNE=0
B=tools/bbench_cv4
for args in "f 2 28 28 13 32 64 3 3 2 1" "f 2 26 26 12 64 64 3 3 1 1" "f 2 12 12 12 64 128 3 3 2 1" "f 2 10 10 11 128 128 3 3 1 1" "f 2 16 16 12 64 64 3 3 2 1" "db 2 10 10 11 128 64 3 3 2 0" "db 2 8 8 11 128 128 3 3 1 0"; do
  for force in "" "16,1,1,4" "16,1,2,8" "16,1,4,8"; do
    HCU_BCONV_FORCE=$force timeout -k 5 60 $B $args 30 2>&1 | grep -v amdgpu.ids | head -4 || true
  done
done
