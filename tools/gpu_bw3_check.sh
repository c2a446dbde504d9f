set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u tools/cmp_libs.py hcunet_amd/libhcunet.so hcunet_amd/libhcunet_old.so --bf16 --wide 2>&1 | tail -2 || exit 1
bash tools/gpu_abx.sh bw3 3 3 'HCU_X=0' 'HCU_LIB_PATH=hcunet_amd/libhcunet_old.so'
