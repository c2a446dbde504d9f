set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
export BCONV_ES=4 HCU_BCONV_TUNE=0
for args in "f 2 12 12 12 64 128 3 3 2 1" "f 2 10 10 11 128 128 3 3 1 1" "db 2 8 8 11 128 128 3 3 1 0"; do
  timeout -k 5 60 tools/bbench_cv4 $args 30 2>&1 | grep -v amdgpu.ids | head -3 || true
done
unset BCONV_ES HCU_BCONV_TUNE
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_modes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/dual_tests.log 2>&1 || { tail -40 $O/dual_tests.log; exit 1; }
tail -1 $O/dual_tests.log
bash tools/gpu_abx.sh dual 2 3 'HCU_X=0' 'HCU_LIB_PATH=hcunet_amd/libhcunet_old.so'
