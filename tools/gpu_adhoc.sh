set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_runet.py tests/test_gpu_modes.py -x -v -s --timeout 300 --timeout-method thread -k "residual or split_forward or rdcnet_bf16" > $O/adv_tests.log 2>&1 || { tail -60 $O/adv_tests.log; exit 1; }
grep -E "PASS|FAIL|relative L2|passed|failed" $O/adv_tests.log | tail -20
bash tools/gpu_check.sh up 1 "2 3" 1
