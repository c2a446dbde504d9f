cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_runet.py -v -rA --timeout 120 --timeout-method thread > gpurun_out/r03d_runet.log 2>&1
grep -E "PASSED|FAILED|ok   |FAIL |Error|assert" gpurun_out/r03d_runet.log | head -150
