cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runet.py tests/test_gpu_dist.py -v -s -rA --timeout 200 --timeout-method thread > gpurun_out/r03g.log 2>&1
grep -E "PASSED|FAILED|FAIL |Error|train grad .*rel L2 [0-9.e-]+" gpurun_out/r03g.log | grep -v "^ok" | head -40
grep -E "train grad" gpurun_out/r03g.log | sort -t' ' -k6 -g | tail -5
