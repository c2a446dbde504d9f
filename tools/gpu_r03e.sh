cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_runet.py tests/test_gpu_chain.py "tests/test_gpu_bf16.py::test_bf16_config3_full_size" -v -s -rA --timeout 300 --timeout-method thread > gpurun_out/r03e_new.log 2>&1
grep -E "PASSED|FAILED|FAIL |Error|bf16 vs" gpurun_out/r03e_new.log | head -60
timeout -k 10 300 python -u bench.py --runet --steps 5 --warmup 2 > gpurun_out/r03e_bench5.json 2> gpurun_out/r03e_bench5.err || { tail -30 gpurun_out/r03e_bench5.err; exit 1; }
cut -c1-1500 gpurun_out/r03e_bench5.json
