cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runet.py -v --timeout 120 --timeout-method thread > gpurun_out/r03c_runet.log 2>&1
rc=$?
tail -40 gpurun_out/r03c_runet.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread --deselect tests/test_gpu_runet.py > gpurun_out/r03c_tests.log 2>&1
tail -3 gpurun_out/r03c_tests.log
