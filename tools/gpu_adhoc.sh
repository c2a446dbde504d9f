set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_modes.py -x -q --timeout 200 --timeout-method thread -k "ncxyz or fresh" > $O/ncx_tests.log 2>&1 || { tail -40 $O/ncx_tests.log; exit 1; }
tail -1 $O/ncx_tests.log
bash tools/gpu_check.sh ncx 1 "2 3" 1 || exit 1
timeout -k 10 300 python -u bench.py --config 3 --input-dtype fp16 --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing > $O/ncx_b3f16.json 2> $O/ncx_b3f16.err || { tail -20 $O/ncx_b3f16.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/ncx_b3f16.json')); print('config 3 fp16 input %.4f ms/step' % d['ms_per_step'])"
