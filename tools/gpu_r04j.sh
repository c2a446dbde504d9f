#!/usr/bin/env bash
# Channels-last chain boundaries: chain + r_unet GPU tests, the --runet bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_runet.py -m gpu -x -q --timeout 360 --timeout-method thread \
  > $O/r04j_tests.log 2>&1 || { tail -50 $O/r04j_tests.log; exit 1; }
tail -1 $O/r04j_tests.log
timeout -k 10 300 python -u bench.py --runet --steps 5 --warmup 2 --no-cpu-baseline > $O/r04j_runet.json 2> $O/r04j_runet.err \
  || { tail -30 $O/r04j_runet.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/r04j_runet.json').read().strip().splitlines()[-1])
print('runet ms/step', d['ms_per_step'], 'kernel ms', d['kernels']['kernel_ms_per_step'], 'launches', d['kernels']['launches_per_step'])
for r in d['layers'][:14]: print(r['layer'], r['measured_us'], r['launches'], r['tflops'])"
