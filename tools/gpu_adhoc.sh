set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
timeout -k 10 300 python -u bench.py --runet --steps 5 --warmup 2 --no-cpu-baseline > $O/rb_fix.json 2> $O/rb_fix.err || { tail -20 $O/rb_fix.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/rb_fix.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['kernels']['kernel_ms_per_step'], d['kernels']['launches_per_step'])
for r in d['kernels']['top']: print(r)
PY
