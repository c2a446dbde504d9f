set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
timeout -k 10 300 python -u bench.py --runet --steps 3 --warmup 2 --no-cpu-baseline > $O/rl_runet.json 2> $O/rl_runet.err || { tail -20 $O/rl_runet.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/rl_runet.json').read().strip().splitlines()[-1])
print(d['ms_per_step'])
for k in d['kernels']['top']: print(k)
for l in d['layers'][:8]: print(l['layer'], l['measured_us'], {k:v for k,v in l['kernels'].items() if 'wgrad' in k})
PY
