set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
timeout -k 10 300 python -u bench.py --runet --steps 10 --warmup 3 --no-cpu-baseline > $O/rb_k.json 2> $O/rb_k.err || { tail -20 $O/rb_k.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/rb_k.json').read().strip().splitlines()[-1])
print(d['ms_per_step'])
k=d.get('kernels') or {}
for row in (k.get('top') or [])[:25]: print(row)
PY
