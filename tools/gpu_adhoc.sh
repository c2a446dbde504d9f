set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_runet.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bf16_autocast" > $O/t_runet2.log 2>&1 || { tail -30 $O/t_runet2.log; exit 1; }
grep -E "PASS|FAIL|RDCNet bf16" $O/t_runet2.log | tail -5
timeout -k 10 400 python -u bench.py --runet --steps 5 --warmup 2 > $O/rb_full.json 2> $O/rb_full.err || { tail -20 $O/rb_full.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/rb_full.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['cpu_baseline'], d.get('step_roofline'))
PY
for arm in "HCU_X=0" "HCU_SPLIT_FWD_PARAMS=999999999"; do
  env $arm timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing > $O/c3_$arm.json 2>$O/c3.err || { tail -20 $O/c3.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c3_$arm.json').read().strip().splitlines()[-1]);print('$arm', d['ms_per_step'], d['config']['host_enqueue_ms_per_step'])"
done
