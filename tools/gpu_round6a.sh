set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r6a_tests.log 2>&1 || { tail -40 $O/r6a_tests.log; exit 1; }
tail -1 $O/r6a_tests.log
for C in 2 3; do
timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing > $O/r6a_b$C.json 2> $O/r6a_b$C.err || { tail -20 $O/r6a_b$C.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/r6a_b$C.json').read().strip().splitlines()[-1]);print('config $C', d['ms_per_step'], d['config']['host_enqueue_ms_per_step'], d['config']['host_enqueue_idle_ms'])"
done
timeout -k 10 300 python -u bench.py --runet --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $O/r6a_brun.json 2> $O/r6a_brun.err || { tail -20 $O/r6a_brun.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/r6a_brun.json').read().strip().splitlines()[-1]);print('runet', d['ms_per_step'])"
