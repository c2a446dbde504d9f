# RDCNet (config 5) pass: optional GPU tests, then interleaved A/B of env
# settings on bench.py --runet (ms/step per run).
#   bash tools/gpu_runet_ab.sh TAG REPS 'pytest args or -' 'ENV_A' 'ENV_B' ...
set -o pipefail
TAG=$1; REPS=$2; TESTS=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
if [ "$TESTS" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 400 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
  tail -1 $O/${TAG}_tests.log
fi
for r in $(seq 1 "$REPS"); do
  k=0
  for arm in "$@"; do
    k=$((k + 1))
    env $arm timeout -k 10 300 python -u bench.py --runet --steps 6 --warmup 2 --no-cpu-baseline --no-kernel-timing \
      > $O/${TAG}_${k}_${r}.json 2> $O/${TAG}_${k}_${r}.err || { tail -20 $O/${TAG}_${k}_${r}.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/${TAG}_${k}_${r}.json').read().strip().splitlines()[-1]);print('rep $r arm $k [$arm]: %.3f ms/step loss %.5f' % (d['ms_per_step'], d['config']['final_loss']))"
  done
done
