set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
for E in "X=0" "HCU_BCONV_TUNE_TOP=12" "HCU_BCONV_KS_TARGET=512" "HCU_BCONV_KS_TARGET=128" "HCU_BCONV_KS_TARGET=1024"; do
  for C in 2 3; do
    env $E timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing > $O/sw.json 2>$O/sw.err || { tail -5 $O/sw.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/sw.json').read().strip().splitlines()[-1]);print('$E config $C', round(d['ms_per_step'],4))"
  done
done
