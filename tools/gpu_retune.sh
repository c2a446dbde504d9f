#!/usr/bin/env bash
# Re-tunes the bench configs' convolution tilings from scratch with the model's
# best TOP candidates timed (default 12) into a scratch table, then benches the
# shipped table against it (interleaved).   bash tools/gpu_retune.sh TAG [TOP]
set -o pipefail
TAG=${1:-rt}; TOP=${2:-12}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
T=$O/${TAG}_table.txt
rm -f $T
for C in 2 3; do
  HCU_TUNE_FILE=$T HCU_BCONV_TUNE=2 HCU_BCONV_TUNE_TOP=$TOP HCU_TUNE_SAVE=$T timeout -k 10 400 python -u bench.py \
    --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing > $O/${TAG}_tune$C.json 2> $O/${TAG}_tune$C.err \
    || { tail -20 $O/${TAG}_tune$C.err; exit 1; }
done
for C in 2 3; do
  for r in 1 2; do
    for arm in shipped new; do
      if [ $arm = new ]; then E="HCU_TUNE_FILE=$T HCU_BCONV_TUNE=1"; else E="HCU_BCONV_TUNE=1"; fi
      env $E timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing \
        > $O/${TAG}_b.json 2> $O/${TAG}_b.err || { tail -20 $O/${TAG}_b.err; exit 1; }
      python3 -c "import json;d=json.loads(open('$O/${TAG}_b.json').read().strip().splitlines()[-1]);print('config $C $arm ms/step',round(d['ms_per_step'],4),'host',round(d['config']['host_enqueue_ms_per_step'],3))"
    done
  done
done
echo done
