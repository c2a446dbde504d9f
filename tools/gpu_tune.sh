#!/usr/bin/env bash
# Regenerates the persistent convolution tiling table (hcunet_amd/tuning/
# bconv_gfx950.txt) on an MI355X: each bench config plans with timing on a
# miss and saves the table; later processes load it.  Copies the table to
# gpurun_out/ so it can be committed.      bash tools/gpu_tune.sh [configs...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
mkdir -p $O hcunet_amd/tuning
T=hcunet_amd/tuning/bconv_gfx950.txt
CFGS=${*:-2 3}
for C in $CFGS; do
  HCU_TUNE_SAVE=$T timeout -k 10 300 python -u bench.py --config $C --steps 3 --warmup 1 \
    --no-cpu-baseline --no-kernel-timing > $O/tune_$C.json 2> $O/tune_$C.err || { tail -30 $O/tune_$C.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/tune_$C.json').read().strip().splitlines()[-1]);print('config $C tiling', d['tiling'])"
done
cp $T $O/bconv_gfx950.txt
echo tune done
