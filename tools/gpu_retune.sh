#!/usr/bin/env bash
# Re-times every bconv tiling of configs 2 and 3 into a fresh table (the
# kernels changed since the committed table was measured), then an
# interleaved A/B of the fresh table against the committed one.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
NEW=$PWD/$O/tune_new.txt
: > $NEW
for C in 2 3; do
  HCU_TUNE_FILE=$NEW HCU_BCONV_TUNE=2 HCU_BCONV_TUNE_TOP=${TOP:-6} HCU_TUNE_SAVE=$NEW timeout -k 10 400 python -u bench.py --config $C --steps 3 --warmup 1 \
    --no-cpu-baseline --no-kernel-timing > $O/retune_$C.json 2> $O/retune_$C.err || { tail -30 $O/retune_$C.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/retune_$C.json').read().strip().splitlines()[-1]);print('config $C tiling', d['tiling'])"
done
cp $NEW $O/tune_new_saved.txt
bash tools/gpu_abx.sh ab24 2 3 "" "HCU_TUNE_FILE=$NEW" || exit 1
bash tools/gpu_abx.sh ab25 3 2 "" "HCU_TUNE_FILE=$NEW"
