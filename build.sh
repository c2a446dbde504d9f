#!/usr/bin/env bash
# Builds hcunet_amd/libhcunet.so for gfx950 (hipcc cross-compiles without a GPU).
# Usage: ./build.sh [extra hipcc flags]
set -euo pipefail
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
OUT=${OUT:-hcunet_amd/libhcunet.so}   # (OUT / BDIR: a variant build for A/B runs)
BDIR=${BDIR:-build}
SRC="hcunet_amd/csrc/timing.cpp hcunet_amd/csrc/gconv.hip hcunet_amd/csrc/conv2.hip hcunet_amd/csrc/conv8.hip hcunet_amd/csrc/wgrad.hip hcunet_amd/csrc/wgrad8.hip hcunet_amd/csrc/wgrad3.hip hcunet_amd/csrc/pointwise.hip hcunet_amd/csrc/loss_adam.hip hcunet_amd/csrc/loss_ext.hip hcunet_amd/csrc/prep_all.hip hcunet_amd/csrc/bconv.hip hcunet_amd/csrc/bconv_f32.hip hcunet_amd/csrc/bconv_f32_cv1.hip hcunet_amd/csrc/bconv_f32_cv2.hip hcunet_amd/csrc/bconv_f32_cv4.hip hcunet_amd/csrc/bconv_bf16_cv1.hip hcunet_amd/csrc/bconv_bf16_cv2.hip hcunet_amd/csrc/bconv_bf16_cv4.hip hcunet_amd/csrc/bwgrad.hip hcunet_amd/csrc/segment.hip hcunet_amd/csrc/ingest.hip hcunet_amd/csrc/layout.hip hcunet_amd/csrc/pwconv.hip hcunet_amd/csrc/unet.cpp"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude $*"
mkdir -p "$BDIR"
objs=()
pids=()
for s in $SRC; do
  o=$BDIR/$(basename "$s").o
  if [ ! -f "$o" ] || [ "$s" -nt "$o" ] || [ hcunet_amd/csrc/common.h -nt "$o" ] || [ hcunet_amd/csrc/bconv_kernel.h -nt "$o" ] || [ include/hcunet.h -nt "$o" ] || [ build.sh -nt "$o" ]; then
    lang=""
    case "$s" in *.cpp) lang="-x hip";; esac
    $HIPCC $lang $FLAGS -c "$s" -o "$o.tmp" && mv "$o.tmp" "$o" &
    pids+=($!)
  fi
  objs+=("$o")
done
status=0
for p in "${pids[@]:-}"; do
  [ -z "$p" ] && continue
  wait "$p" || status=1
done
if [ $status -ne 0 ]; then echo "build failed" >&2; exit 1; fi
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$OUT.tmp" "${objs[@]}"
mv "$OUT.tmp" "$OUT"
echo "built $OUT"
