# RDCNet check pass: the runet GPU tests that cover the dilated convolutions,
# the all-taps weight-gradient phase counters (measurement build), the
# per-layer kernel table, then an optional interleaved A/B against a variant.
#   bash tools/gpu_runet_check.sh [VARIANT_LIB]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out
export HCU_BCONV_TUNE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_runet.py -m gpu -x -q --timeout 400 --timeout-method thread -k "all_taps or rdcnet_train or bf16_autocast" > $O/at2_tests.log 2>&1 || { tail -40 $O/at2_tests.log; exit 1; }
tail -1 $O/at2_tests.log
if [ -f hcunet_amd/libhcunet_ph.so ]; then
  HCU_LIB_PATH=hcunet_amd/libhcunet_ph.so timeout -k 10 200 python -u tools/bw_phases.py 2>&1 | grep step || exit 1
fi
bash tools/gpu_runet_layers.sh || exit 1
if [ -n "$1" ]; then bash tools/gpu_runet_ab.sh vb 2 - 'HCU_X=0' "HCU_LIB_PATH=$1"; fi
