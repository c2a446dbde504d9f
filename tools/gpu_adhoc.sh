set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_unet.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_ops.log 2>&1 || { tail -30 $O/t_ops.log; exit 1; }
tail -2 $O/t_ops.log
for v in "" _e7; do
  echo "== lib$v"
  HCU_LIB_PATH=$PWD/hcunet_amd/libhcunet$v.so timeout -k 10 120 python -u tools/conv_bench.py --reps 20 --only d0.c2,d1.c1,d0.c1 > $O/cb$v.txt 2>&1 || { tail -20 $O/cb$v.txt; exit 1; }
  grep -v amdgpu.ids $O/cb$v.txt
done
