# Host-cost pass (via gpurun): per-phase host enqueue of a training step and
# the native forward/backward's steady-state launch / HIP-call costs
# (HCU_HOST_PROF=1), optional GPU tests first, then the config-2/3 bench lines.
#   bash tools/gpu_hostcost.sh TAG ['pytest args']
set -o pipefail
TAG=${1:-hc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest $2 -m gpu -x -q --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1 || { tail -40 $O/${TAG}_tests.log; exit 1; }
  tail -1 $O/${TAG}_tests.log
fi
for C in 2 3; do
HCU_HOST_PROF=1 timeout -k 10 120 python -u tools/host_split.py --config $C > $O/${TAG}_host_split_$C.txt 2>&1 || { tail $O/${TAG}_host_split_$C.txt; exit 1; }
grep -v amdgpu.ids $O/${TAG}_host_split_$C.txt
done
for C in 2 3; do
timeout -k 10 300 python -u bench.py --config $C --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > $O/${TAG}_b$C.json 2> $O/${TAG}_b$C.err || { tail -20 $O/${TAG}_b$C.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/${TAG}_b$C.json').read().strip().splitlines()[-1]);print('config $C', d['ms_per_step'], d['config']['host_enqueue_ms_per_step'], d['config']['host_enqueue_idle_ms'])"
done
