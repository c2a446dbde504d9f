set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
for C in 2 3; do
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/tl$C -o run -- python3 bench.py --config $C --steps 6 --warmup 3 --no-cpu-baseline --no-kernel-timing > $O/tl${C}_bench.log 2>&1 || { tail -20 $O/tl${C}_bench.log; exit 1; }
python3 tools/timeline.py "$O/tl$C/*/*.db" $O/tl$C/*.db > $O/tl${C}_timeline.txt 2>&1 ; head -40 $O/tl${C}_timeline.txt
find $O/tl$C -name '*.db' -delete
done
