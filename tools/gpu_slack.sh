set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export HCU_BCONV_TUNE=1
timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing > $O/b2.json 2> $O/b2.err || { tail -20 $O/b2.err; exit 1; }
cut -c1-300 $O/b2.json
timeout -k 10 300 python -u tools/host_slack.py --where end > $O/slack_end.txt 2>&1 || { tail -20 $O/slack_end.txt; exit 1; }
cat $O/slack_end.txt
timeout -k 10 300 python -u tools/host_slack.py --where mid > $O/slack_mid.txt 2>&1 || { tail -20 $O/slack_mid.txt; exit 1; }
cat $O/slack_mid.txt
