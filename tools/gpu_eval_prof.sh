#!/bin/bash
# Eval throughput (fp32 / bf16 / fp16 / x3) and a rocprofv3 kernel summary of one precision's scoring pass.
#   bash tools/gpu_eval_prof.sh <tag> <prof mode> [throughput modes, "" to skip]
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06}
MODE=${2:-fp32}
TMODES=${3-fp32,bf16,fp16}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$TMODES" ]; then
  timeout -k 10 400 python -u tools/bench_eval.py --batches 6 --modes $TMODES > $O/eval.json 2> $O/eval.err
  cat $O/eval.json
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 tools/bench_eval.py --batches 4 --warmup 1 --modes $MODE > $O/prof.log 2>&1
cp "$(find /tmp/$TAG -name '*kernel_stats.csv' | head -1)" $O/kernel_stats.csv
python3 tools/stats_top.py $O/kernel_stats.csv 45 > $O/kernel_top.txt
cat $O/kernel_top.txt
