#!/bin/bash
# Kernel trace of the x3 (or another precision's) scoring pass, summarised over the last batches.
#   bash tools/gpu_eval_trace.sh <tag> <mode> <marker>
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06}; MODE=${2:-x3}; MARK=${3:-fe_conv0_kernel}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/$TAG -o run -- python3 tools/bench_eval.py --batches 4 --warmup 2 --modes $MODE > $O/prof.log 2>&1
cp "$(find /tmp/$TAG -name '*kernel_trace.csv' | head -1)" $O/kernel_trace.csv
python3 tools/trace_tail.py $O/kernel_trace.csv --marker $MARK --iters 4 --top 45 > $O/steady.txt
gzip -f $O/kernel_trace.csv
cat $O/steady.txt
