#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x3b}
mkdir -p $O
timeout -k 10 300 python -u tools/bench_x3.py > $O/bench_x3.jsonl 2> $O/bench_x3.err
cat $O/bench_x3.jsonl
timeout -k 10 400 python -u tools/bench_eval.py --batches 6 --modes fp32,x3 > $O/eval.json 2> $O/eval.err
cat $O/eval.json
