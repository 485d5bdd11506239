#!/bin/bash
# x3 scoring path: kernel tests, the full-model test, eval throughput of every precision.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_x3_gpu.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed|\[x3" $O/pytest.log | tail -30
timeout -k 10 400 python -u tools/bench_eval.py --batches 6 > $O/eval.json 2> $O/eval.err
cat $O/eval.json
