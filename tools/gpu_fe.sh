#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-fe}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_featconv_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/bench_fe.py > $O/bench_fe.jsonl 2> $O/bench_fe.err
cat $O/bench_fe.jsonl
