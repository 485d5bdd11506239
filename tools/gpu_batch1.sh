#!/bin/bash
# CNN on batched hgemm (tests + timing), bf16 window error diagnosis, then the bench line.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-b1}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_featconv_gpu.py tests/test_graph_ws_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/bench_fe.py > $O/bench_fe.jsonl 2> $O/bench_fe.err
cat $O/bench_fe.jsonl
timeout -k 10 300 python -u tools/diag_window_groups.py > $O/diag_window.jsonl 2> $O/diag_window.err
cat $O/diag_window.jsonl
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'mfma', d['step_mfma_frac'])"
