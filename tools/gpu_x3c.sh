#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x3c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_graph_ws_gpu.py tests/test_x3_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u tools/bench_eval.py --batches 6 --modes x3 > $O/eval.json 2> $O/eval.err
cat $O/eval.json
RADHIP_PROBE_NO_SINC=1 timeout -k 10 400 python -u tools/bench_eval.py --batches 6 --modes x3 > $O/eval_nosinc.json 2> $O/eval_nosinc.err
cat $O/eval_nosinc.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RADHIP_PROBE_NO_SINC=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/x3c -o run -- python3 tools/bench_eval.py --batches 4 --warmup 2 --modes x3 > $O/prof.log 2>&1
cp "$(find /tmp/x3c -name '*kernel_trace.csv' | head -1)" $O/kernel_trace.csv
python3 tools/trace_tail.py $O/kernel_trace.csv --marker fe_conv0_kernel --iters 4 --top 30 > $O/steady_nosinc.txt
gzip -f $O/kernel_trace.csv
cat $O/steady_nosinc.txt
