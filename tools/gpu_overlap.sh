#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ov}
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/ov -o run -- python3 bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_eager.json 2> $O/prof.err
cp "$(find /tmp/ov -name '*kernel_trace.csv' | head -1)" $O/kernel_trace_eager.csv
python3 tools/stream_overlap.py $O/kernel_trace_eager.csv
gzip -f $O/kernel_trace_eager.csv
