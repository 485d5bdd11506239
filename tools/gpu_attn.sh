#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-attn}
mkdir -p $O
for B in 8 32; do for P in 0.1 0; do
  B=$B P=$P timeout -k 10 120 python -u tools/bench_attn.py
done; done
B=8 RADHIP_ATTN_SPLIT=0 timeout -k 10 120 python -u tools/bench_attn.py
B=8 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/attn -o run -- python3 tools/bench_attn.py > $O/prof.log 2>&1
python3 tools/stats_top.py "$(find /tmp/attn -name '*kernel_stats.csv' | head -1)" 8
