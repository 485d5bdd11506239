#!/bin/bash
# A/B of RADHIP_SINC_EARLY_BWD (SincNet backward issued from a hook on its output) on one box, 2 rounds.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abe}
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    RADHIP_SINC_EARLY_BWD=$v timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/e${v}_$r.json 2> $O/e${v}_$r.err
    python3 -c "import json; d=json.loads(open('$O/e${v}_$r.json').read().strip().splitlines()[-1]); print('early=$v round $r', d['value'], d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RADHIP_SINC_EARLY_BWD=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/abe -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/prof.json 2> $O/prof.err
cp "$(find /tmp/abe -name '*kernel_trace.csv' | head -1)" $O/kernel_trace.csv
python3 tools/stream_overlap.py $O/kernel_trace.csv
gzip -f $O/kernel_trace.csv
