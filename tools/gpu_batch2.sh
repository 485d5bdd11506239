#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-b2}
mkdir -p $O
timeout -k 10 300 python -u tools/op_sites_window.py --top 150 > $O/op_sites.txt 2> $O/op_sites.err || tail -5 $O/op_sites.err
timeout -k 10 400 python -u tools/diag_window_groups.py > $O/diag_window.jsonl 2> $O/diag_window.err
cat $O/diag_window.jsonl | cut -c1-200
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'], 'mfma', d['step_mfma_frac'])"
