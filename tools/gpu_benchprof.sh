#!/bin/bash
# The bench line, then a rocprofv3 kernel trace of a short bench run summarised over its TIMED region (the unstamped
# window replays, before the stamped kernel-timing replay: tools/prof_summary.py --before ts_acc_kernel).
#   bash tools/gpu_benchprof.sh <tag> [bench steps]
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r06}; STEPS=${2:-20}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'ms/step', d['ms_per_step'], 'roofline', {k: d['roofline'][k] for k in ('kernel','frac','achieved')}, 'mfma', d['step_mfma_frac'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err
find /tmp/$TAG -name "*kernel_stats.csv" -exec cp {} $O/ \;
cp "$(find /tmp/$TAG -name '*kernel_trace.csv' | head -1)" $O/kernel_trace.csv
python3 tools/prof_summary.py $O/kernel_trace.csv --micro 16 --before ts_acc_kernel --top 45 > $O/steady_state.txt
gzip -f $O/kernel_trace.csv
head -60 $O/steady_state.txt
