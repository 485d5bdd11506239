#!/bin/bash
# Round-6 evidence on the final tree. Part "pmc": the two PMC passes over bench.py's own launches and their summary
# (profiles/pmc_traffic.json, read by the bench line's roofline.traffic). Part "line": smoke, the default bench line
# (with the bounded CPU baseline), a rocprofv3 kernel trace of a short bench run and its timed-region summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r06f}
PART=${1:-line}
O=gpurun_out/$TAG
mkdir -p $O
if [ "$PART" = pmc ]; then
  TAG=${TAG}_pmc bash tools/gpu_pmc_bench.sh || exit $?
  cd "$GRAFT_REPO_ROOT"
  python3 tools/pmc_bench.py gpurun_out/${TAG}_pmc > $O/pmc_traffic.json || exit $?
  python3 -c "import json; d=json.load(open('$O/pmc_traffic.json')); print('hgemm', d.get('hgemm'))"
  exit 0
fi
[ -f $O/pmc_traffic.json ] && cp $O/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('BENCH', d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:300], json.dumps(d['cpu_baseline'])[:300])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err || { tail -10 $O/prof.err; exit 1; }
find /tmp/$TAG -name "*kernel_stats.csv" -exec cp {} $O/ \;
cp "$(find /tmp/$TAG -name '*kernel_trace.csv' | head -1)" $O/kernel_trace.csv
python3 tools/prof_summary.py $O/kernel_trace.csv --micro 16 --before ts_acc_kernel --top 60 > $O/steady_state.txt
gzip -f $O/kernel_trace.csv
head -12 $O/steady_state.txt
