# Targeted GPU tests (env TESTS) then the default bench without the CPU baseline; TAG names gpurun_out/<TAG>.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-chk}
mkdir -p gpurun_out/$TAG
timeout -k 10 ${TTIME:-700} python -u -m pytest ${TESTS} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/$TAG/bench.json'));print('BENCH', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
