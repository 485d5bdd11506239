# Targeted GPU check: the named pytest files (env TESTS), then an optional short bench (env BENCH=1).
# Stops at the first failing step. TAG names the output directory under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-check}
mkdir -p gpurun_out/$TAG
timeout -k 10 ${TTIME:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout ${TTEST:-300} --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/$TAG/pytest.log | tail -3
[ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
timeout -k 10 500 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; rc=$?
tail -c 3000 gpurun_out/$TAG/bench.json
exit $rc
fi
