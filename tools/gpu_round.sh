# Full round check: smoke -> default bench (with CPU baseline) -> rocprof kernel-trace stats -> GPU tests.
# Stops at the first failing step. TAG names the output directory under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-round}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1; rc=$?
tail -1 gpurun_out/$TAG/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; rc=$?
cat gpurun_out/$TAG/bench.json
[ $rc -eq 0 ] || exit $rc
if [ -z "$NOPROF" ]; then
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/$TAG/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof.err); rc=$?
find /tmp/$TAG -name "*stats*.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/$TAG/ \;
find /tmp/$TAG -name "*kernel_trace.csv" -exec sh -c 'gzip -c "$1" > '$GRAFT_REPO_ROOT'/gpurun_out/'$TAG'/kernel_trace.csv.gz' _ {} \;
echo PROF EXIT $rc
[ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/$TAG/pytest.log | tail -3
exit $rc
fi
