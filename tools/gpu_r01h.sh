# LoRA weight-grad kernel check: fused-layer parity -> bench -> rocprof stats -> window tests.
# A heartbeat file under gpurun_out/ keeps long silent tests (MIOpen fp32 find) from looking hung.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r01h}
O=gpurun_out/$TAG
mkdir -p $O
(while true; do date >> $O/heartbeat.log; sleep 50; done) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u -m pytest tests/test_wavlm_fused_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -30 $O/pytest_fused.log; exit 1; }
tail -2 $O/pytest_fused.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/prof.err) || exit 1
find /tmp/$TAG -name "*stats*.csv" -exec cp {} $O/ \;
find /tmp/$TAG -name "*kernel_trace.csv" -exec sh -c 'gzip -c "$1" > '$O'/kernel_trace.csv.gz' _ {} \;
grep -i lora $O/run_kernel_stats.csv || true
timeout -k 10 900 python -u -m pytest tests/test_window_gpu.py -v --timeout 600 --timeout-method thread > $O/pytest_window.log 2>&1; rc=$?
tail -3 $O/pytest_window.log
exit $rc
