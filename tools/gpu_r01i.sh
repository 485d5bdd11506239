# A/B of the pipelined LoRA weight-grad kernel: fused-layer parity, then rocprof kernel stats of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r01i}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wavlm_fused_gpu.py -v --timeout 200 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -30 $O/pytest_fused.log; exit 1; }
tail -2 $O/pytest_fused.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/prof.err) || exit 1
find /tmp/$TAG -name "*stats*.csv" -exec cp {} $O/ \;
find /tmp/$TAG -name "*kernel_trace.csv" -exec sh -c 'gzip -c "$1" > '$O'/kernel_trace.csv.gz' _ {} \;
grep -i lora $O/run_kernel_stats.csv || true
cut -c1-120 $O/bench_prof.json
