set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_r01c.json 2> gpurun_out/bench_r01c.err; rc=$?
cat gpurun_out/bench_r01c.json; grep -v amdgpu.ids gpurun_out/bench_r01c.err | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --eager --no-cpu-baseline > gpurun_out/bench_r01c_eager.json 2> gpurun_out/bench_r01c_eager.err; rc=$?
cat gpurun_out/bench_r01c_eager.json
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r01c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_r01c_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_r01c.err
rc=$?
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof_r01c
find /tmp/prof_r01c -name "*stats*.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof_r01c/ \;
find /tmp/prof_r01c -name "*kernel_trace.csv" -exec sh -c 'gzip -c "$1" > '$GRAFT_REPO_ROOT'/gpurun_out/prof_r01c/kernel_trace.csv.gz' _ {} \;
echo EXIT $rc
