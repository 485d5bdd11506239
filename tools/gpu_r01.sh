set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== default" > gpurun_out/gms.log
timeout -k 10 200 python tools/graph_memset_repro.py 2>&1 | grep -v amdgpu.ids | head -4 >> gpurun_out/gms.log
echo "== DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" >> gpurun_out/gms.log
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python tools/graph_memset_repro.py 2>&1 | grep -v amdgpu.ids | head -4 >> gpurun_out/gms.log
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python tools/graph_replay_repro.py 2>&1 | grep -v amdgpu.ids | grep replay >> gpurun_out/gms.log
cat gpurun_out/gms.log
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r01 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_r01_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_r01.err
rc=$?
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/prof_r01
find /tmp/prof_r01 -type f | head -20
find /tmp/prof_r01 -name "*stats*.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof_r01/ \;
find /tmp/prof_r01 -name "*kernel_trace.csv" -exec sh -c 'gzip -c "$1" > '$GRAFT_REPO_ROOT'/gpurun_out/prof_r01/kernel_trace.csv.gz' _ {} \;
ls -la $GRAFT_REPO_ROOT/gpurun_out/prof_r01
echo EXIT $rc
