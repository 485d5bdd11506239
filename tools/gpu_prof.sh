# rocprofv3 kernel trace of a short graph-mode bench; keeps stats CSVs + gzipped trace under gpurun_out/$TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-prof}
make -C robust-audio-deepfake-evolution_amd/csrc -j8 > /dev/null || exit 1
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/$TAG/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/err.log
rc=$?
find /tmp/$TAG -name "*stats*.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/$TAG/ \;
find /tmp/$TAG -name "*kernel_trace.csv" -exec sh -c 'gzip -c "$1" > '$GRAFT_REPO_ROOT'/gpurun_out/'$TAG'/kernel_trace.csv.gz' _ {} \;
echo EXIT $rc
exit $rc
