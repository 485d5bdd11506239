# rocprofv3 kernel trace (+stats) of a short bench run; TAG names gpurun_out/<TAG>; extra env passes through.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-trace}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err
rc=$?
find /tmp/$TAG -name "*stats*.csv" -exec cp {} $O/ \;
find /tmp/$TAG -name "*kernel_trace.csv" -exec sh -c 'gzip -c "$1" > '$O'/kernel_trace.csv.gz' _ {} \;
echo "TRACE EXIT $rc"
exit $rc
