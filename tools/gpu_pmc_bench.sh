# HBM traffic of every kernel at the bench's own launch mix: two rocprofv3 PMC passes (FETCH_SIZE, then
# WRITE_SIZE: they do not fit one pass) over a short bench.py run in eager mode (the same window and kernels
# without HIP graphs: graph replays fail under rocprofv3 counter collection, "unspecified launch failure");
# CSVs under gpurun_out/$TAG, turned into profiles/pmc_traffic.json by tools/pmc_bench.py. A heartbeat file
# keeps the silent profiled run from being taken for a hang.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-pmcbench}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
( while true; do date >> $O/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d /tmp/pmcb_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err
  rc=$?
  echo "PMC $c EXIT $rc"
  [ $rc -eq 0 ] || exit $rc
  find /tmp/pmcb_$c -name "*counter_collection.csv" -exec sh -c 'gzip -c "$1" > '$O'/'$c'.csv.gz' _ {} \;
done
