# Evidence for the bench line: rocprofv3 kernel-trace stats of a short bench run (the same command as the
# driver's, fewer steps), then HBM traffic of the attention kernels from separate PMC passes (FETCH_SIZE,
# WRITE_SIZE; one counter group per run) over tools/bench_kernels.py at the window's two batch shapes.
# Outputs under gpurun_out/$TAG; tools/pmc_traffic.py turns the PMC CSVs into profiles/pmc_traffic.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-prof}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ -z "$NOTRACE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err
  rc=$?
  find /tmp/$TAG -name "*stats*.csv" -exec cp {} $O/ \;
  find /tmp/$TAG -name "*kernel_trace.csv" -exec sh -c 'gzip -c "$1" > '$O'/kernel_trace.csv.gz' _ {} \;
  echo "TRACE EXIT $rc"
  [ $rc -eq 0 ] || exit $rc
fi
for B in 8 32; do
  for c in FETCH_SIZE WRITE_SIZE; do
    B=$B timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d /tmp/pmc_${c}_$B -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_kernels.py > $O/attn_${c}_$B.out 2>&1
    rc=$?
    echo "PMC $c B=$B EXIT $rc"
    [ $rc -eq 0 ] || exit $rc
    find /tmp/pmc_${c}_$B -name "*counter_collection.csv" -exec cp {} $O/attn_${c}_$B.csv \;
  done
done
