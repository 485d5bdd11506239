# Diagnostics: rocprofv3 kernel stats of the scan microbenchmark (both scan implementations) and the op-site
# census of one eager micro-step (tools/op_sites.py); outputs under gpurun_out/$TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-diag}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/scanprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_scan.py > $O/scan_prof.log 2>&1) || exit $?
find /tmp/scanprof -name "*kernel_stats.csv" -exec cp {} $O/scan_kernel_stats.csv \;
timeout -k 10 300 python tools/op_sites.py > $O/op_sites.txt 2> $O/op_sites.err || exit $?
tail -5 $O/op_sites.txt
