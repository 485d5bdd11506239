# Scan kernels: parity tests, then rocprofv3 kernel stats of tools/bench_scan.py (gpurun_out/$TAG).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-scan}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fixtures_gpu.py -m gpu -x -q -k "mamba or scan2 or pn_bimamba or bimamba" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/scanprof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_scan.py > $O/scan_prof.log 2>&1) || exit $?
find /tmp/scanprof -name "*kernel_stats.csv" -exec cp {} $O/scan_kernel_stats.csv \;
python3 -c "
import csv
for r in csv.DictReader(open('$O/scan_kernel_stats.csv')):
    if 's2::' in r['Name'] or 'scan' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1e3,2), r['Name'][:60])
"
