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
# PMC: HBM bytes per scan kernel launch (FETCH_SIZE x 2 + WRITE_SIZE, KiB) over tools/bench_scan.py
if [ -n "$PMC" ]; then
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d /tmp/scanpmc_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_scan.py > $O/pmc_$c.log 2>&1) || exit $?
  find /tmp/scanpmc_$c -name "*counter_collection.csv" -exec cp {} $O/pmc_$c.csv \;
done
python3 - "$O" <<'PY'
import csv, sys, collections
o = sys.argv[1]
acc = collections.defaultdict(lambda: [0.0, 0.0, set()])
for j, c in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
    for r in csv.DictReader(open(f"{o}/pmc_{c}.csv")):
        if r.get("Counter_Name") != c or "s2::" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void rdx::s2::", "")
        acc[k][j] += float(r["Counter_Value"]) * 1024 * (2 if j == 0 else 1)
        acc[k][2].add((j, r.get("Dispatch_Id")))
for k, (f, w, ids) in acc.items():
    n = max(1, len([i for i in ids if i[0] == 0]))
    print(f"PMC {k:40s} {(f + w * n / max(1, len([i for i in ids if i[0] == 1]))) / n / 1e6:8.2f} MB/launch (fetch x2 {f / n / 1e6:.2f}, write {w / max(1, len([i for i in ids if i[0] == 1])) / 1e6:.2f})")
PY
fi
