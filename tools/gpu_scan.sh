set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_kern.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_kern.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_scan.py 2>&1 | grep -v amdgpu.ids
RADHIP_SCAN_BWD_SEG=2 timeout -k 10 120 python tools/bench_scan.py 2>&1 | grep -v amdgpu.ids
