# End-of-round evidence in one call: the scan parity tests, then tools/gpu_round.sh (smoke, default bench line with
# the CPU baseline, rocprofv3 kernel-trace stats) and the two PMC passes of tools/gpu_pmc_bench.sh.
# TAG names gpurun_out/<TAG> (the PMC CSVs go to gpurun_out/<TAG>_pmc).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-final}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_wgrad_gpu.py -m gpu -x -q -k "scan or mamba or wgrad" --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests_quick.log 2>&1 || { tail -20 gpurun_out/$TAG/tests_quick.log; exit 1; }
tail -1 gpurun_out/$TAG/tests_quick.log
TAG=$TAG NOTESTS=1 bash tools/gpu_round.sh || exit $?
TAG=${TAG}_pmc bash tools/gpu_pmc_bench.sh || exit $?
