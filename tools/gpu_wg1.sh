set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wg1
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wg1/tests.log 2>&1; rc=$?
tail -3 gpurun_out/wg1/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/bench_wgemm.py --B 8,32 --reps 30 --tiles 5,45,6,46,12,52,16,56,20,21,12x2,12x3,12x4,20x2,20x4,16x4,14x2,14x4,18x4,0x2,5x2 > gpurun_out/wg1/bench.jsonl 2> gpurun_out/wg1/bench.err
