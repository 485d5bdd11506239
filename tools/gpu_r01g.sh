# Round-1 iteration on the GPU box: the kernels' parity tests first (small shapes), then the fused-layer /
# window tests, then the bench (accumulation window + HIP graphs). A plain test failure (exit 1) still runs
# the bench; a GPU fault, abort or time limit ends the script. TAG names the output directory under
# gpurun_out/; KTESTS / TESTS override the two test groups, BENCH_ARGS is passed to bench.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r01g}
mkdir -p $O
run_tests() {  # $1 = log name, the rest = pytest targets
  local log=$1
  shift
  timeout -k 10 ${TT:-700} python -u -m pytest "$@" -v --timeout 300 --timeout-method thread > $O/$log 2>&1
  local rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" $O/$log | tail -${NL:-60}
  return $rc
}
rc1=0
if [ -z "$SKIP_KERNELS" ]; then
  run_tests pytest_kernels.log ${KTESTS:-tests/test_kernels_gpu.py}
  rc1=$?
  case $rc1 in 0|1) ;; *) exit $rc1 ;; esac
fi
run_tests pytest_model.log ${TESTS:-tests/test_wavlm_fused_gpu.py tests/test_window_gpu.py}
rc2=$?
case $rc2 in 0|1) ;; *) exit $rc2 ;; esac
if [ -z "$NOBENCH" ]; then
  timeout -k 10 500 python bench.py --no-cpu-baseline ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || exit $?
  python3 tools/brief.py $O/bench.json
fi
exit $(( rc1 | rc2 ))
