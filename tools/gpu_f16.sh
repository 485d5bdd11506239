# fp16 product path: smoke, the fp16 kernel tests, the tests parametrized over fp16, then the e2e floor test.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-f16}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -1 $O/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_f16_gpu.py tests/test_b0x_gpu.py -m gpu -v -x --timeout 300 --timeout-method thread > $O/f16.log 2>&1; rc=$?
grep -E "passed|failed|Error" $O/f16.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -v -x -k "scan2 or layer_weighted or residual_block" --timeout 300 --timeout-method thread > $O/kern.log 2>&1; rc=$?
grep -E "passed|failed|Error" $O/kern.log | tail -5
[ $rc -eq 0 ] || exit $rc
if [ -z "$NOE2E" ]; then
timeout -k 10 900 python -u -m pytest tests/test_e2e_gpu.py -m gpu -v -s -x --timeout 600 --timeout-method thread > $O/e2e.log 2>&1; rc=$?
grep -E "floor|e2e|passed|failed" $O/e2e.log | tail -30
exit $rc
fi
