# Named GPU test files (env TESTS) only; TAG names gpurun_out/<TAG>.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-t}
mkdir -p gpurun_out/$TAG
timeout -k 10 ${TTIME:-600} python -u -m pytest ${TESTS} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/$TAG/tests.log | tail -30
exit $rc
