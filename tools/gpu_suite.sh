#!/bin/bash
# The whole -m gpu suite as the driver runs it (one process), log under gpurun_out/<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-suite}
mkdir -p $O
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
exit $rc
