# pgemm sweep: correctness + timing of csrc/pgemm.hip tiles vs hipBLASLt / wgemm (tools/bench_pgemm.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-pg}
mkdir -p gpurun_out/$TAG
timeout -k 10 ${TTIME:-500} python -u tools/bench_pgemm.py ${PGARGS} > gpurun_out/$TAG/sweep.jsonl 2> gpurun_out/$TAG/sweep.err; rc=$?
tail -3 gpurun_out/$TAG/sweep.err
exit $rc
