# A/B of the bench between the tree's defaults (A) and env B_ENV (B), alternating, on one box; optional GPU tests
# first (TESTS). Prints value per run; lines in gpurun_out/$TAG/{a,b}N.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-ab}
mkdir -p gpurun_out/$TAG
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1; rc=$?
  tail -3 gpurun_out/$TAG/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 ${ROUNDS:-2}); do
  timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/a$i.json 2> gpurun_out/$TAG/a$i.err || exit $?
  env $B_ENV timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/b$i.json 2> gpurun_out/$TAG/b$i.err || exit $?
  python -c "import json;a=json.load(open('gpurun_out/$TAG/a$i.json'));b=json.load(open('gpurun_out/$TAG/b$i.json'));print('A',a['value'],'B',b['value'])"
done
