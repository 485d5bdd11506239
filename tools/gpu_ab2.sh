# Tests (env TESTS) then an A/B of the bench: default vs the env assignment in $B (e.g. B="RADHIP_B0X=0"), twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-ab2}
mkdir -p gpurun_out/$TAG
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest ${TESTS} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1; rc=$?
  tail -3 gpurun_out/$TAG/tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/a$i.json 2> gpurun_out/$TAG/a$i.err || exit $?
  env $B timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/b$i.json 2> gpurun_out/$TAG/b$i.err || exit $?
  python -c "import json;a=json.load(open('gpurun_out/$TAG/a$i.json'));b=json.load(open('gpurun_out/$TAG/b$i.json'));print('default',a['value'],'variant',b['value'])"
done
