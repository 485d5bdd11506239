# wgemm policy check: the fused-layer / e2e / GEMM GPU tests, then an A/B of the bench under two policies.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-wgab}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_wavlm_fused_gpu.py tests/test_e2e_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$TAG/tests.log
[ $rc -eq 0 ] || exit $rc
OLD='{"b8": {"out": [5, 1], "d_out": [5, 1], "ffn1": [6, 1]}, "b32": {}}'
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/new$i.json 2> gpurun_out/$TAG/new$i.err || exit $?
  RADHIP_WGEMM_POLICY="$OLD" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$TAG/old$i.json 2> gpurun_out/$TAG/old$i.err || exit $?
  python -c "import json;a=json.load(open('gpurun_out/$TAG/new$i.json'));b=json.load(open('gpurun_out/$TAG/old$i.json'));print('new',a['value'],'old',b['value'])"
done
