set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fz
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_wavlm_fused_gpu.py tests/test_cli_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py} -x -v --timeout 300 --timeout-method thread > gpurun_out/fz/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/fz/pytest.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/fz/bench.json 2> gpurun_out/fz/bench.err; rc=$?
tail -3 gpurun_out/fz/bench.err; python3 -c "import json;d=json.load(open('gpurun_out/fz/bench.json'));print('VALUE',d['value'],'ms/step',d['ms_per_step'],'loss',d['final_loss']);print({k:(round(v['avg_ms']*1e3,1),v['launches']) for k,v in d['kernels'].items()})"
exit $rc
