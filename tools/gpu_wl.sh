set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wl2
timeout -k 10 300 python tools/bench_wl.py > gpurun_out/wl2/bench_wl.json 2>&1 || exit $?
cat gpurun_out/wl2/bench_wl.json | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_wavlm_fused_gpu.py tests/test_graph_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/wl2/tests.log 2>&1; rc=$?
tail -3 gpurun_out/wl2/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/wl2/bench.json 2> gpurun_out/wl2/bench.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/wl2/bench.json'));print('BENCH', d['value'], d['ms_per_step'])"
