# WavLM row-kernel micro-benchmark; hipBLASLt / rocBLAS solution tuning of the WavLM layer GEMM shapes only
# (PyTorch TunableOp, tools/tune_wavlm_gemms.py); the bench with that table read back (tuning off).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-tune}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python tools/bench_wl.py > gpurun_out/$TAG/bench_wl.json 2>&1 || exit $?
cat gpurun_out/$TAG/bench_wl.json
timeout -k 10 400 python tools/tune_wavlm_gemms.py --out gpurun_out/$TAG/wavlm_gemms.csv > gpurun_out/$TAG/tune.log 2>&1 || exit $?
tail -3 gpurun_out/$TAG/tune.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$(ls gpurun_out/$TAG/wavlm_gemms*.csv | head -1) \
  timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/$TAG/bench_tuned.json 2> gpurun_out/$TAG/bench_tuned.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/$TAG/bench_tuned.json'));print('TUNED', d['value'], d['ms_per_step'])"
