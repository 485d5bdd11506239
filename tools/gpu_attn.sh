# Attention parity tests + kernel-trace timing of the attention kernels at the window's two batch shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-attn}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_wavlm_fused_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTK:-attention or fused}" > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -3
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for B in 8 32; do
  B=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt_$B -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_kernels.py > $O/kbench_$B.json 2> $O/kbench_$B.err
  rc=$?
  echo "B=$B EXIT $rc"; cat $O/kbench_$B.json
  [ $rc -eq 0 ] || exit $rc
  find /tmp/kt_$B -name "*kernel_stats.csv" -exec cp {} $O/kstats_$B.csv \;
  grep -E "attn|posconv|b0_bwd" $O/kstats_$B.csv | cut -d, -f1-8
done
