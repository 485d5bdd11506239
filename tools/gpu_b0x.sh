#!/bin/bash
# SincNet block-0 fused kernels on the GPU: parity tests, then the standalone timing under rocprofv3 (kernel stats).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-b0x}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_b0x_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/b0x -o run -- python3 tools/bench_b0x.py --only fused --amp fp16 --reps 6 > $O/bench.log 2>&1
cat $O/bench.log | grep -v "^W\|rocprof" | tail -3
python3 tools/stats_top.py "$(find /tmp/b0x -name '*kernel_stats.csv' | head -1)" 6
if [ -f robust-audio-deepfake-evolution_amd/radhip/libradhip_f16_old.so ]; then   # A/B against a kept build
  for r in 1 2; do
    RADHIP_LIB16=$PWD/robust-audio-deepfake-evolution_amd/radhip/libradhip_f16_old.so timeout -k 10 120 python3 tools/bench_b0x.py --only fused --amp fp16 --reps 8 2>/dev/null | tail -1 | sed 's/^/old /'
    timeout -k 10 120 python3 tools/bench_b0x.py --only fused --amp fp16 --reps 8 2>/dev/null | tail -1 | sed 's/^/new /'
  done
fi
