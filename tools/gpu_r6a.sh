#!/bin/bash
# Round-6 checks: b0x forward (weights in registers) and the fused feature_projection: their GPU tests, then an
# in-step A/B (bench.py, interleaved) of the new tree against the previous b0x build and the module feature_projection.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_b0x_gpu.py tests/test_featproj_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
OLD=$PWD/robust-audio-deepfake-evolution_amd/radhip/libradhip_f16_old.so
for r in 1 2; do
  for v in new old_b0x no_fp; do
    case $v in
      new) E="";;
      old_b0x) E="RADHIP_LIB16=$OLD";;
      no_fp) E="RADHIP_FEATPROJ=0";;
    esac
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', $r, d['value'], d['ms_per_step'], 'b0x_fwd', k['b0x_fwd']['avg_ms'])"
  done
done
