#!/bin/bash
# posconv window staging loads-first and the per-window SincNet weight layouts in one launch: GPU tests, then an
# in-step A/B of the weight preparation (RADHIP_SCONV_PREP=0 = on first use, torch ops).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6d}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sconv_wprep_gpu.py tests/test_kernels_gpu.py tests/test_f16_gpu.py tests/test_sconv_gpu.py tests/test_window_gpu.py -k "wprep or posconv or sconv or window" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in new noprep; do
    E=""; [ $v = noprep ] && E="RADHIP_SCONV_PREP=0"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', $r, d['value'], d['ms_per_step'], 'posconv', k['posconv_fwd']['avg_ms'], k['posconv_bwd']['avg_ms'])"
  done
done
