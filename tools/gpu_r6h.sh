#!/bin/bash
# Fused head pieces (SE, attention pooling, upsample + concat): their GPU tests, the model / window / e2e tests, then an in-step A/B
# against the module path (RADHIP_SE_FUSED=0 RADHIP_POOL_FUSED=0 RADHIP_UPCAT_FUSED=0).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6h}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_head_gpu.py tests/test_model_gpu.py tests/test_e2e_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in new module; do
    E=""; [ $v = module ] && E="RADHIP_SE_FUSED=0 RADHIP_POOL_FUSED=0 RADHIP_UPCAT_FUSED=0"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
