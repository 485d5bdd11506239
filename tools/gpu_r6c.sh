#!/bin/bash
# LN1 staging by LDS-DMA: the fused-layer GPU tests, the row micro-benchmark, an in-step A/B against the previous
# LN1 kernels (a separately built library, RADHIP_LIB16).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wavlm_fused_gpu.py tests/test_e2e_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -u tools/bench_wl.py > $O/bench_wl.json 2> $O/bench_wl.err || tail -5 $O/bench_wl.err
python3 - $O/bench_wl.json <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    for b, o in d.items():
        print(b, {k: v for k, v in o.items() if k.startswith(("ln1", "add_ln", "ln_bwd", "copy"))})
PY
OW=$PWD/robust-audio-deepfake-evolution_amd/radhip/libradhip_f16_oldwl.so
for r in 1 2; do
  for v in new oldwl; do
    E=""; [ $v = oldwl ] && E="RADHIP_LIB16=$OW"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
