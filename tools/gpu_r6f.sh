#!/bin/bash
# LN1 LoRA down-projection / LoRA-A backward on packed dot products: fused-layer GPU tests, the row micro-benchmark
# against the previous LN1 build (RADHIP_LIB), and the in-step A/B (RADHIP_LIB16).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6f}
mkdir -p $O
D=$PWD/robust-audio-deepfake-evolution_amd/radhip
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wavlm_fused_gpu.py tests/test_e2e_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in new old; do
  E=""; [ $v = old ] && E="RADHIP_LIB=$D/libradhip_oldwl.so"
  env $E timeout -k 10 120 python -u tools/bench_wl.py > $O/bench_wl_$v.json 2> $O/bench_wl_$v.err || { tail -5 $O/bench_wl_$v.err; exit 1; }
  python3 - $O/bench_wl_$v.json $v <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    for b, o in d.items():
        print(sys.argv[2], b, {k: v for k, v in o.items() if k.startswith("ln1")})
PY
done
for r in 1 2; do
  for v in new old; do
    E=""; [ $v = old ] && E="RADHIP_LIB16=$D/libradhip_f16_oldwl.so"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
