#!/bin/bash
# sconv forward with branch-free buffer IO and LDS operand reads 4 steps ahead: its GPU tests (sconv, b0x, the
# SincNet fixtures, the window), the per-shape micro-benchmark against the previous build (tools/ab/old, the
# same sources with HEAD's sconv.hip), then an in-step A/B (new vs old library), two rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6i}
mkdir -p $O
OLD="RADHIP_LIB=$PWD/tools/ab/old/libradhip.so RADHIP_LIB16=$PWD/tools/ab/old/libradhip_f16.so"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sconv_gpu.py tests/test_b0x_gpu.py tests/test_fixtures_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/bench_sconv.py --batch 8 32 > $O/sconv_new.jsonl 2> $O/sconv_new.err || { tail -5 $O/sconv_new.err; exit 1; }
env $OLD timeout -k 10 300 python -u tools/bench_sconv.py --batch 8 32 > $O/sconv_old.jsonl 2> $O/sconv_old.err || { tail -5 $O/sconv_old.err; exit 1; }
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
def rd(f):
    return [json.loads(l) for l in open(f) if l.startswith("{")]
for a, b in zip(rd(f"{o}/sconv_new.jsonl"), rd(f"{o}/sconv_old.jsonl")):
    print({k: a[k] for k in a if not isinstance(a[k], float)}, {k: (round(a[k], 1), round(b[k], 1)) for k in a if isinstance(a[k], float)})
PY
for r in 1 2; do
  for v in new old; do
    E=""; [ $v = old ] && E="$OLD"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['value'], d['ms_per_step'])"
  done
done
