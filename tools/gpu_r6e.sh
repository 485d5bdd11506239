#!/bin/bash
# LN1 rows per workgroup 4 / 8 / 16 with the LDS-DMA staging: the row micro-benchmark per build (bf16 libraries,
# RADHIP_LIB) and the in-step A/B (fp16 libraries, RADHIP_LIB16).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6e}
mkdir -p $O
D=$PWD/robust-audio-deepfake-evolution_amd/radhip
for R in 4 8 16; do
  E=""; [ $R != 4 ] && E="RADHIP_LIB=$D/libradhip_r$R.so"
  env $E timeout -k 10 120 python -u tools/bench_wl.py > $O/bench_wl_r$R.json 2> $O/bench_wl_r$R.err || { tail -5 $O/bench_wl_r$R.err; exit 1; }
  python3 - $O/bench_wl_r$R.json $R <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    for b, o in d.items():
        print("rows", sys.argv[2], b, {k: v for k, v in o.items() if k.startswith("ln1")})
PY
done
for r in 1 2; do
  for R in 4 8 16; do
    E=""; [ $R != 4 ] && E="RADHIP_LIB16=$D/libradhip_f16_r$R.so"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/r${R}_$r.json 2> $O/r${R}_$r.err || { echo "$R failed"; tail -5 $O/r${R}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/r${R}_$r.json').read().strip().splitlines()[-1]); print('rows$R', $r, d['value'], d['ms_per_step'])"
  done
done
