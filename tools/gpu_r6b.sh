#!/bin/bash
# 16-bit lora_A staging in the WavLM LN1 kernels and the loads-first attention forward: their GPU tests, the row and
# attention micro-benchmarks under rocprofv3, then an in-step A/B against the previous attention forward and against
# 8 rows per LN1 workgroup (separately built libraries, RADHIP_LIB16).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wavlm_fused_gpu.py tests/test_e2e_gpu.py tests/test_kernels_gpu.py -k "attention or wavlm or e2e or bench_config" tests/test_f16_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -u tools/bench_wl.py > $O/bench_wl.json 2> $O/bench_wl.err || tail -5 $O/bench_wl.err
python3 - $O/bench_wl.json <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    for b, o in d.items():
        print(b, {k: v for k, v in o.items() if k.startswith(("ln1", "add_ln", "ln_bwd", "copy", "attn"))})
PY
for L in new oldattn; do
  E=""; [ $L = oldattn ] && E="RADHIP_LIB16=$PWD/robust-audio-deepfake-evolution_amd/radhip/libradhip_f16_oldattn.so"
  rm -rf /tmp/at_$L
  env $E B=8 P=0.1 DT=fp16 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/at_$L -o run -- python3 tools/bench_attn.py > $O/attn_$L.log 2>&1
  echo "== $L"; python3 tools/stats_top.py "$(find /tmp/at_$L -name '*kernel_stats.csv' | head -1)" 4
done
OA=$PWD/robust-audio-deepfake-evolution_amd/radhip/libradhip_f16_oldattn.so
R8=$PWD/robust-audio-deepfake-evolution_amd/radhip/libradhip_f16_r8.so
for r in 1 2; do
  for v in new oldattn rows8; do
    E=""; [ $v = oldattn ] && E="RADHIP_LIB16=$OA"; [ $v = rows8 ] && E="RADHIP_LIB16=$R8"
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', $r, d['value'], d['ms_per_step'], 'attn_fwd', k['attn_fwd']['avg_ms'])"
  done
done
