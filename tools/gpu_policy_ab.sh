#!/bin/bash
# In-step A/B of WavLM GEMM policy variants (RADHIP_WGEMM_POLICY JSON tables), interleaved, 2 rounds, one box.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pab}
mkdir -p $O
BASE8='"qkv": ["hg", 3, 1, 4], "out": ["hg", 6, 1, 4], "d_out": ["hg", 6, 1, 4], "ffn1": ["hg", 202, 1, 0], "d_ffn2": ["hg", 202, 1, 0], "ffn2": ["hg", 4, 2, 4], "d_ffn1": ["hg", 4, 2, 4], "d_qkv": ["hg", 4, 2, 4]'
B32='"b32": {"qkv": ["hg", 1, 1, 4], "out": ["hg", 2, 1, 4], "d_out": ["hg", 2, 1, 4], "ffn1": ["hg", 0, 1, 4], "d_ffn2": ["hg", 0, 1, 4], "ffn2": ["hg", 2, 1, 4], "d_ffn1": ["hg", 2, 1, 4], "d_qkv": ["hg", 2, 1, 4]}'
declare -A P
P[base]="{\"b8\": {$BASE8}, $B32}"
P[f7]="{\"b8\": {$BASE8, \"ffn1\": [\"hg\", 7, 1, 4], \"d_ffn2\": [\"hg\", 7, 1, 4]}, $B32}"
P[k6]="{\"b8\": {$BASE8, \"ffn2\": [\"hg\", 6, 2, 4], \"d_ffn1\": [\"hg\", 6, 2, 4], \"d_qkv\": [\"hg\", 6, 2, 4]}, $B32}"
P[q7]="{\"b8\": {$BASE8, \"qkv\": [\"hg\", 7, 1, 4]}, $B32}"
P[b32k4]="{\"b8\": {$BASE8}, \"b32\": {\"qkv\": [\"hg\", 1, 1, 4], \"out\": [\"hg\", 2, 1, 4], \"d_out\": [\"hg\", 2, 1, 4], \"ffn1\": [\"hg\", 0, 1, 4], \"d_ffn2\": [\"hg\", 0, 1, 4], \"ffn2\": [\"hg\", 5, 1, 4], \"d_ffn1\": [\"hg\", 5, 1, 4], \"d_qkv\": [\"hg\", 5, 1, 4]}}"
ROUNDS=${ROUNDS:-2}
VARIANTS=${VARIANTS:-base f7 k6 q7 b32k4}
for r in $(seq 1 $ROUNDS); do
  for v in $VARIANTS; do
    RADHIP_WGEMM_POLICY="${P[$v]}" timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -3 $O/${v}_$r.err; continue; }
    python3 -c "import json; d=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v round $r', d['value'], d['ms_per_step'])"
  done
done
