# PMC passes over tools/bench_b0x.py (fused only), one counter group per run; outputs under gpurun_out/$TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-pmcb0}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 python tools/bench_b0x.py --reps 5 > $O/bench.txt 2>&1 || exit $?
cat $O/bench.txt
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d /tmp/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_b0x.py --reps 2 --only fused > $O/pmc$i.out 2>&1
  rc=$?
  echo "PMC group $i EXIT $rc"
  [ $rc -eq 0 ] || exit $rc
  find /tmp/pmc$i -name "*counter_collection.csv" -exec cp {} $O/pmc$i.csv \;
done
