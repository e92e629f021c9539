# Wave-state and instruction counters per kernel (run on the GPU box):
#   bash scripts/sq_pmc.sh CONFIG [STEPS]   -> gpurun_out/sq_CONFIG/summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=$1; steps=${2:-30}
O=gpurun_out/sq_$cfg
rm -rf $O; mkdir -p $O
p1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR"
p2="SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum"
i=0
for ctrs in "$p1" "$p2"; do
  i=$((i+1))
  FDBCS_LIVE=0 timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d $O/p$i -o run -- \
    python3 -u bench.py --config $cfg --no-cpu --no-shim --lm-batches 0 --stage-batches 0 --latency-batches 0 \
    --steps $steps --warmup 2 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $O $((steps - 1)) k_ingest > $O/summary.txt 2>&1
rm -rf $O/p1 $O/p2
cat $O/summary.txt | head -20
