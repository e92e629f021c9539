# PMC counters for the steady-state bench workload, one rocprofv3 pass per
# counter group (MI355X_MICROARCH.md: separate --pmc passes; FETCH_SIZE and
# WRITE_SIZE cannot share a pass).  Summaries: scripts/pmc_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${OUT:-pmc}
WARM=${WARM:-2500}
STEPS=${STEPS:-50}
i=0
mkdir -p gpurun_out/$OUT
for grp in "$@"; do
  i=$((i+1))
  ctrs=$(echo $grp | tr ',' ' ')
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/$OUT/p$i -o run -- python3 -u bench.py --warmup $WARM --steps $STEPS --stage-batches 0 --pcie-batches 0 --lm-batches 0 --no-cpu > gpurun_out/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$OUT/p$i.log; exit 1; }
  echo "pass $i ($ctrs) ok"
done
