# N=2 rehearsal of the bench's multi-GPU path on ONE GPU over gloo host
# collectives (both ranks share GPU 0), per-rank kernel traces (GPU box):
#   bash scripts/rehearse_n2.sh TREE LABEL [trace=1]
# TREE: a repo tree (. or a worktree of an older commit, built in place).
# Outputs: gpurun_out/reh_LABEL/{line.json, r0.log, r1.log, kt_r{0,1}.txt}
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$PWD/gpurun_out/reh_$2
mkdir -p $O
cd $1
export TMPDIR=/tmp FDBCS_BENCH_BACKEND=gloo WORLD_SIZE=2 MASTER_ADDR=127.0.0.1
args="--gpus 2 --steps ${STEPS:-20} --warmup 5 --no-cpu"
run() {  # $1: port, $2: prefix command for each rank (empty, or a rocprofv3 invocation)
  for r in 0 1; do
    RANK=$r LOCAL_RANK=$r MASTER_PORT=$1 timeout -k 10 420 $2 python3 -u bench.py $args > $O/r$r$3.log 2>&1 &
  done
  wait %1 && wait %2
}
run 29611 "" "" || { echo "rehearsal failed"; tail -5 $O/r0.log $O/r1.log; exit 1; }
grep "^{" $O/r0.log | tail -1 > $O/line.json
python3 -c "
import json; d=json.load(open('$O/line.json'))
print('$2', 'ms_per_step', d['ms_per_step'], 'p50', d['p50_batch_ms'], 'p99', d['p99_batch_ms'], 'adds', d['add_us_mean'])"
[ "${3:-1}" = 1 ] || exit 0
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r MASTER_PORT=29612 timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/kt_r$r -o run -- python3 -u bench.py $args > $O/r${r}_kt.log 2>&1 &
done
wait %1 && wait %2 || { echo "traced rehearsal failed"; tail -5 $O/r0_kt.log; exit 1; }
for r in 0 1; do
  kt=$(find $O/kt_r$r -name "*kernel_trace.csv" | head -1)
  python3 $GRAFT_REPO_ROOT/scripts/prof_summary.py "$kt" ${STEPS:-20} k_ingest > $O/kt_r$r.txt 2>&1
  rm -rf $O/kt_r$r
done
head -25 $O/kt_r0.txt
