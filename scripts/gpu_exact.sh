# Exact sharded mode rehearsal on one GPU: N ranks over gloo sharing the card, plus an N=1 check.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${1:-2}
WARM=${WARM:-500}
[ -n "$SKIP1" ] || timeout -k 10 300 python -u bench.py --warmup $WARM --steps 100 --stage-batches 20 --no-cpu > gpurun_out/ex_n1.log 2> gpurun_out/ex_n1.err || { echo "n1 failed"; tail -20 gpurun_out/ex_n1.err; exit 1; }
[ -n "$SKIP1" ] || cat gpurun_out/ex_n1.log
FDBCS_VERBOSE=1 FDBCS_PHASES_HOST=1 FDBCS_BENCH_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $N --warmup $WARM --steps 100 --no-cpu > gpurun_out/ex_n$N.log 2> gpurun_out/ex_n$N.err || { echo "n$N failed"; tail -30 gpurun_out/ex_n$N.err; exit 1; }
cat gpurun_out/ex_n$N.log
grep "phase" gpurun_out/ex_n$N.err
grep "grow\|timed" gpurun_out/ex_n$N.err | tail -40
