# Rehearse the multi-resolver bench path: 2 ranks on one GPU over gloo (the
# driver runs the real N-GPU RCCL version on an 8-GPU node).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FDBCS_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --warmup ${WARM:-300} --steps 50 --stage-batches 10 > gpurun_out/bench_mr.log 2> gpurun_out/bench_mr.err || { echo "mr bench failed"; tail -30 gpurun_out/bench_mr.err; exit 1; }
cat gpurun_out/bench_mr.log
