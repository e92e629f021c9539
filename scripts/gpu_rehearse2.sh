# Rehearse the N=2 exact mode on ONE GPU (two ranks on device 0, gloo exchanges), protocols B and A.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp FDBCS_BENCH_BACKEND=gloo FDBCS_BENCH_ALT=0 FDBCS_PHASES_HOST=1
W=${WARM:-1000}
for P in b a; do
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2951$RANDOM_SUFFIX bench.py --gpus 2 --steps 100 --warmup $W --no-cpu --protocol $P > gpurun_out/reh2_$P.log 2> gpurun_out/reh2_$P.err || { echo "rehearsal $P failed"; tail -30 gpurun_out/reh2_$P.err; exit 1; }
echo "== protocol $P"; grep "phase" gpurun_out/reh2_$P.err; cat gpurun_out/reh2_$P.log
done
