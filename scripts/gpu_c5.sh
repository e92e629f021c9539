# Config 5 (1 M-txn batches over a 10^8-boundary preloaded history) on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c5}; shift
FDBCS_GROWLOG=1 timeout -k 10 900 python -u bench.py --config 5 "$@" > gpurun_out/bench_$TAG.log 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -30 gpurun_out/bench_$TAG.err; cat gpurun_out/bench_$TAG.log
exit $rc
