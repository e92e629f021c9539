# Full-size bench (defaults = the driver's run) + rocprof kernel trace of the same workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${1:-r01}
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$OUT.log 2> gpurun_out/bench_$OUT.err || { echo "bench failed"; tail -20 gpurun_out/bench_$OUT.err; exit 1; }
cat gpurun_out/bench_$OUT.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$OUT -o run -- python3 -u bench.py --no-cpu > gpurun_out/prof_$OUT.log 2> gpurun_out/prof_$OUT.err || { echo "prof failed"; tail -20 gpurun_out/prof_$OUT.err; exit 1; }
cat gpurun_out/prof_$OUT.log
find gpurun_out/prof_$OUT -name "*stats*"
