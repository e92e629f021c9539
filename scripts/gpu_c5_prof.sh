# Config 5 bench (with the CPU baseline) + rocprof kernel stats of a short config 5 run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c5}
timeout -k 10 600 python -u bench.py --config 5 --cpu-seconds 10 > gpurun_out/bench_$TAG.log 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --config 5 --steps 6 --stage-batches 0 --pcie-batches 0 --no-cpu > gpurun_out/prof_$TAG.log 2> gpurun_out/prof_$TAG.err || { echo "prof failed"; tail -20 gpurun_out/prof_$TAG.err; exit 1; }
cp gpurun_out/prof_$TAG/run_kernel_stats.csv gpurun_out/kernel_stats_$TAG.csv
python3 scripts/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv 6 > gpurun_out/kstats_$TAG.txt && cat gpurun_out/kstats_$TAG.txt
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv
