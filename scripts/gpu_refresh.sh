# Round-end measurement refresh: default bench, rocprof kernel stats, PMC traffic.
# usage: bash scripts/gpu_refresh.sh r01
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${1:-r01}
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$R.log 2> gpurun_out/bench_$R.err || { echo "bench failed"; tail -20 gpurun_out/bench_$R.err; exit 1; }
cat gpurun_out/bench_$R.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R -o run -- python3 -u bench.py --steps 200 --stage-batches 0 --pcie-batches 0 --lm-batches 0 --no-cpu > gpurun_out/prof_$R.log 2> gpurun_out/prof_$R.err || { echo "prof failed"; tail -20 gpurun_out/prof_$R.err; exit 1; }
cat gpurun_out/prof_$R.log
python3 scripts/prof_summary.py gpurun_out/prof_$R/run_kernel_trace.csv 199 > gpurun_out/kstats_$R.txt && cat gpurun_out/kstats_$R.txt
cp gpurun_out/prof_$R/run_kernel_stats.csv gpurun_out/kernel_stats_$R.csv 2>/dev/null
rm -f gpurun_out/prof_$R/run_kernel_trace.csv
OUT=pmc_$R bash scripts/gpu_pmc.sh FETCH_SIZE WRITE_SIZE || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc_$R 50 k_ingest gpurun_out/pmc_traffic_$R.json > gpurun_out/pmc_$R.txt && cat gpurun_out/pmc_$R.txt
rm -rf gpurun_out/pmc_$R
