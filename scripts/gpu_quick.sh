# Parity tests + short bench (+ optional rocprof of the short bench).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-q}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --warmup ${WARM:-2500} --steps 200 --cpu-seconds 3 > gpurun_out/bench_$TAG.log 2> gpurun_out/bench_$TAG.err || { echo bench failed; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.log
if [ -n "$PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --warmup ${WARM:-2500} --steps 200 --no-cpu > gpurun_out/prof_$TAG.log 2> gpurun_out/prof_$TAG.err || { echo prof failed; tail -20 gpurun_out/prof_$TAG.err; exit 1; }
python3 scripts/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv 199
fi
