set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 3; }
tail -3 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --warmup 300 --steps 50 --cpu-seconds 5 > gpurun_out/bench_short.log 2> gpurun_out/bench_short.err
echo "bench rc=$?"
tail -3 gpurun_out/bench_short.log; tail -5 gpurun_out/bench_short.err
