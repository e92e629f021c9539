set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${1:-prof}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT -o run -- python3 -u bench.py --warmup 300 --steps 50 --no-cpu > gpurun_out/$OUT.log 2> gpurun_out/$OUT.err
echo "prof rc=$?"
tail -1 gpurun_out/$OUT.log
