# GPU parity tests only (optionally one file): bash scripts/gpu_tests.sh TAG [pytest args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-t}; shift
timeout -k 10 500 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests_$TAG.log | tail -40
exit $rc
