# rocprofv3 kernel trace + stats of the bench workload (run on the GPU box).
#   bash scripts/profile_kernels.sh OUT [bench args...]
# Summaries: python scripts/prof_summary.py gpurun_out/OUT
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${1:-prof}
shift
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT -o run -- \
  python3 -u bench.py --no-cpu --lm-batches 0 "$@" > gpurun_out/$OUT.log 2> gpurun_out/$OUT.err
rc=$?
echo "rc=$rc"
tail -1 gpurun_out/$OUT.log
exit $rc
