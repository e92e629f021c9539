set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${1:-prof}
WARM=${2:-300}
STEPS=${3:-50}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT -o run -- python3 -u bench.py --warmup $WARM --steps $STEPS --no-cpu > gpurun_out/$OUT.log 2> gpurun_out/$OUT.err
echo "rc=$?"
tail -2 gpurun_out/$OUT.log
find gpurun_out/$OUT -name "*stats*" | head
