set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${1:-pmc}
REGEX=${2:-k_sort_tiles}
shift 2
# one counter pass per argument group (comma separated)
i=0
mkdir -p gpurun_out/$OUT
for grp in "$@"; do
  i=$((i+1))
  ctrs=$(echo $grp | tr ',' ' ')
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "$REGEX" --output-format csv -d gpurun_out/$OUT/p$i -o run -- python3 -u bench.py --warmup 50 --steps 10 --no-cpu --stage-timing 0 > gpurun_out/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
