# A/B of the adds alone (scripts/micro/resolver_loop, pinned) between library
# builds in scripts/micro/var/<name>/libfdbcs.so:
#   bash scripts/micro/ab_adds.sh CONFIG name...    (GPU box)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cfg=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    for args in "300 40 $cfg 1" "300 40 $cfg 1 1"; do
      LD_LIBRARY_PATH=$PWD/scripts/micro/var/$v timeout -k 10 120 python scripts/micro/pinned.py \
        ./scripts/micro/resolver_loop $args > gpurun_out/aba.log 2>&1 || { echo "$v $args failed"; cat gpurun_out/aba.log; exit 1; }
      echo "c$cfg $v [$args]: $(tail -1 gpurun_out/aba.log)"
    done
  done
done
