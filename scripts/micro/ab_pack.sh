# A/B of the add's range packer (stage_pack.h FDBCS_PACK_MODE variants built
# by scripts/build_variants.sh into scripts/micro/var/<name>/libfdbcs.so):
#   bash scripts/micro/ab_pack.sh name...    (GPU box; adds only, pinned)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    for mode in 2 3 1; do
      LD_LIBRARY_PATH=$PWD/scripts/micro/var/$v timeout -k 10 120 python scripts/micro/pinned.py \
        ./scripts/micro/resolver_loop 300 60 2 1 $mode > gpurun_out/abp.log 2>&1 || { echo "$v $mode failed"; cat gpurun_out/abp.log; exit 1; }
      echo "$v mode $mode: $(tail -1 gpurun_out/abp.log)"
    done
  done
done
