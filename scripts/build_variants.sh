# Build experiment variants of libfdbcs.so: scripts/build_variants.sh name:"-DFLAG ..." ...
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/micro/var
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  FDBCS_EXTRA_FLAGS="$flags" FDBCS_OBJ_DIR=obj_$name FDBCS_LIB_OUT=$PWD/scripts/micro/var/libfdbcs_$name.so \
    python -c "from foundationdb_amd import build; print(build.build_hip())"
done
