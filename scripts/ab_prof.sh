# A/B library variants (scripts/build_variants.sh) by kernel time: one
# rocprofv3 --kernel-trace --stats run of the config's bench per variant, then
# the average duration of the named kernels.
#   bash scripts/ab_prof.sh CONFIG "kernel1|kernel2" name...   (run on the GPU box)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg=$1; shift
pat=$1; shift
for v in "$@"; do
  rm -rf gpurun_out/abp_$v
  export FDBCS_LIB_PATH=$PWD/scripts/micro/var/libfdbcs_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abp_$v -o run -- python3 -u bench.py --config $cfg \
    --no-cpu --no-shim --lm-batches 0 --steps ${STEPS:-30} --warmup ${WARMUP:-5} > gpurun_out/abp_${cfg}_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/abp_${cfg}_$v.log; exit 1; }
  f=$(ls gpurun_out/abp_$v/*/run_kernel_stats.csv gpurun_out/abp_$v/run_kernel_stats.csv 2>/dev/null | head -n1)
  python3 - "$f" "$pat" "$v" <<'EOF'
import csv, re, sys
f, pat, v = sys.argv[1:]
for r in csv.DictReader(open(f)):
    if re.search(pat, r["Name"]):
        print(v, r["Name"][11:60], r["Calls"], "avg_us=%.2f" % (float(r["AverageNs"]) / 1e3))
EOF
  rm -rf gpurun_out/abp_$v  # (the traces are large; the summary lines above are what is kept)
done
