# Kernel-trace stats of the Resolver window (resolver_loop, config 2) for
# library builds in scripts/micro/var/<name>/libfdbcs.so (GPU box):
#   bash scripts/micro/kt_ab.sh name...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/kt_ab
for v in "$@"; do
  rm -rf /tmp/kt_$v
  LD_LIBRARY_PATH=$PWD/scripts/micro/var/$v timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d /tmp/kt_$v -o run -- ./scripts/micro/resolver_loop ${PREFILL:-2500} 100 ${CFG:-2} 0 > gpurun_out/kt_ab/$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/kt_ab/$v.log; exit 1; }
  kt=$(find /tmp/kt_$v -name "*kernel_trace.csv" | head -1)
  # (the live batches only: dispatches from the first k_live_ingest on)
  echo "== $v"; python3 -c "
import csv, collections
rows = sorted(csv.DictReader(open('$kt')), key=lambda r: int(r['Start_Timestamp']))
i0 = next(i for i, r in enumerate(rows) if 'k_live_ingest' in r['Kernel_Name'])
d = collections.defaultdict(list)
for r in rows[i0:]:
    d[r['Kernel_Name'].split('(')[0].replace('void ', '').replace('fdbcs_dev::', '')].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:16]:
    print('%-36s %6d calls %9.2f us avg' % (k[:36], len(v), sum(v) / len(v)))"
  rm -rf /tmp/kt_$v
done
