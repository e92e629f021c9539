# A/B of detect time (window minus adds) in the bench's Resolver window
# (scripts/micro/resolver_loop, pinned, config 2 at H ~ 19 M) between library
# builds in scripts/micro/var/<name>/libfdbcs.so:
#   bash scripts/micro/ab_detect.sh REPS name...    (GPU box)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
reps=$1; shift
for rep in $(seq $reps); do
  for v in "$@"; do
    LD_LIBRARY_PATH=$PWD/scripts/micro/var/$v timeout -k 10 120 python scripts/micro/pinned.py \
      ./scripts/micro/resolver_loop 2500 150 2 0 > gpurun_out/abd.log 2>&1 || { echo "$v failed"; cat gpurun_out/abd.log; exit 1; }
    python3 -c "
import re
for l in open('gpurun_out/abd.log'):
    m = re.match(r'rep (\d): ([\d.]+) us per batch, add ([\d.]+) us', l)
    if m and m.group(1) != '0':
        w, a = float(m.group(2)), float(m.group(3))
        print('$v', 'window %.1f add %.1f detect %.1f' % (w, a, w - a))"
  done
done
