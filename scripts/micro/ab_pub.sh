cd $GRAFT_REPO_ROOT
for rep in 1 2; do for p in 16 8 32; do
  FDBCS_LIVE_PUB=$p timeout -k 10 120 python scripts/micro/pinned.py ./scripts/micro/resolver_loop 2500 150 2 0 > gpurun_out/pub.log 2>&1 || { cat gpurun_out/pub.log; exit 1; }
  python3 -c "
import re
for l in open('gpurun_out/pub.log'):
    m = re.match(r'rep (\d): ([\d.]+) us per batch, add ([\d.]+) us', l)
    if m and m.group(1) != '0':
        w, a = float(m.group(2)), float(m.group(3)); print('pub $p window %.1f add %.1f detect %.1f' % (w, a, w - a))"
done; done
