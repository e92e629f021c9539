# Register / LDS / scratch use of kernels in a built object: scripts/kres.sh build/obj/kernels_hist.o [name-regex]
set -e
o=$1; pat=${2:-.}
t=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$t/fb.bin "$o" /dev/null
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$t/fb.bin --output=$t/k.co \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $t/k.co | python3 -c "
import sys,re
txt=sys.stdin.read()
for blk in re.split(r'\n\s+- \.agpr_count', txt)[1:]:
    g=lambda k: (re.search(r'\.'+k+r':\s+(\S+)', blk) or [None,'?'])[1]
    n=g('name')
    if re.search('$pat', n): print(f\"{n:50s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} lds {g('group_segment_fixed_size'):>6} scratch {g('private_segment_fixed_size'):>4}\")
"
rm -rf $t
