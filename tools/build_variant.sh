#!/bin/bash
# usage: build_variant.sh OUTDIR "a.hip b.hip[=/path/to/alt.hip]" -DFLAGS...
#   rebuilds the named kernel sources with extra flags and links a variant _hip.so
#   with the other in-tree objects (A/B in one environment: CGNN_HIP_LIB=OUTDIR/_hip...so);
#   name=path compiles an alternative source file in place of the in-tree one
set -e
out=$1; shift
srcs=$1; shift
mkdir -p $out
R=/root/repo
INC="-I$R/cgnn_amd/csrc/include -I$R/cgnn_amd/csrc/kernels $(python3 -c 'import pybind11,sysconfig;print("-I"+pybind11.get_include(),"-I"+sysconfig.get_paths()["include"])')"
objs=$(ls $R/build/hip/*.o)
bases=""
for spec in $srcs; do
  base=${spec%%=*}
  src=$R/cgnn_amd/csrc/kernels/$base
  [ "$spec" != "$base" ] && src=${spec#*=}
  /opt/rocm/bin/hipcc -c -fPIC -std=c++17 -O3 -x hip --offload-arch=gfx950 $INC -Wno-unused-result -fvisibility=hidden "$@" $src -o $out/$base.o
  objs=$(echo "$objs" | grep -v "/$base.o")
  bases="$bases $base"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $(for b in $bases; do echo $out/$b.o; done) -o $out/_hip.cpython-310-x86_64-linux-gnu.so
