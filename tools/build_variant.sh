#!/bin/bash
# usage: build_variant.sh OUTDIR -DFLAGS...  (rebuilds gnn_sparse.hip with flags, links a variant _hip.so)
set -e
out=$1; shift
mkdir -p $out
R=/root/repo
INC="-I$R/cgnn_amd/csrc/include $(python3 -c 'import pybind11,sysconfig;print("-I"+pybind11.get_include(),"-I"+sysconfig.get_paths()["include"])')"
/opt/rocm/bin/hipcc -c -fPIC -std=c++17 -O3 -x hip --offload-arch=gfx950 $INC -Wno-unused-result -fvisibility=hidden "$@" $R/cgnn_amd/csrc/kernels/gnn_sparse.hip -o $out/gnn_sparse.hip.o
objs=$(ls $R/build/hip/*.o | grep -v gnn_sparse.hip.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $out/gnn_sparse.hip.o -o $out/_hip.cpython-310-x86_64-linux-gnu.so
