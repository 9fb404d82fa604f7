#!/bin/bash
# Kernel-lab variant library: gcn_nm.hip rebuilt with extra -D flags, linked with the
# product objects.  Usage: tools/lab/variant.sh <name> "<defines>"  ->  leak-det-gnn_amd/lib/<name>/libleakgnn.so
set -e
NAME=$1; DEFS=$2
R=$(cd "$(dirname "$0")/../.." && pwd)/leak-det-gnn_amd
make -s -C "$R" >/dev/null
mkdir -p "$R/build/$NAME" "$R/lib/$NAME"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/../include" -Wall -Wno-unused-function $DEFS \
  -c "$R/csrc/gcn_nm.hip" -o "$R/build/$NAME/gcn_nm.o"
OBJS=$(ls "$R"/build/*.o | grep -v "/gcn_nm.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS "$R/build/$NAME/gcn_nm.o" -o "$R/lib/$NAME/libleakgnn.so"
echo "$R/lib/$NAME/libleakgnn.so"
