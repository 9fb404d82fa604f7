#!/bin/bash
# Kernel-lab variant library: ONE source file rebuilt with extra -D flags, linked with the
# product objects.  Usage: tools/lab/variant_file.sh <name> <file stem> "<defines>"
set -e
NAME=$1; STEM=$2; DEFS=$3
R=$(cd "$(dirname "$0")/../.." && pwd)/leak-det-gnn_amd
make -s -C "$R" >/dev/null
mkdir -p "$R/build/$NAME" "$R/lib/$NAME"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/../include" -Wall -Wno-unused-function $DEFS \
  -c "$R/csrc/$STEM.hip" -o "$R/build/$NAME/$STEM.o"
OBJS=$(ls "$R"/build/*.o | grep -v "/$STEM.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS "$R/build/$NAME/$STEM.o" -o "$R/lib/$NAME/libleakgnn.so"
echo "$R/lib/$NAME/libleakgnn.so"
