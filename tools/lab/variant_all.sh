#!/bin/bash
# full-library lab variant: every source rebuilt with extra -D flags
set -e
NAME=$1; DEFS=$2
R=/root/repo/leak-det-gnn_amd
mkdir -p "$R/lib/$NAME"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$R/../include" -Wno-unused-function $DEFS -shared $R/csrc/*.hip -o "$R/lib/$NAME/libleakgnn.so"
echo "$R/lib/$NAME/libleakgnn.so"
