#!/bin/bash
# Same-box A/B of kernel-lab libraries: kbench.py with each library in turn, REPS rounds.
#   bash tools/lab/ab.sh <out> "<kbench args>" <reps> base|<libname> ...
# base = the product library; <libname> = leak-det-gnn_amd/lib/<libname>/libleakgnn.so
set -o pipefail
OUT=$1; ARGS=$2; REPS=$3; shift 3
mkdir -p "$(dirname "$OUT")"
export TMPDIR=/tmp
for r in $(seq 1 "$REPS"); do
  for v in "$@"; do
    if [[ $v == base ]]; then unset LEAKGNN_LIB; else export LEAKGNN_LIB=$PWD/leak-det-gnn_amd/lib/$v/libleakgnn.so; fi
    echo "== $v round $r" >> "$OUT"
    timeout -k 10 120 python tools/kbench.py $ARGS >> "$OUT" 2>&1 || { echo "kbench failed ($v)"; tail -5 "$OUT"; exit 1; }
  done
done
unset LEAKGNN_LIB
python3 - "$OUT" <<'PY'
import sys, json, re, collections
cur=None; acc=collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1]):
    m=re.match(r"== (\S+) round", line)
    if m: cur=m.group(1); continue
    parts=line.strip().split(" ",1)
    if len(parts)==2 and parts[1].startswith("{"):
        try: v=json.loads(parts[1])
        except Exception: continue
        if "us" in v: acc[parts[0]][cur].append(round(v["us"],2))
for k,vs in acc.items():
    print(k, {v: sorted(x) for v,x in vs.items()})
PY
