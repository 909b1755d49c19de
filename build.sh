#!/usr/bin/env bash
# Build libgwn.so (HIP, gfx950) in-tree.  Used by __graft_entry__.build() and by hand.
#   OUT=<path> EXTRA="-DFOO=1" ./build.sh    builds an experiment variant elsewhere
set -euo pipefail
ROOT="$(cd "$(dirname "$0")" && pwd)"
SRC="$ROOT/graph-wavenet_amd/csrc"
OUT="${OUT:-$ROOT/graph-wavenet_amd/gwn_amd/libgwn.so}"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
"$HIPCC" --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result ${EXTRA:-} \
  -I"$ROOT/include" -o "$OUT.tmp" "$SRC/gemm.hip" "$SRC/gemm_nt.hip" "$SRC/ops.hip" "$SRC/gcn_fused.hip" "$SRC/rowgemm.hip" "$SRC/gram.hip" "$SRC/wgrad.hip" "$SRC/infer.hip" "$SRC/bigdiff.hip"
mv "$OUT.tmp" "$OUT"
echo "built $OUT"
