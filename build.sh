#!/usr/bin/env bash
# Build libgwn.so (HIP, gfx950) in-tree.  Used by __graft_entry__.build() and by hand.
#   OUT=<path> EXTRA="-DFOO=1" ./build.sh    builds an experiment variant elsewhere
# Each source compiles to its own object in parallel (JOBS, default 8), then one link.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")" && pwd)"
SRC="$ROOT/graph-wavenet_amd/csrc"
OUT="${OUT:-$ROOT/graph-wavenet_amd/gwn_amd/libgwn.so}"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result ${EXTRA:-} -I$ROOT/include"
OBJ="$(mktemp -d)"
trap 'rm -rf "$OBJ"' EXIT
pids=()
for f in gemm gemm_nt ops gcn_fused gcn_slice supports rowgemm gram wgrad wgrad_group infer bigdiff; do
  "$HIPCC" $FLAGS -c -o "$OBJ/$f.o" "$SRC/$f.hip" &
  pids+=($!)
  while [ "$(jobs -rp | wc -l)" -ge "${JOBS:-8}" ]; do sleep 0.2; done
done
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" --offload-arch=gfx950 -shared -fPIC -o "$OUT.tmp" "$OBJ"/*.o
mv "$OUT.tmp" "$OUT"
echo "built $OUT"
