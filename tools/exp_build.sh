#!/usr/bin/env bash
# Experiment builds of libgwn (never the product): copy csrc, apply a sed script to gcn_fused.hip,
# build into graph-wavenet_amd/gwn_amd/exp/libgwn_<name>.so (git-ignored; select with GWN_LIB).
#   tools/exp_build.sh <name> '<sed expression>'
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name=$1; expr=$2
D=$(mktemp -d)
mkdir -p "$D/g"
cp -r "$ROOT/graph-wavenet_amd/csrc" "$D/g/csrc"
ln -s "$ROOT/include" "$D/include"   # csrc includes ../../include/gwn.h
if [[ "$expr" == *.py ]]; then
  python "$expr" "$D/g/csrc/gcn_fused.hip"   # a transform script edits the copy in place
else
  sed -i -e "$expr" "$D/g/csrc/gcn_fused.hip"
fi
mkdir -p "$ROOT/graph-wavenet_amd/gwn_amd/exp"
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I$ROOT/include"
pids=()
for f in $(cd "$D/g/csrc" && ls *.hip | sed 's/\.hip$//'); do
  fl="$FLAGS"  # as build.sh: no packed fp32 ops in the GCN tile kernels
  case " gcn_fused gcn_slice " in *" $f "*) fl="$FLAGS -Xclang -target-feature -Xclang -packed-fp32-ops" ;; esac
  $HIPCC $fl -c -o "$D/$f.o" "$D/g/csrc/$f.hip" 2>/dev/null & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$ROOT/graph-wavenet_amd/gwn_amd/exp/libgwn_$name.so" "$D"/*.o
rm -rf "$D"
echo "built exp/libgwn_$name.so"
