#!/usr/bin/env bash
# Round-6 final measurement set, part 1 (through gpurun): GPU suite + smoke, the driver's default
# bench line, the pems / n2048 lines, one-step kernel traces of METR and PEMS, and a rocprofv3
# kernel-stats pass of the driver's exact bench command.  Part 2: tools/gpu.sh <out> pmc:metr pmc:pems.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-r6final}
bash tools/gpu.sh $O suite bench:default bench:pems bench:n2048 stats:metr stats:pems || exit 1
mkdir -p gpurun_out/$O/defcmd
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$O/defcmd -o run -- \
  python bench.py > gpurun_out/$O/default_cmd_bench.json 2> gpurun_out/$O/default_cmd.err || { tail -20 gpurun_out/$O/default_cmd.err; exit 1; }
echo "default cmd done"
