#!/bin/bash
# HBM traffic and SQ counters of k_step on the bench's secondary lattices (run through gpurun):
#   tools/pmc_lattices.sh <tag> <cases> [lib-dir]   e.g. tools/pmc_lattices.sh r03e c3,c4x4,coronary
# Each case is stepped by tools/ab_lattices.py --child (20 warm-up + timed + 200 profiled steps).
# Passes per case, each its own rocprofv3 run: kernel trace; FETCH_SIZE; WRITE_SIZE; SQ counters.
# -> gpurun_out/pmcl_<tag>/<case>/{kt,fetch,write,sq}/  (summarise: tools/pmc_lattices.py)
set -euo pipefail
tag=$1
cases=$2
lib=${3:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
if [ -n "$lib" ]; then export LBM_LIBRARY=$R/$lib/liblbm.so; fi
cd /tmp
SQ=SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY
for c in ${cases//,/ }; do
  out=$R/gpurun_out/pmcl_$tag/$c
  mkdir -p "$out"
  P="python3 $R/tools/ab_lattices.py --child $c"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- $P > "$out/kt.json" 2> "$out/kt.log"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- $P > /dev/null 2> "$out/fetch.log"
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o write -- $P > /dev/null 2> "$out/write.log"
  timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d "$out/sq" -o sq -- $P > /dev/null 2> "$out/sq.log"
  echo "$c done"
done
