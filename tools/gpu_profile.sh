#!/bin/bash
# Kernel-trace and HBM-traffic profiles of bench.py on one MI355X (run through gpurun).
#   tools/gpu_profile.sh <tag>
# -> gpurun_out/prof_<tag>/{kt,fetch,write}/...  (rocprofv3 CSVs), summarised by
#    tools/pmc_traffic.py into profiles/.
set -euo pipefail
tag=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
out=$R/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- python3 $B > "$out/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- python3 $B > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o write -- python3 $B > "$out/write.log" 2>&1
echo done
