#!/bin/bash
# Kernel time and HBM read traffic of liblbm variants at 512^3 (run through gpurun):
#   tools/ab_profile.sh <tag> <lib-dir>...   (each dir holds a liblbm.so; "product" = the in-tree one)
# -> gpurun_out/ab_<tag>/<variant>/{kt,fetch}/ + bench lines in <variant>.json
set -euo pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline"
for v in "$@"; do
  name=$(basename "$v")
  out=$R/gpurun_out/ab_$tag/$name
  mkdir -p "$out"
  if [ "$v" = product ]; then unset LBM_LIBRARY; else export LBM_LIBRARY=$R/$v/liblbm.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- python3 $B > "$out.json" 2> "$out/kt.log"
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- python3 $B > /dev/null 2> "$out/fetch.log"
done
echo done
