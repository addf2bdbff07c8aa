#!/bin/bash
# One GPU session through gpurun (replaces the round-5 one-off recipes under tools/exp/):
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_run.sh <tag> <step>[,<step>...]
# Steps, in the order given; each under its own time limit, and the session stops at the first
# step that fails (a GPU fault, abort, segfault or time limit ends it: nothing more runs):
#   tests      pytest -m gpu (TEST_PATHS="tests/a.py tests/b.py::test_x" narrows it) -> <tag>/tests.txt
#   smoke      __graft_entry__.smoke()                              -> <tag>/smoke.txt
#   bench      python bench.py $BENCH_ARGS (default: the driver's)  -> <tag>/bench.json
#   spread     BENCH_RUNS fresh headline-only bench processes       -> <tag>/bench_spread.jsonl
#   prof       tools/gpu_profile.sh <tag>: kernel trace + FETCH_SIZE / WRITE_SIZE of the 512^3 bench
#   lattices   tools/pmc_lattices.sh <tag> $LATTICES (default c3,c4,c4x4,coronary,ldc64,ldc256,c5)
#   ab         tools/ab_lattices.py $AB_ARGS (AB_CASES selects lattices)  -> <tag>/ab.log
# Output under gpurun_out/ (merged back by gpurun).
set -uo pipefail
tag=$1
steps=$2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
cd "$R"
run() {  # run <seconds> <log> <cmd...>
  local lim=$1 log=$2
  shift 2
  echo "[gpu_run] $(date +%T) $*" | tee -a "$out/steps.log"
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  echo "[gpu_run] $(date +%T) rc=$rc" | tee -a "$out/steps.log"
  if [ $rc -ne 0 ]; then tail -30 "$log"; exit $rc; fi
}
for s in ${steps//,/ }; do
  case $s in
    tests) run 900 "$out/tests.txt" python3 -u -m pytest ${TEST_PATHS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) run 300 "$out/smoke.txt" python3 -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 900 "$out/bench.json" python3 -u bench.py ${BENCH_ARGS:-} ;;
    spread)
      for i in $(seq 1 "${BENCH_RUNS:-3}"); do
        run 300 "$out/bench_spread_$i.json" python3 -u bench.py --steps 50 --warmup 10 --no-secondary --no-cpu-baseline
        tail -1 "$out/bench_spread_$i.json" >> "$out/bench_spread.jsonl"
      done ;;
    prof) run 1000 "$out/gpu_profile.log" bash tools/gpu_profile.sh "$tag" ;;
    lattices) run 1100 "$out/pmc_lattices.log" bash tools/pmc_lattices.sh "$tag" "${LATTICES:-c3,c4,c4x4,coronary,ldc64,ldc256,c5}" ;;
    ab) run 1100 "$out/ab.log" python3 -u tools/ab_lattices.py ${AB_ARGS} ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "[gpu_run] done" | tee -a "$out/steps.log"
