set -e
mkdir -p gpurun_out/r05s
AB_CASES=ldc256 timeout -k 10 300 python3 -u tools/ab_alloc.py 4 0 2 > gpurun_out/r05s/alloc_pair.log 2>&1
AB_CASES=ldc256 timeout -k 10 400 python3 -u tools/ab_lattices.py 4 product product@4:2 > gpurun_out/r05s/pair_ab.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in a b; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05s/kt_$v -o kt -- python3 tools/ab_lattices.py --child ldc256 > gpurun_out/r05s/kt_$v.json 2> gpurun_out/r05s/kt_$v.log
done
AB_CASES=ldc512 timeout -k 10 600 python3 -u tools/ab_lattices.py 3 product tools/ab/budget160 > gpurun_out/r05s/budget_ab.log 2>&1
