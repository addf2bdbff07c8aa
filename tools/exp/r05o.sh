set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05o
for v in prod prev xcd1 prod2 prev2; do
  case $v in
    prod|prod2) unset LBM_LIBRARY; export AB_TUNE= ;;
    prev|prev2) export LBM_LIBRARY=$PWD/tools/ab/prev_head/liblbm.so; export AB_TUNE= ;;
    xcd1) unset LBM_LIBRARY; export AB_TUNE=13:1 ;;
  esac
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05o/$v -o run -- python3 tools/ab_lattices.py --child c3 > gpurun_out/r05o/$v.log 2>&1
done
