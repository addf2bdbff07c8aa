set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05p
for v in prod prev prodx prevx prod2 prev2 prodx2 prevx2; do
  case $v in
    prod*) unset LBM_LIBRARY ;;
    prev*) export LBM_LIBRARY=$PWD/tools/ab/prev_head/liblbm.so ;;
  esac
  case $v in *x*) export AB_TUNE=13:1 ;; *) export AB_TUNE= ;; esac
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05p/$v -o run -- python3 tools/ab_lattices.py --child c3,c4x4 > gpurun_out/r05p/$v.log 2>&1
done
