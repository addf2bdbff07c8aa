set -e
mkdir -p gpurun_out/r05f
export TMPDIR=/tmp
R=$PWD
AB_CASES=ldc256,c3,ldc512 timeout -k 10 500 python3 -u tools/ab_lattices.py 3 tools/ab/xcdrun@13:0 tools/ab/xcdrun@13:5 tools/ab/xcdrun@13:7 tools/ab/xcdrun@13:1 > gpurun_out/r05f/xcd_ab.log 2>&1
for v in "product@" "product@12:1" "tools/ab/no_nee@12:1"; do
  lib=${v%@*}; tune=${v#*@}
  if [ "$lib" = product ]; then unset LBM_LIBRARY; else export LBM_LIBRARY=$R/$lib/liblbm.so; fi
  echo "== $v" >> gpurun_out/r05f/scale.log
  SCALE_ONLY=pipe AB_TUNE=$tune timeout -k 10 200 python3 -u tools/scale_lab.py 1 >> gpurun_out/r05f/scale.log 2>&1
done
unset LBM_LIBRARY
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05f/kt_c3 -o kt -- python3 $R/tools/ab_lattices.py --child c3 > $R/gpurun_out/r05f/kt_c3.log 2>&1
