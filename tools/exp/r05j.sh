set -e
mkdir -p gpurun_out/r05j
AB_CASES=c3 timeout -k 10 500 python3 -u tools/ab_lattices.py 3 product tools/ab/rec_nosub tools/ab/rec_noprod tools/ab/rec_nowait tools/ab/no_nee@12:1 > gpurun_out/r05j/rec_parts.log 2>&1
LBM_LIBRARY=$PWD/tools/ab/wave_ts/liblbm.so timeout -k 10 300 python3 -u tools/wave_ts_lab.py c3 ldc256 > gpurun_out/r05j/wave_ts.log 2>&1
