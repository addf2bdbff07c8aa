set -e
mkdir -p gpurun_out/r05r
AB_CASES=ldc256,c3 timeout -k 10 400 python3 -u tools/ab_alloc.py 4 0 2 > gpurun_out/r05r/alloc_pair.log 2>&1
AB_CASES=ldc256 timeout -k 10 400 python3 -u tools/ab_lattices.py 4 product product@4:2 > gpurun_out/r05r/pair_ab.log 2>&1
AB_CASES=c4x4 timeout -k 10 300 python3 -u tools/ab_lattices.py 3 product product@9:16 product@9:32 > gpurun_out/r05r/seg_ab.log 2>&1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05r/tests.txt 2>&1
