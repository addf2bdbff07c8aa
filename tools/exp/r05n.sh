set -e
mkdir -p gpurun_out/r05n
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_checkpoint.py tests/test_gpu_mask.py "tests/test_gpu_parity.py" > gpurun_out/r05n/tests.txt 2>&1
AB_CASES=c3,c4x4,ldc256 timeout -k 10 600 python3 -u tools/ab_lattices.py 3 product tools/ab/prev_head product@13:1 > gpurun_out/r05n/posts_ab.log 2>&1
