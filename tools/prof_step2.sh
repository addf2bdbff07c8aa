export TMPDIR=/tmp
mkdir -p gpurun_out/p2
P="timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv"
$P -d gpurun_out/p2/kt -o kt -- python3 tools/prof_step2.py 512 2 8 > gpurun_out/p2/kt.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/p2/c1 -o c1 -- python3 tools/prof_step2.py 512 2 8 > gpurun_out/p2/c1.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum TCC_MISS_sum -d gpurun_out/p2/c2 -o c2 -- python3 tools/prof_step2.py 512 2 8 > gpurun_out/p2/c2.log 2>&1 || exit 3
timeout -s KILL 90 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/p2/c3 -o c3 -- python3 tools/prof_step2.py 512 2 8 > gpurun_out/p2/c3.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/p2/c4 -o c4 -- python3 tools/prof_step2.py 512 2 8 > gpurun_out/p2/c4.log 2>&1 || exit 5
