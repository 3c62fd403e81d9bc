# round 5: where chow_all_kernel's wave-cycles go (C2, one lane so the kernel runs solo): two SQ counter passes
OUT=gpurun_out/chpmc
mkdir -p $OUT
export TMPDIR=/tmp
export DFM_NO_LANES=1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM --kernel-include-regex "chow_all" -f csv -d $OUT/p1 -o run -- python3 tools/bench_configs.py --configs c2 --reps 1 > $OUT/p1.out 2> $OUT/p1.err; echo p1=$?
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU --kernel-include-regex "chow_all" -f csv -d $OUT/p2 -o run -- python3 tools/bench_configs.py --configs c2 --reps 1 > $OUT/p2.out 2> $OUT/p2.err; echo p2=$?
find $OUT -name "*counter_collection*" | head
