# round 5: the two-lane defect — clone tests on the round-4 library and on the fixed one; RCCL world-1 tests
mkdir -p gpurun_out/fx2
DFM_LIB_PATH=variants/r04/libdfm.so timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -k "clone" -v --timeout 120 --timeout-method thread > gpurun_out/fx2/unfixed.txt 2>&1; echo unfixed_rc=$?
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py -v --timeout 150 --timeout-method thread > gpurun_out/fx2/fixed.txt 2>&1; echo fixed_rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/fx2/unfixed.txt | head -20; grep -E "PASS|FAIL|Error|assert " gpurun_out/fx2/fixed.txt | head -40; tail -3 gpurun_out/fx2/fixed.txt
