# round 5: the host-side threading of libdfm under ASan + UBSan and under TSan
# (csrc Makefile `san` / `tsan`; tests/c_harness/dfm_threads.c; reports of the
# TSan run filtered to libdfm's own code by tools/tsan_filter.py)
mkdir -p gpurun_out/san
export LD_LIBRARY_PATH=/opt/rocm/lib/llvm/lib/clang/22/lib/linux${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}
ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  timeout -k 10 300 tests/c_harness/dfm_threads_san > gpurun_out/san/asan.txt 2>&1; echo asan_rc=$?
grep -c "ERROR: AddressSanitizer\|runtime error" gpurun_out/san/asan.txt; tail -3 gpurun_out/san/asan.txt
TSAN_OPTIONS=halt_on_error=0:second_deadlock_stack=1 \
  timeout -k 10 400 tests/c_harness/dfm_threads_tsan > gpurun_out/san/tsan.txt 2>&1; echo tsan_rc=$?
grep "dfm_threads OK" gpurun_out/san/tsan.txt; python3 tools/tsan_filter.py gpurun_out/san/tsan.txt
