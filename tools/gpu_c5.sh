set -o pipefail
mkdir -p gpurun_out/c5 && export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 1 > gpurun_out/c5/bench_c5.json 2> gpurun_out/c5/bench_c5.err && cat gpurun_out/c5/bench_c5.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c5/trace -o run -- python3 bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/c5/trace.json 2> gpurun_out/c5/trace.err &&
timeout -k 10 600 python -u tools/bench_configs.py --cpu > gpurun_out/c5/configs.jsonl 2> gpurun_out/c5/configs.err && cat gpurun_out/c5/configs.jsonl && echo ALLDONE
