# round 5: fused middle Horner steps — bench A/B (DFM_MID_FUSED), then the factored-path GPU tests
mkdir -p gpurun_out/mid
b() { env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-all-fields --steps 10 > gpurun_out/mid/b.json 2>gpurun_out/mid/b.err || { tail -5 gpurun_out/mid/b.err; return 1; }
python - <<'P'
import json; r=json.load(open("gpurun_out/mid/b.json")); e=r["eig_iterations"]
print(r["ms_per_step"], r["value"], "frac", r["roofline"]["frac"], "mid", r.get("roofline_gemm_mid"), "rr/rep", round(e["replicate_iterations"]/99990,3), "prod", e["gemm_products"], e["gemm_mid_products"], r["kernels_ms"], r["outputs_finite"])
P
}
echo "== fused"; b DFM_MID_FUSED=1 && echo "== separate" && b DFM_MID_FUSED=0 && echo "== fused" && b DFM_MID_FUSED=1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_compaction.py tests/test_gpu_multi.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/mid/pytest.txt 2>&1; echo pytest_rc=$?; tail -3 gpurun_out/mid/pytest.txt
