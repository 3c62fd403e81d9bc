# round 5: factored block A/B (DFM_FACT_GUARD = p - k; DFM_FACT_D0 / DFM_FACT_BETA: the warm first filter)
mkdir -p gpurun_out/pab
run() { echo "== $*"; env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-all-fields --steps 10 > gpurun_out/pab/b.json 2>gpurun_out/pab/b.err || { tail -5 gpurun_out/pab/b.err; return 1; }
python - <<'P'
import json; r=json.load(open("gpurun_out/pab/b.json")); e=r["eig_iterations"]
print(r["ms_per_step"], r["value"], "frac", r["roofline"]["frac"], "pz", r["roofline"].get("block_columns"), "rr/rep", round(e["replicate_iterations"]/99990,3), "prod/rep", round(e["gemm_products"]/99990,3), r["kernels_ms"])
P
}
run DFM_FACT_GUARD=8 && run DFM_FACT_GUARD=4 && run DFM_FACT_GUARD=2 && run DFM_FACT_GUARD=2 DFM_FACT_D0=7 DFM_FACT_BETA=0.25 && run DFM_FACT_GUARD=4 DFM_FACT_D0=7 && run DFM_FACT_GUARD=3 DFM_FACT_D0=7 DFM_FACT_BETA=0.25
