#!/usr/bin/env python3
"""Does the C2 fused eigensolver's G.S product speed up when the batch's
Grams fit the XCDs' L2?  Runs the C2 job (T=600 N=130 B=999, the
bench_configs.py c2 workload) with the device batch capped (DFM_NO_LANES=1
and model.set_batch(nb)): a fused launch then holds nb one-workgroup
replicates, nb / 8 per XCD, nb / 8 x 135 KB of Grams per 4 MB L2.  Run with
DFM_EIG_PROF=1: the library prints replicate 0's phase split of every fused
solve (gq = the Y = G Q products, cheb = the filter products) to stderr.

    DFM_NO_LANES=1 DFM_EIG_PROF=1 python tools/c2_l2_probe.py 999 240 160 80"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import dfm_pkg
    D = dfm_pkg.load()
    ctx = D.Context(0)
    T, N, B, bp = 600, 130, 999, 300
    y, x, *_ = D.factor_model_DGP(T, N, 3, model="Breitung_Eickmeier_2011", b=0.5,
                                  rng=np.random.default_rng(20261015 + 2))
    x = D.normalize(x, ctx=ctx)
    w = np.ones((T, 1))
    model = D.DynamicFactorModel(y, w, x, "ICp2", kmax=8, ctx=ctx)
    S = D.Stat
    stats = [S.V(), S.criterion(), S.LR_all(bp), S.LM_all(bp), S.Wald_all(bp)]
    arr = D.api._stat_array(stats)
    width = int(ctx.lib.dfm_stats_width(model.handle, arr, len(stats)))
    idx, eta = D.draw_wild_fast(7, B, T)
    dev = torch.device("cuda", 0)
    di, de = torch.from_numpy(idx).to(dev), torch.from_numpy(eta).to(dev)
    out = torch.empty((B, width), dtype=torch.float64, device=dev)
    ref = None
    for nb in [int(a) for a in sys.argv[1:]] or [999, 160]:
        model.set_batch(nb)

        def run():
            ctx.check(ctx.lib.dfm_bootstrap_dev(model.handle, 0, B, di.data_ptr(), de.data_ptr(), arr, len(stats),
                                                out.data_ptr()))
        run()
        ctx.synchronize()
        ctx.reset_timing()
        ctx.enable_timing(True)
        t0 = time.perf_counter()
        for _ in range(3):
            run()
        ctx.synchronize()
        el = (time.perf_counter() - t0) / 3
        ctx.enable_timing(False)
        tm = ctx.read_timing()
        rows = out.cpu().numpy()
        same = ref is None or bool(np.array_equal(rows, ref))
        ref = rows if ref is None else ref
        print(f"batch {nb}: {el * 1e3:.3f} ms per job, eig class {tm.get('eig_gq', (0, 0))[0] / 3:.3f} ms per job, "
              f"rows equal to the first batch size: {same}", flush=True)
        sys.stderr.write(f"== batch {nb} done\n")


if __name__ == "__main__":
    main()
