"""The factored bootstrap's straggler phase (once a poll finds < 1/8 of the
batch active, the H.Z GEMMs tile only the listed stragglers' column groups,
dfm_eig.hip active_list_kernel + launch_gemm clist) must not change a single
bit of any replicate's statistics.  A C3-shaped 512-replicate job (whose
slowest replicates finish in the compacted phase) is compared with the same
slowest replicates run as a batch of their own, where every one of them is
active at every poll and no column is compacted away."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_straggler_compaction_is_bit_identical(dfm, oracle):
    rng = np.random.default_rng(3003)
    y, x, *_ = oracle.factor_model_DGP(500, 2000, 8, rng)
    x = oracle.normalize(x)
    w = np.ones((500, 1))
    g = dfm.DynamicFactorModel(y, w, x, 8, "ICp2")
    idx, eta = dfm.draw_wild_fast(11, 512, 500)
    stats = [dfm.Stat.V(), dfm.Stat.criterion(), dfm.Stat.t_stat(2), dfm.Stat.iterations()]
    full = dfm.wild_bootstrap(g, 512, stats, idx=idx, eta=eta)
    assert np.all(np.isfinite(full))
    its = full[:, -1]
    slow = np.argsort(-its, kind="stable")[:16]
    assert its[slow[0]] == its.max() and its[slow].min() >= np.median(its)   # the stragglers first
    alone = dfm.wild_bootstrap(g, 16, stats, idx=idx[slow], eta=eta[slow])
    assert np.array_equal(full[slow, :-1], alone[:, :-1])


@pytest.mark.parametrize("r", [10, 12])
def test_factored_iterations_at_r_beyond_8(dfm, oracle, r):
    """at r = 9..12 the factored solver's block (k + 4 <= 16)
    picks the 16-column template while the direct solvers' block (k + 8) is
    wider; the iteration counts (Stat.iterations) must be read from the
    factored solver's own workspace layout, not the direct one's.  The
    counts must be whole steps in [1, maxit] and the statistics must match
    the oracle's refits of the same draws (src/bootstrap.jl:41-51)."""
    T, N, B = 120, 300, 24
    rng = np.random.default_rng(7000 + r)
    y, x, *_ = oracle.factor_model_DGP(T, N, r, rng)
    x = oracle.normalize(x)
    w = np.ones((T, 1))
    g = dfm.DynamicFactorModel(y, w, x, r, "ICp2")
    g.set_bootstrap_mode("factored")
    assert g.fact_block()[0] == r + 4
    idx, eta = dfm.draw_wild_fast(77 + r, B, T)
    stats = [dfm.Stat.V(), dfm.Stat.criterion(), dfm.Stat.iterations()]
    got = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    its = got[:, 2]
    assert np.all(its == np.round(its)) and its.min() >= 1 and its.max() <= 400
    base = oracle.DynamicFactorModel(y, w, x, r, "ICp2")
    for b in (0, B // 2, B - 1):
        d = oracle.DynamicFactorModel(y, w, base.common_component + eta[b][:, None] * base.factor_residuals[idx[b]],
                                      r, "ICp2")
        assert abs(got[b, 0] - oracle.factor_residual_variance(d)) <= 1e-10 * abs(got[b, 0])
        assert abs(got[b, 1] - d.number_of_factors_criterion_value) <= 1e-10 * abs(got[b, 1])
