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
