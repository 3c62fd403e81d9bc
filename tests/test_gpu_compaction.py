"""The factored bootstrap's straggler phase (once a poll finds < 1/8 of the
batch active, the H.Z GEMMs tile only the listed stragglers' column groups,
dfm_eig.hip active_list_kernel + launch_gemm clist) must not change a single
bit of any replicate's statistics: the same C3-shaped job is run here with
compaction on (the default) and in a child process with DFM_GEMM_COMPACT=0
(the switch is read once per process)."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys
    import numpy as np
    sys.path.insert(0, {root!r})
    sys.path.insert(0, {oracle!r})
    import dfm_pkg
    import dfm_oracle as O
    D = dfm_pkg.load()
    rng = np.random.default_rng(3003)
    y, x, *_ = O.factor_model_DGP(500, 2000, 8, rng)
    x = O.normalize(x)
    w = np.ones((500, 1))
    g = D.DynamicFactorModel(y, w, x, 8, "ICp2")
    idx, eta = D.draw_wild_fast(11, 512, 500)
    out = D.wild_bootstrap(g, 512, [D.Stat.V(), D.Stat.criterion(), D.Stat.t_stat(2)], idx=idx, eta=eta)
    np.save({path!r}, out)
""")


def test_straggler_compaction_is_bit_identical(dfm, oracle, tmp_path):
    rng = np.random.default_rng(3003)
    y, x, *_ = oracle.factor_model_DGP(500, 2000, 8, rng)
    x = oracle.normalize(x)
    w = np.ones((500, 1))
    g = dfm.DynamicFactorModel(y, w, x, 8, "ICp2")
    idx, eta = dfm.draw_wild_fast(11, 512, 500)
    stats = [dfm.Stat.V(), dfm.Stat.criterion(), dfm.Stat.t_stat(2)]
    on = dfm.wild_bootstrap(g, 512, stats, idx=idx, eta=eta)
    path = str(tmp_path / "off.npy")
    env = dict(os.environ, DFM_GEMM_COMPACT="0")
    code = CHILD.format(root=ROOT, oracle=os.path.join(ROOT, "oracle"), path=path)
    subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=300)
    off = np.load(path)
    assert np.all(np.isfinite(on))
    assert np.array_equal(on, off)
