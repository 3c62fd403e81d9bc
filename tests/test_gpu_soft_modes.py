"""The lasso path kernel's coordinate-descent forms for active sets past the
LDS cache (dfm_soft.hip lasso_path_kernel: DFM_SOFT_CD=0 the default, four
waves with row k+1 of the compacted G_AA prefetched; 1 wave 0 alone; 2 the
thread-0-broadcast form) apply the same updates in the same order, so the
whole CV path must be bit-identical across them.  Run at C4 full size
(T=400, N=5000: the active sets reach several hundred variables) with the
default in this process and each other form in a child process (the switch
is read once per process)."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")

CHILD = textwrap.dedent("""
    import sys
    import numpy as np
    sys.path.insert(0, {root!r})
    sys.path.insert(0, {gold!r})
    import dfm_pkg
    import make_golden
    D = dfm_pkg.load()
    y, w, x, folds = make_golden.c4_inputs()
    mask, path = D.targeted_predictors(y, w, x, "soft", folds=folds, return_path=True)
    np.savez({path!r}, mask=mask, beta=path["beta"], lam=path["lambda"], loss=path["meanloss"])
""")


def run_soft(dfm):
    sys.path.insert(0, GOLD)
    import make_golden
    y, w, x, folds = make_golden.c4_inputs()
    mask, path = dfm.targeted_predictors(y, w, x, "soft", folds=folds, return_path=True)
    return dict(mask=mask, beta=path["beta"], lam=path["lambda"], loss=path["meanloss"])


@pytest.mark.parametrize("mode", ["1", "2"])
def test_soft_cd_forms_bit_identical(dfm, tmp_path, mode):
    ref = run_soft(dfm)
    out = str(tmp_path / f"cd{mode}.npz")
    env = dict(os.environ, DFM_SOFT_CD=mode)
    code = CHILD.format(root=ROOT, gold=GOLD, path=out)
    subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=300)
    got = np.load(out)
    for k in ("mask", "beta", "lam", "loss"):
        assert np.array_equal(ref[k], got[k]), k
