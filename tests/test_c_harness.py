"""The C ABI from plain C: tests/c_harness/dfm_harness.c makes the Julia
shim's calls through include/dfm.h alone, so header / ABI
drift is caught independently of the Python ctypes table.

CPU: the harness compiles as strict C99 against the header (-Wall -Wextra
-Werror -pedantic), links every call against libdfm.so, and without a GPU
exits 3 after a clean dfm_ctx_create failure.  GPU: its results equal the
Python binding's bit for bit (same library, same inputs) and the oracle's
within the north-star tolerances."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c_harness", "dfm_harness.c")
LIBDIR = os.path.join(ROOT, "dynamicfactormodels.jl_amd")
BIN = os.path.join(ROOT, "tests", "c_harness", "dfm_harness")


def build_harness(dst=BIN):
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    subprocess.run([cc, "-std=c99", "-O1", "-Wall", "-Wextra", "-Werror", "-pedantic",
                    "-I", os.path.join(ROOT, "include"), SRC, "-L", LIBDIR, "-ldfm",
                    f"-Wl,-rpath,{LIBDIR}", "-o", dst], check=True)
    return dst


def write_input(path, T, N, B, seed):
    rng = np.random.default_rng(seed)
    y = rng.standard_normal(T)
    f = rng.standard_normal((T, 3))
    X = f @ rng.standard_normal((3, N)) + rng.standard_normal((T, N))
    X = (X - X.mean(0)) / X.std(0, ddof=1)
    idx = rng.integers(0, T, size=(B, T), dtype=np.int32)
    eta = rng.standard_normal((B, T))
    with open(path, "wb") as fh:
        np.array([T, N, B], dtype="<i8").tofile(fh)
        y.astype("<f8").tofile(fh)
        np.asfortranarray(X).ravel(order="F").astype("<f8").tofile(fh)
        idx.astype("<i4").tofile(fh)
        eta.astype("<f8").tofile(fh)
    return y, X, idx, eta


def read_output(path):
    out = {}
    for line in open(path):
        parts = line.split()
        out[parts[0]] = np.array([float(v) for v in parts[1:]])
    return out


def test_harness_compiles_as_c99_and_fails_cleanly_without_gpu(tmp_path):
    import torch
    binp = build_harness(str(tmp_path / "h"))
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present: the gpu test runs the harness")
    write_input(tmp_path / "in.bin", 20, 30, 2, 0)
    rc = subprocess.run([binp, str(tmp_path / "in.bin"), str(tmp_path / "out.txt")]).returncode
    assert rc == 3
    assert open(tmp_path / "out.txt").read().strip() == "NO_GPU"


@pytest.mark.gpu
def test_harness_matches_python_binding_and_oracle(dfm, oracle, tmp_path):
    binp = BIN if os.path.exists(BIN) else build_harness(str(tmp_path / "h"))
    T, N, B = 96, 150, 6
    y, X, idx, eta = write_input(tmp_path / "in.bin", T, N, B, 11)
    p = subprocess.run([binp, str(tmp_path / "in.bin"), str(tmp_path / "out.txt")], capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    h = read_output(tmp_path / "out.txt")
    w = np.ones((T, 1))
    g = dfm.DynamicFactorModel(y, w, X, "ICp2", kmax=8)
    r = g.number_of_factors
    assert h["fit_scalars"][0] == r and h["fit_scalars"][1] == g.V
    assert np.array_equal(h["fit_coef"], g.coefficients) and np.array_equal(h["fit_ic"], g.ic_values.ravel())
    o = oracle.DynamicFactorModel_ic(y, w, X, "ICp2", kmax=8)
    assert o.number_of_factors == r
    assert abs(h["fit_scalars"][2] - o.number_of_factors_criterion_value) < 1e-10 * abs(
        o.number_of_factors_criterion_value)
    S = dfm.Stat
    stats = [S.V(), S.criterion(), S.LR_all(T // 2)]
    wild = dfm.wild_bootstrap(g, B, stats, idx=idx, eta=eta)
    assert np.array_equal(h["wild"].reshape(B, -1), wild)
    assert np.array_equal(h["wild_multi"], h["wild"])               # 2-context shards, bit-identical
    fl = dfm.wild_bootstrap(g, B, [S.factors(), S.loadings(1)], idx=idx, eta=eta)
    assert fl.shape == (B, (T + N) * r) and np.array_equal(h["wild_factors_loadings"].reshape(B, -1), fl)
    assert np.array_equal(h["lasso_stats"], np.zeros(len(dfm._lib.LASSO_STATS)))
    assert np.array_equal(h["residual_V"], dfm.residual_bootstrap(g, B, S.V(), idx=idx))
    for b in range(2):
        d = oracle.DynamicFactorModel(y, w, o.common_component + eta[b][:, None] * o.factor_residuals[idx[b]],
                                      r, "ICp2")
        assert abs(wild[b, 0] - oracle.factor_residual_variance(d)) < 1e-10 * oracle.factor_residual_variance(d)
    LR, LM, W = dfm.chow_all(g, T // 2)
    assert np.array_equal(h["chow_LR"], LR) and np.array_equal(h["chow_LM"], LM) and np.array_equal(h["chow_Wald"], W)
    bo = oracle.DynamicFactorModel(y, w, X, 2, "BIC", [T // 2 + 1])
    ref = np.array([oracle.LR_test(bo, T // 2 + 1, i) for i in range(10)])
    assert np.max(np.abs(h["break_chow_LR"][:10] - ref) / np.abs(ref)) < 1e-10
    assert np.max(np.abs(h["normalize_col0"] - oracle.normalize(X)[:, 0])) < 1e-13 * 10
    tx, _ = oracle.targeted_predictors_hard(y, w, X, "per_candidate")
    assert np.max(np.abs(h["tp_hard_t"] - tx) / np.abs(tx)) < 1e-10
    pred, true = dfm.pseudo_out_of_sample_forecasts(dfm.DynamicFactorModel, y, w, X, "ICp2", num_predictions=4,
                                                    kmax=4)
    assert np.array_equal(h["windows_pred"], pred)
    assert h["error_rc"][0] < 0 and h["error_msg_nonempty"][0] == 1
    # predict / get_factors / per-variable Chow / model criteria on rows 0..T-3
    gp = dfm.DynamicFactorModel(y[:T - 2], w[:T - 2], X[:T - 2], 3, "ICp2")
    assert np.array_equal(h["predict"], dfm.predict(gp, w[T - 2:], X[T - 2:]))
    assert np.array_equal(h["get_factors"], dfm.get_factors(gp, X[T - 2:]).ravel(order="F"))
    op = oracle.DynamicFactorModel(y[:T - 2], w[:T - 2], X[:T - 2], 3, "ICp2")
    po = oracle.predict(op, w[T - 2:], X[T - 2:])
    assert np.max(np.abs(h["predict"] - po)) <= 1e-10 * np.max(np.abs(po))
    bp = (T - 2) // 2
    assert h["chow_one"][0] == dfm.LR_test(gp, bp, 5)
    assert abs(h["chow_one"][2] - oracle.Wald_test(op, bp, 4)) <= 1e-10 * abs(oracle.Wald_test(op, bp, 4))
    for c, name in enumerate(dfm.CRITERIA):
        ref = oracle.criterion_value(name, op)
        assert abs(h["model_criteria"][c] - ref) <= 1e-10 * abs(ref), name
    # rolling windows, workhorse r = 2 with BIC
    res = dfm.pseudo_out_of_sample_windows(y, w, X, 2, "BIC", num_predictions=4, rolling=T // 2, forecast=True)
    assert np.array_equal(h["rolling_r"], res["number_of_factors"])
    assert np.array_equal(h["rolling_V"], res["V"]) and np.array_equal(h["rolling_pred"], res["predictions"])
    ro, _, _ = oracle.rolling_window_forecasts(lambda yy, ww, xx: oracle.DynamicFactorModel(yy, ww, xx, 2, "BIC"),
                                               y, w, X, 4, T // 2)
    assert np.max(np.abs(h["rolling_pred"] - ro)) <= 1e-10 * np.max(np.abs(ro))
