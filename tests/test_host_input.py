"""Host input layer: lag builders, row/vector normalisers and
the CSV panel loader of the reference's own test (test/DynamicFactorModel.jl:6-20,
src/utils.jl:5-51) — CPU only."""
import os

import numpy as np
import pytest


@pytest.fixture(scope="module")
def host(dfm_host):
    return dfm_host


@pytest.fixture(scope="module")
def dfm_host():
    import dfm_pkg
    import importlib
    dfm_pkg.load()
    return importlib.import_module("dfm_amd.host")


def test_lag_vector_and_matrix(host):
    v = np.array([1.0, 2.0, 3.0, 4.0])
    l1 = host.lag_vector(v)
    assert list(np.ma.getmaskarray(l1)) == [True, False, False, False]
    assert list(np.ma.getdata(l1)[1:]) == [1.0, 2.0, 3.0]
    l2 = host.lag_vector(l1)          # the DataArray method keeps the NA shifting
    assert list(np.ma.getmaskarray(l2)) == [True, True, False, False]
    assert list(np.ma.getdata(l2)[2:]) == [1.0, 2.0]
    m = host.lag_matrix(np.arange(12.0).reshape(4, 3))
    assert m.shape == (4, 3) and np.all(np.ma.getmaskarray(m)[0])
    assert np.array_equal(np.ma.getdata(m)[1:], np.arange(9.0).reshape(3, 3))


def test_norms_and_possemidef(host):
    rng = np.random.default_rng(1)
    a = rng.standard_normal((5, 3))
    assert np.allclose(np.linalg.norm(host.norm_matrix(a), axis=1), 1.0)
    assert np.isclose(np.linalg.norm(host.norm_vector(a[:, 0])), 1.0)
    assert host.possemidef(a.T @ a) and not host.possemidef(-np.eye(3))


def test_csv_and_reference_test_design(host, tmp_path):
    rng = np.random.default_rng(2)
    T, N = 30, 6
    data = rng.standard_normal((T, N + 1))
    p = tmp_path / "panel.csv"
    with open(p, "w") as fh:
        fh.write("sasdate," + ",".join(f"S{i}" for i in range(N + 1)) + "\n")
        for t in range(T):
            fh.write(f"{t + 1}/1/1959," + ",".join(repr(float(v)) for v in data[t]) + "\n")
    names, d = host.read_panel_csv(str(p))
    assert names == [f"S{i}" for i in range(N + 1)] and np.array_equal(d, data)
    y, w, x = host.reference_test_design(d, 4)
    assert y.shape == (T - 4,) and w.shape == (T - 4, 5) and x.shape == (T - 4, N)
    assert np.array_equal(y, data[4:, 0]) and np.array_equal(x, data[4:, 1:])
    assert np.all(w[:, 0] == 1.0)
    for k in range(1, 5):
        assert np.array_equal(w[:, k], data[4 - k:T - k, 0])
    with open(p, "a") as fh:
        fh.write("x/1/2000," + ",".join(["NA"] * (N + 1)) + "\n")
    with pytest.raises(ValueError):
        host.read_panel_csv(str(p))
