"""dfm_amd — MI355X-native engine for the data-parallel core of
DynamicFactorModels.jl: principal-components factor extraction, the Bai–Ng
IC sweep, the wild/residual bootstrap and the Chow-test replicate loops, and
hard-threshold targeted predictors.

The compute lives in ``libdfm.so`` (HIP, gfx950) behind the C ABI of
``include/dfm.h``; this package is the Python mirror of the reference's
exported Julia API (``src/DynamicFactorModels.jl:16-20``).  Import it through
the repo-root helper ``dfm_pkg.load()`` (the directory name contains a dot).
"""
from .host import (factor_model_DGP, draw_wild, draw_wild_fast, draw_residual,
                   t_quantile, glmnet_default_folds, lag_vector, lag_matrix, norm_vector, norm_matrix,
                   possemidef, read_panel_csv, reference_test_design)
from .api import (Context, DFMError, Stat, DynamicFactorModel, DynamicFactorModelResult,
                  calculate_factors, principal_components, gram_spectrum, calculate_criterion,
                  factor_residual_variance, criterion_value, wild_bootstrap, residual_bootstrap,
                  chow_all, LR_test, LM_test, Wald_test, targeted_predictors, default_context,
                  CRITERIA, pseudo_out_of_sample_refits, pseudo_out_of_sample_refits_dev,
                  pseudo_out_of_sample_forecasts, MSE, normalize, normalize_dev, clone_model,
                  lasso_path, lasso_stats, get_factors, predict, pseudo_out_of_sample_windows)
from .api import (criterion_PCp1, criterion_PCp2, criterion_PCp3, criterion_ICp1,  # noqa: F401
                  criterion_ICp2, criterion_ICp3, criterion_BIC)
from . import _lib

__all__ = [
    "normalize", "factor_model_DGP", "draw_wild", "draw_wild_fast", "draw_residual", "t_quantile",
    "glmnet_default_folds",
    "Context", "DFMError", "Stat", "DynamicFactorModel", "DynamicFactorModelResult",
    "calculate_factors", "principal_components", "gram_spectrum", "calculate_criterion",
    "factor_residual_variance", "criterion_value", "wild_bootstrap", "residual_bootstrap",
    "chow_all", "LR_test", "LM_test", "Wald_test", "targeted_predictors", "default_context",
    "CRITERIA", "pseudo_out_of_sample_refits", "pseudo_out_of_sample_refits_dev",
    "pseudo_out_of_sample_forecasts", "MSE", "normalize_dev", "clone_model", "lasso_path", "lasso_stats",
    "get_factors", "predict", "pseudo_out_of_sample_windows",
]
