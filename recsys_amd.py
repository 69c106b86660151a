"""Importable alias for the package directory `recommendation-system-maang-nvidia-_amd/`.

    import recsys_amd
    from recsys_amd import ModelConfig, ProductionTrainer
    from recsys_amd.models import MultiTaskModel

The package directory name (required by the build layout) contains hyphens, so it cannot be
named in an import statement; this module registers the real package and its submodules under
this name as well (one module object each, so classes keep a single identity).
"""
import importlib
import sys

_NAME = "recommendation-system-maang-nvidia-_amd"
_SUBMODULES = ("config", "lookup", "_native", "functional", "models", "optim", "distributed",
               "retrieval", "data", "trainer", "metrics", "serving", "model_service", "graphs")

_pkg = importlib.import_module(_NAME)
for _sub in _SUBMODULES:
    try:
        sys.modules[f"{__name__}.{_sub}"] = importlib.import_module(f"{_NAME}.{_sub}")
    except ImportError:  # pragma: no cover - a missing optional submodule
        pass
sys.modules[__name__] = _pkg
