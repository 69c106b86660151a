"""MI355X-native two-tower retrieval + DCN ranking hot path (drop-in for the reference's
src/models.py + src/trainer.py path of OnlyAhad13/Recommendation-System-MAANG-NVIDIA-).

Exports mirror src/__init__.py (ModelConfig, ProductionTrainer) plus the model classes of
src/models.py. The hot ops are hand-written gfx950 HIP kernels in librecsys_hip.so (C-ABI:
include/recsys_hip.h); this package is the host-side mirror of the reference interface.

The directory name is not a Python identifier; import it with
``importlib.import_module("recommendation-system-maang-nvidia-_amd")`` or through the
``recsys_amd`` alias module at the repository root.
"""
from .config import ModelConfig

__version__ = "0.1.0"


def __getattr__(name):
    # Lazy: importing the config must not require a GPU or the native library.
    if name in ("ProductionTrainer",):
        from .trainer import ProductionTrainer
        return ProductionTrainer
    if name in ("MultiTaskModel", "MultiTowerModel", "DeepCrossNetwork"):
        from . import models
        return getattr(models, name)
    raise AttributeError(name)


__all__ = ["ModelConfig", "ProductionTrainer", "MultiTaskModel", "MultiTowerModel", "DeepCrossNetwork"]
