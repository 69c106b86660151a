"""ModelConfig — the reference's hyper-parameter dataclass, field-for-field.

Mirrors src/config.py:9-61 (same names, defaults, __post_init__ list defaults and to_dict) so
configs written by the reference (config.json via asdict) load unchanged. Four build-only
fields are appended at the end (with defaults, so positional/keyword construction of the
reference fields is unaffected). They are never written into config.json — the trainer puts
them in config_ext.json (``save_config`` / ``load_config``) — so a config.json written here
still loads through the reference's ``ModelConfig(**json.load(f))`` (src/models.py:98-102,
app/model_service.py:40):
  * ctr_loss_mode — how the rank-1 CTR sample weights combine with the per-sample BCE
    (SURVEY Appendix A.6): "per_sample" = (1/B) sum sw*bce (default), "keras3" =
    mean(bce) * mean(sw);
  * clipnorm — the optimizer's clipnorm (src/trainer.py:163 hard-codes 1.0);
  * contraction_precision — how the GEMM-shaped contractions run (Dense layers of the towers and
    the deep net, the DCN-v2 cross stack, the in-batch retrieval U C^T, P.C, P^T.U at D = 128): 0 = fp32 operands on the f32 MFMA; 6 (default) / 9 = every fp32 operand split
    exactly into three bf16 terms on the bf16 MFMA with 6 / 9 cross products (9: the fp32
    products exactly; 6: each product within 2^-23 of its magnitude, one fp32 ulp); fp32
    accumulation in every mode (include/recsys_hip.h RS_PREC_*). The reference's TF-CPU path is
    fp32; its GPU path runs mixed_float16 (scripts/train.py:30-34);
  * early_stopping_restore — which Keras EarlyStopping(restore_best_weights=True) the trainer
    follows (src/trainer.py:166): "keras3" (default: the reference pins only tensorflow>=2.13,
    requirements.txt:2, and from TF 2.16 on tf.keras is Keras 3) restores the best weights at the
    end of training whenever a best epoch was recorded; "keras2" restores them only when the
    stop triggers.
"""
import json
import os
from dataclasses import asdict, dataclass, fields
from typing import Any, Dict, List


@dataclass
class ModelConfig:
    """Configuration for the recommendation model (src/config.py:9)."""

    # Embedding dimensions (src/config.py:13-16)
    embedding_dim: int = 128
    user_tower_dims: List[int] = None
    item_tower_dims: List[int] = None

    # DCN parameters (src/config.py:18-22)
    cross_layers: int = 3
    dnn_dims: List[int] = None
    dropout_rate: float = 0.2
    l2_reg: float = 1e-4

    # Training parameters (src/config.py:24-30)
    batch_size: int = 2048
    learning_rate_retrieval: float = 0.001
    learning_rate_ranking: float = 0.0001
    epochs_retrieval: int = 20
    epochs_ranking: int = 5
    warmup_steps: int = 1000

    # Negative sampling (src/config.py:32-35)
    num_hard_negatives: int = 5
    num_random_negatives: int = 10
    negative_sampling_strategy: str = "mixed"

    # Multi-task weights (src/config.py:37-40)
    retrieval_weight: float = 1.0
    ctr_weight: float = 2.0
    rating_weight: float = 0.2

    # Evaluation (src/config.py:42-43)
    eval_topk: List[int] = None

    # System settings (src/config.py:45-47)
    mixed_precision: bool = True
    distributed_strategy: str = "none"

    # build extensions (see module docstring)
    ctr_loss_mode: str = "per_sample"
    clipnorm: float = 1.0
    contraction_precision: int = 6
    early_stopping_restore: str = "keras3"

    def __post_init__(self):
        # src/config.py:49-57
        if self.user_tower_dims is None:
            self.user_tower_dims = [256, 128, 64]
        if self.item_tower_dims is None:
            self.item_tower_dims = [256, 128, 64]
        if self.dnn_dims is None:
            self.dnn_dims = [256, 128]
        if self.eval_topk is None:
            self.eval_topk = [5, 10, 20, 50]
        if self.ctr_loss_mode not in ("per_sample", "keras3"):
            raise ValueError(f"ctr_loss_mode must be 'per_sample' or 'keras3', got {self.ctr_loss_mode!r}")
        if self.contraction_precision not in (0, 6, 9):
            raise ValueError(f"contraction_precision must be 0, 6 or 9, got {self.contraction_precision!r}")
        if self.early_stopping_restore not in ("keras3", "keras2"):
            raise ValueError("early_stopping_restore must be 'keras3' or 'keras2', "
                             f"got {self.early_stopping_restore!r}")

    def to_dict(self):
        """Convert config to dictionary (src/config.py:59-61)."""
        return asdict(self)

    @property
    def ctr_mode_code(self) -> int:
        return 0 if self.ctr_loss_mode == "per_sample" else 1

    def reference_dict(self) -> Dict[str, Any]:
        """The src/config.py:9-61 fields only: what ``config.json`` holds."""
        d = asdict(self)
        return {k: d[k] for k in REFERENCE_FIELDS}

    def extension_dict(self) -> Dict[str, Any]:
        d = asdict(self)
        return {k: d[k] for k in EXTENSION_FIELDS}


EXTENSION_FIELDS = ("ctr_loss_mode", "clipnorm", "contraction_precision", "early_stopping_restore")
REFERENCE_FIELDS = tuple(f.name for f in fields(ModelConfig) if f.name not in EXTENSION_FIELDS)
CONFIG_FILE, CONFIG_EXT_FILE = "config.json", "config_ext.json"


def save_config(config: ModelConfig, model_dir) -> None:
    """config.json (reference schema, src/trainer.py:232-233) + config_ext.json (build fields)."""
    with open(os.path.join(model_dir, CONFIG_FILE), "w") as f:
        json.dump(config.reference_dict(), f, indent=2)
    with open(os.path.join(model_dir, CONFIG_EXT_FILE), "w") as f:
        json.dump(config.extension_dict(), f, indent=2)


def load_config(model_dir) -> ModelConfig:
    """Inverse of save_config. Unknown keys are ignored (as the services always did); a missing
    config.json gives the defaults; config_ext.json is optional (reference-written dirs)."""
    names = {f.name for f in fields(ModelConfig)}
    raw: Dict[str, Any] = {}
    for fn in (CONFIG_FILE, CONFIG_EXT_FILE):
        path = os.path.join(model_dir, fn)
        if os.path.exists(path):
            with open(path) as f:
                raw.update(json.load(f))
    return ModelConfig(**{k: v for k, v in raw.items() if k in names})
