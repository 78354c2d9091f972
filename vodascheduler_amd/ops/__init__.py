"""Hand-written CDNA4 (gfx950) ops with PyTorch CPU references."""
from .bucket import cast_scale_, multi_tensor_copy_
from .layernorm import FusedLayerNorm, layer_norm
from .optim import FusedAdam, FusedAdamW, FusedRMSprop, FusedSGD, make_optimizer
from .softmax import masked_softmax, reference_masked_softmax

__all__ = [
    "cast_scale_", "multi_tensor_copy_", "FusedLayerNorm", "layer_norm", "FusedAdam", "FusedAdamW",
    "FusedRMSprop", "FusedSGD", "make_optimizer", "masked_softmax", "reference_masked_softmax",
]
