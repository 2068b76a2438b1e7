"""zonos_vibes_amd — MI355X-native (gfx950) Zonos generate() + DAC decode hot path.

Public surface mirrors the reference (BreakTheBeta/Zonos_Vibes):
    Zonos.generate(...)           reference zonos/model.py:218-315            (model.py)
    DACAutoencoder.decode(codes)  reference zonos/autoencoder.py:25-27        (autoencoder.py)
    apply/revert_delay_pattern    reference zonos/codebook_pattern.py:5-12   (codebook_pattern.py)
    sample_from_logits            reference zonos/sampling.py:117-182        (sampling.py)
    BACKBONES["hip"]              reference zonos/backbone/__init__.py:1-12  (backbone.py)
Transformer (Zonos-v0.1-transformer) and hybrid (Zonos-v0.1-hybrid: Mamba2 + attention,
reference zonos/backbone/_mamba_ssm.py:9-57; hybrid.py) backbones.
"""
from .config import BackboneConfig, InferenceParams, PrefixConditionerConfig, ZonosConfig  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: importing the package must not require a GPU or the built library
    if name in ("Zonos",):
        from .model import Zonos
        return Zonos
    if name == "DACAutoencoder":
        from .autoencoder import DACAutoencoder
        return DACAutoencoder
    if name in ("apply_delay_pattern", "revert_delay_pattern"):
        from . import codebook_pattern
        return getattr(codebook_pattern, name)
    if name == "sample_from_logits":
        from .sampling import sample_from_logits
        return sample_from_logits
    if name in ("BACKBONES", "HipZonosBackbone"):
        from . import backbone
        return getattr(backbone, name)
    raise AttributeError(name)
