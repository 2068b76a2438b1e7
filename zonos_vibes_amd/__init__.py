"""zonos_vibes_amd — MI355X-native (gfx950) Zonos generate() + DAC decode hot path.

Public surface mirrors the reference (BreakTheBeta/Zonos_Vibes):
    Zonos.generate(...)           reference zonos/model.py:218-315
    DACAutoencoder.decode(codes)  reference zonos/autoencoder.py:25-27
    apply/revert_delay_pattern    reference zonos/codebook_pattern.py:5-12
    sample_from_logits            reference zonos/sampling.py:117-182 (HIP sampler kernel)
    BACKBONES["hip"]              reference zonos/backbone/__init__.py:1-12
"""
from .config import BackboneConfig, PrefixConditionerConfig, ZonosConfig  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: importing the package must not require a GPU or the built library
    if name in ("Zonos",):
        from .model import Zonos
        return Zonos
    if name == "DACAutoencoder":
        from .autoencoder import DACAutoencoder
        return DACAutoencoder
    raise AttributeError(name)
