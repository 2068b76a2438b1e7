"""Golden fixture for DACAutoencoder.encode, produced by the REFERENCE (in this container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_dac_enc.py

The reference's `DACAutoencoder.encode` (zonos/autoencoder.py:22-23 -> transformers DacModel.encode)
runs on a random-init 44.1 kHz DacModel whose every tensor is overwritten with the synthetic values of
zonos_vibes_amd.synthetic (dac_specs + dac_encoder_specs), on 2 x 16 frames of a synthetic waveform
(sum of sines + noise, |x| <= 0.9). Recorded: the input, the encoder latents, and the codes
(tests/golden/dac_encode.safetensors).
"""
from __future__ import annotations

import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from make_golden import import_reference, save  # noqa: E402
from zonos_vibes_amd import synthetic as syn  # noqa: E402
from tests.helpers import synthetic_wav  # noqa: E402


def main():
    import_reference()
    from transformers import DacConfig, DacModel
    from zonos.autoencoder import DACAutoencoder
    torch.set_num_threads(8)
    dac = DacModel(DacConfig(sampling_rate=44100)).eval()
    dsd = dac.state_dict()
    for k, v in syn.iter_torch_cpu(syn.dac_specs() + syn.dac_encoder_specs(), 0):
        assert dsd[k].shape == v.shape, (k, dsd[k].shape, v.shape)
        dsd[k].copy_(v)
    dac.load_state_dict(dsd)
    ae = DACAutoencoder.__new__(DACAutoencoder)
    ae.dac = dac
    wav = synthetic_wav(2, 16 * 512, 11)
    with torch.inference_mode():
        codes = ae.encode(wav)
        lat = dac.encoder(wav)
    save("dac_encode", {"wav": wav, "latents": lat, "codes": codes}, {"threads": 8})


if __name__ == "__main__":
    main()
