"""Loaders (CPU): the DAC weight-norm fold in both key styles, and the safetensors / config.json
files Zonos.from_local reads (reference model.py:65-88; GPU round trip in test_gpu_api.py)."""
import json

import torch

from zonos_vibes_amd.autoencoder import _fold_weight_norm
from zonos_vibes_amd.config import ZonosConfig, tiny_transformer


def _weight_norm_pair(w):
    g = w.flatten(1).norm(dim=1).view(-1, *([1] * (w.dim() - 1)))
    return g, w.clone()


def test_weight_norm_fold_both_key_styles():
    torch.manual_seed(0)
    w = torch.randn(16, 8, 7)
    g, v = _weight_norm_pair(w * 3.0)
    v = v * 0.5  # the fold must divide by |v|, not assume |v| = g
    a = _fold_weight_norm({"decoder.conv1.weight_g": g, "decoder.conv1.weight_v": v, "decoder.conv1.bias": torch.ones(16)})
    b = _fold_weight_norm({"decoder.conv1.parametrizations.weight.original0": g,
                           "decoder.conv1.parametrizations.weight.original1": v, "decoder.conv1.bias": torch.ones(16)})
    for sd in (a, b):
        assert set(sd) == {"decoder.conv1.weight", "decoder.conv1.bias"}
        torch.testing.assert_close(sd["decoder.conv1.weight"], w * 3.0, rtol=1e-5, atol=1e-5)
    assert torch.equal(a["decoder.conv1.weight"], b["decoder.conv1.weight"])


def test_weight_norm_fold_matches_torch_parametrization():
    conv = torch.nn.Conv1d(8, 16, 7)
    conv = torch.nn.utils.parametrizations.weight_norm(conv)
    sd = {"c." + k: v for k, v in conv.state_dict().items()}
    assert "c.parametrizations.weight.original0" in sd
    out = _fold_weight_norm(sd)
    torch.testing.assert_close(out["c.weight"], conv.weight.detach(), rtol=1e-6, atol=1e-6)


def test_config_json_round_trip(tmp_path):
    cfg = tiny_transformer(2)
    p = tmp_path / "config.json"
    p.write_text(json.dumps(cfg.to_dict()))
    back = ZonosConfig.from_dict(json.loads(p.read_text()))
    assert back == cfg and back.backbone.num_heads == 4 and back.backbone.num_heads_kv == 1
