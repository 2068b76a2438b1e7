"""The reference's module-level API on the HIP path (MI355X only):
codebook_pattern (zonos/codebook_pattern.py:5-12), sample_from_logits (zonos/sampling.py:117-182),
the backbone plugin BACKBONES["hip"] (zonos/backbone/__init__.py:1-12, _torch.py:52-80) and
Zonos.from_local (zonos/model.py:65-88) from files on disk."""
import json

import pytest
import torch

from tests.helpers import dac_weights, load_golden, synthetic_weights
from zonos_vibes_amd.config import tiny_transformer

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_delay_pattern_api_matches_reference():
    from zonos_vibes_amd.codebook_pattern import apply_delay_pattern, revert_delay_pattern
    t, _ = load_golden("delay_pattern")
    d = apply_delay_pattern(t["codes"].to(DEV), 1025)
    assert torch.equal(d.cpu(), t["delayed"])
    assert torch.equal(revert_delay_pattern(d).cpu(), t["reverted"])


def test_sample_from_logits_api_matches_reference():
    from zonos_vibes_amd.sampling import sample_from_logits
    t, _ = load_golden("penalty_greedy")
    g = sample_from_logits(t["logits"].to(DEV), temperature=0.0, generated_tokens=t["generated"].to(DEV))
    assert torch.equal(g.cpu(), t["greedy"])
    t, meta = load_golden("samplers")
    for i, ps in enumerate(meta["params"]):
        out = sample_from_logits(t["logits"].to(DEV), generated_tokens=t["generated"].to(DEV), noise=t[f"q{i}"], **ps)
        assert torch.equal(out.cpu(), t[f"out{i}"]), ps
    t, meta = load_golden("penalty_windows")
    for w in meta["windows"]:
        out = sample_from_logits(t["logits"].to(DEV), temperature=0.0, generated_tokens=t["generated"].to(DEV),
                                 repetition_penalty_window=w)
        assert torch.equal(out.cpu(), t[f"greedy{w}"]), w


def _ulps(got, ref):
    """|got - ref| in bf16 ulps of the larger of the element and its row's RMS (LayerNorm'd rows
    have RMS ~1: near-zero elements are measured on the row's scale, not their own)."""
    got, ref = got.float().cpu(), ref.float().cpu()
    rms = ref.pow(2).mean(-1, keepdim=True).sqrt()
    ulp = torch.ldexp(torch.ones_like(ref), torch.frexp(torch.maximum(ref.abs(), rms))[1] - 8)
    return (got - ref).abs() / ulp


def test_backbone_plugin_matches_oracle_backbone():
    """Prefill of 2 x 12 positions then 3 single-position steps through BACKBONES["hip"], against the
    oracle's restatement of TorchZonosBackbone.forward (+ norm_f) on the same weights."""
    from oracle.zonos_cpu import OracleZonos
    from zonos_vibes_amd.backbone import BACKBONES
    from zonos_vibes_amd.config import InferenceParams
    cfg = tiny_transformer(2)
    w = synthetic_weights(cfg)
    om = OracleZonos(cfg, w)
    bb = BACKBONES["hip"](cfg.backbone, DEV)
    bb.load_state_dict({k[len("backbone."):]: v for k, v in w.items() if k.startswith("backbone.")})
    cache = bb.allocate_inference_cache(2, 64)
    params = InferenceParams(64, 2, key_value_memory_dict=cache,
                             lengths_per_sample=torch.zeros(2, dtype=torch.int32, device=DEV))
    ocache = om.new_cache(2, 64)
    g = torch.Generator().manual_seed(3)
    for s in (12, 1, 1, 1):
        h = torch.randn(2, s, cfg.backbone.d_model, generator=g).to(torch.bfloat16)
        got = bb.forward(h.to(DEV), params)
        ref = om.backbone(h, ocache)
        u = _ulps(got, ref)
        assert (u <= 1).float().mean() > 0.98 and u.max() <= 8, (s, (u <= 1).float().mean().item(), u.max().item())
        params.seqlen_offset += s
        params.lengths_per_sample += s
        ocache["offset"] += s
        ocache["lengths"] += s


def test_from_local_loads_reference_files(tmp_path):
    """config.json + model.safetensors with the reference's state_dict names (heads [1025, d]) and a
    DAC state_dict in weight-norm form: the loaded model generates and decodes exactly as the same
    synthetic model built in memory."""
    from safetensors.torch import save_file
    from zonos_vibes_amd.model import Zonos
    cfg = tiny_transformer(2)
    w = synthetic_weights(cfg, zero_eos=True)
    (tmp_path / "config.json").write_text(json.dumps(cfg.to_dict()))
    save_file({k: v.contiguous() for k, v in w.items()}, str(tmp_path / "model.safetensors"))
    dw = dac_weights()
    dsd = {}
    for k, v in dw.items():  # conv weights as parametrizations.weight.original0/1 pairs
        if k.endswith(".weight") and v.dim() == 3 and "quantizer" not in k:
            gnorm = v.flatten(1).norm(dim=1).view(-1, 1, 1)
            dsd[k[: -len("weight")] + "parametrizations.weight.original0"] = gnorm.contiguous()
            dsd[k[: -len("weight")] + "parametrizations.weight.original1"] = v.contiguous()
        else:
            dsd[k] = v.contiguous()
    save_file(dsd, str(tmp_path / "dac.safetensors"))
    m = Zonos.from_local(str(tmp_path / "config.json"), str(tmp_path / "model.safetensors"), DEV, backbone="hip",
                         dac_path=str(tmp_path / "dac.safetensors"), max_seqlen=64, max_prefill=32)
    ref = Zonos.synthetic(cfg, DEV, zero_eos=True, max_seqlen=64, max_prefill=32)
    t, _ = load_golden("tiny_trajectories")
    cond = t["greedy_maxlen/cond"].to(DEV)
    a = m.generate(cond, max_new_tokens=12, sampling_params=dict(temperature=0.0), progress_bar=False)
    b = ref.generate(cond, max_new_tokens=12, sampling_params=dict(temperature=0.0), progress_bar=False)
    assert torch.equal(a, b)
    wa, wb = m.autoencoder.decode(a), ref.autoencoder.decode(a)
    assert (wa - wb).abs().max() < 1e-3  # weight-norm fold in fp32 vs direct weights
    with pytest.raises(ValueError):
        Zonos.from_local(str(tmp_path / "config.json"), str(tmp_path / "model.safetensors"), DEV, backbone="torch")
