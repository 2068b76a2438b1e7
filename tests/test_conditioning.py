"""Prefix conditioner: oracle and tokenizer pinned to the reference's outputs
(tests/golden/prefix_cond.safetensors, made by make_golden_cond.py); the HIP path
(zmi_prefix_condition) against the same fixture and against the oracle at full width (d = 2048).

Tolerance of the HIP path (bf16 output): every element within one bf16 ulp of the reference value
(absolute floor 2^-20 for outputs near zero), and at least 98 % of them bit-identical. The op order and rounding points are the reference's; the
residual differences are fp32 summation order in the LayerNorm and cos/sin of the device libm."""
import math

import pytest
import torch

from oracle.conditioning_cpu import OracleConditioner
from tests.helpers import load_golden
from zonos_vibes_amd.conditioning import (PHONEME_VOCAB, make_cond_dict, tokenize_phonemes,
                                          v01_transformer_conditioners)


@pytest.fixture(scope="module")
def gold():
    return load_golden("prefix_cond")


def _weights(t):
    return {k[2:]: v for k, v in t.items() if k.startswith("w/")}


def _cond_dict(t, case, device="cpu"):
    kw = dict(case["kw"])
    if "unconditional_keys" in kw:
        kw["unconditional_keys"] = set(kw["unconditional_keys"])
    kw.setdefault("speaker", t["speaker"])
    return make_cond_dict(phonemes=case["text"], language=case["language"], device=device, **kw)


def assert_bf16_close(got, ref, exact_frac=0.98):
    got, ref = got.float().cpu(), ref.float().cpu()
    assert got.shape == ref.shape
    mag = torch.maximum(ref.abs(), got.abs()).clamp_min(2.0 ** -20)  # a flip may cross a binade
    # one bf16 ulp, floored at 2^-20 absolute: an output near zero is the cancellation of O(1) terms, whose
    # fp32 summation-order error (~1e-7) is then several of its own tiny ulps
    ulp = torch.exp2(torch.floor(torch.log2(mag)) - 7).clamp_min(2.0 ** -20)
    diff = (got - ref).abs()
    bad = (diff > ulp).nonzero()
    assert bad.numel() == 0, (f"{bad.shape[0]} elements beyond one bf16 ulp, first at {bad[:4].tolist()}: "
                              f"got {got[tuple(bad[0])].item()} ref {ref[tuple(bad[0])].item()}")
    assert (diff == 0).float().mean().item() >= exact_frac


def test_tokenizer_matches_reference(gold):
    t, meta = gold
    for c in meta["cases"]:
        ids, lengths = tokenize_phonemes([c["text"]])
        assert torch.equal(ids, t[c["tag"] + "/ids"]), c["tag"]
        assert lengths == [t[c["tag"] + "/ids"].shape[1]]
    ids, lengths = tokenize_phonemes(["ab", "a"])
    assert ids[1, 0].item() == 0 and lengths == [4, 3]  # left padding with PAD
    assert int(ids.max()) < PHONEME_VOCAB


def test_make_cond_dict_keys_match_reference(gold):
    t, meta = gold
    for c in meta["cases"]:
        assert sorted(_cond_dict(t, c).keys()) == c["keys"]
    d = make_cond_dict(phonemes="a")
    assert torch.allclose(d["emotion"].sum(), torch.tensor(1.0))
    with pytest.raises(NotImplementedError):
        make_cond_dict(text="hello")


def test_oracle_matches_reference_golden(gold):
    t, meta = gold
    orc = OracleConditioner(meta["conditioners"], meta["d"], _weights(t))
    for c in meta["cases"]:
        out = orc.prepare_conditioning(_cond_dict(t, c))
        assert torch.equal(out, t[c["tag"] + "/out"]), c["tag"]


def test_v01_conditioner_list_shapes():
    from zonos_vibes_amd.conditioning import PrefixConditioner
    pc = PrefixConditioner(v01_transformer_conditioners(), 2048, device="cpu")
    shapes = pc.param_shapes()
    assert shapes["conditioners.6.int_embedder.weight"] == (128, 2048)  # language_id -1..126
    assert shapes["conditioners.1.project.weight"] == (2048, 128)
    assert pc.required_keys == {"espeak"}


@pytest.mark.gpu
def test_hip_conditioner_matches_reference_golden(gold):
    from zonos_vibes_amd.conditioning import PrefixConditioner
    t, meta = gold
    pc = PrefixConditioner(meta["conditioners"], meta["d"], device="cuda")
    pc.load_state_dict(_weights(t))
    for c in meta["cases"]:
        out = pc.prepare_conditioning(_cond_dict(t, c, "cuda"))
        assert_bf16_close(out, t[c["tag"] + "/out"])


@pytest.mark.gpu
def test_hip_conditioner_full_width_matches_oracle():
    from zonos_vibes_amd.conditioning import PrefixConditioner
    d = 2048
    pc = PrefixConditioner(v01_transformer_conditioners(), d, device="cuda")
    g = torch.Generator().manual_seed(5)
    w = {k: torch.randn(s, generator=g).to(torch.bfloat16) for k, s in pc.param_shapes().items()}
    pc.load_state_dict(w)
    spk = (0.3 * torch.randn(1, 128, generator=g)).to(torch.bfloat16)
    cd = make_cond_dict(phonemes="ðɪs ɪz ə tɛst sɛntəns, wɪð sʌm lɛŋθ.", language="en-gb", speaker=spk,
                        pitch_std=45.0, speaking_rate=12.5)
    ref = OracleConditioner(v01_transformer_conditioners(), d, w).prepare_conditioning(cd)
    got = pc.prepare_conditioning({k: (v.cuda() if isinstance(v, torch.Tensor) else v) for k, v in cd.items()})
    assert_bf16_close(got, ref)
    # the conditioning feeds generate() directly
    assert got.dtype == torch.bfloat16 and math.isfinite(got.float().abs().max().item())


@pytest.mark.gpu
def test_prepare_conditioning_feeds_generate():
    """Zonos.prepare_conditioning (model.py:204-212) -> generate() on the HIP path, end to end."""
    from zonos_vibes_amd.config import PrefixConditionerConfig, tiny_transformer
    from zonos_vibes_amd.model import Zonos
    cfg = tiny_transformer(2)
    cfg.prefix_conditioner = PrefixConditionerConfig(v01_transformer_conditioners(), "none")
    m = Zonos.synthetic(cfg, "cuda", zero_eos=True, max_seqlen=96, max_prefill=48)
    g = torch.Generator().manual_seed(9)
    w = {k: torch.randn(s, generator=g).to(torch.bfloat16)
         for k, s in m.prefix_conditioner.param_shapes().items()}
    m.prefix_conditioner.load_state_dict(w)
    cd = make_cond_dict(phonemes="həloʊ", speaker=torch.zeros(1, 128, dtype=torch.bfloat16), device="cuda")
    cond = m.prepare_conditioning(cd)
    assert cond.shape == (2, 7 + 6, cfg.backbone.d_model)
    codes = m.generate(cond, max_new_tokens=12, sampling_params=dict(temperature=0.0), progress_bar=False)
    assert codes.shape == (1, 9, 12) and int(codes.max()) < 1024
