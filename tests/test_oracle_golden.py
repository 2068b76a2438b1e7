"""Pin the CPU oracle against fixtures produced by the reference itself (tests/golden/make_golden.py)."""
import hashlib

import pytest
import torch

from oracle import zonos_cpu as oz
from oracle.dac_cpu import OracleDAC
from tests.helpers import dac_weights, load_golden, synthetic_weights
from zonos_vibes_amd.config import ZonosConfig


def test_delay_pattern_matches_reference():
    t, _ = load_golden("delay_pattern")
    d = oz.apply_delay_pattern(t["codes"], 1025)
    assert torch.equal(d, t["delayed"])
    assert torch.equal(oz.revert_delay_pattern(d), t["reverted"])


def test_penalty_and_greedy_match_reference():
    t, _ = load_golden("penalty_greedy")
    pen = oz.repetition_penalty(t["logits"].clone(), t["generated"], 3.0, 2)
    assert torch.equal(pen, t["penalized"])
    g = oz.sample(t["logits"].clone(), temperature=0.0, generated=t["generated"])
    assert torch.equal(g, t["greedy"])


def test_penalty_windows_match_reference():
    """Any repetition-penalty window, including 0 (the slice [..., -0:] = whole history) and
    negative ones (Python slice semantics), sampling.py:99-114."""
    t, meta = load_golden("penalty_windows")
    for w in meta["windows"]:
        pen = oz.repetition_penalty(t["logits"].clone(), t["generated"], meta["penalty"], w)
        assert torch.equal(pen, t[f"pen{w}"]), w
        g = oz.sample(t["logits"].clone(), temperature=0.0, generated=t["generated"], rep_window=w)
        assert torch.equal(g, t[f"greedy{w}"]), w


def test_samplers_match_reference_with_its_own_noise():
    t, meta = load_golden("samplers")
    for i, ps in enumerate(meta["params"]):
        out = oz.sample(t["logits"].clone(), generated=t["generated"], noise=t[f"q{i}"], **oz.sample_params(ps))
        assert torch.equal(out, t[f"out{i}"]), ps


def test_rope_table_bits():
    t, meta = load_golden("rope")
    fc = oz.rope_table(16384, 128)
    assert hashlib.sha256(fc.numpy().tobytes()).hexdigest() == meta["sha256"]
    assert torch.equal(fc[:8], t["rows_0_8"])


@pytest.mark.parametrize("case_idx", range(5))
def test_tiny_trajectories(case_idx):
    t, meta = load_golden("tiny_trajectories")
    cfg = ZonosConfig.from_dict(meta["cfg"])
    case = meta["cases"][case_idx]
    w = synthetic_weights(cfg, **case["model_kw"])
    m = oz.OracleZonos(cfg, w)
    tag = case["tag"]
    prefix = t.get(tag + "/prefix")
    torch.set_num_threads(4)
    torch.manual_seed(case["seed"])
    out = m.generate(t[tag + "/cond"], prefix, max_new_tokens=case["n"], sampling_params=case["params"])
    assert torch.equal(out, t[tag + "/codes"]), tag


def test_full_width_layer_logits():
    t, meta = load_golden("full_layer")
    cfg = ZonosConfig.from_dict(meta["cfg"])
    m = oz.OracleZonos(cfg, synthetic_weights(cfg, zero_eos=True))
    torch.set_num_threads(meta["threads"])
    with torch.inference_mode():
        cache = m.new_cache(2, 16 + 8 + 9)
        delayed = oz.apply_delay_pattern(torch.full((1, 9, 8), -1), 1025)
        pl = m.prefill(t["cond"], delayed[..., :1], cache, 2.0)
        cache["offset"] += 17
        cache["lengths"][:] += 17
        assert torch.equal(pl, t["prefill_logits"])
        for s in range(3):
            lg = m.decode_one(t["feed"][s], cache, torch.tensor(2.0))
            cache["offset"] += 1
            cache["lengths"][:] += 1
            assert torch.equal(lg, t["step_logits"][s]), s


def test_dac_decode_matches_transformers():
    t, meta = load_golden("dac_decode")
    torch.set_num_threads(meta["threads"])
    wav = OracleDAC(dac_weights()).decode(t["codes"])
    assert wav.shape == t["wav"].shape
    torch.testing.assert_close(wav, t["wav"], rtol=0, atol=1e-6)


def test_attention_block_structure_matches_torch_cpu_sdpa():
    """oracle/attention_cpu.py restates the softmax blocking of the reference's attention op
    (F.scaled_dot_product_attention on bf16 CPU tensors, _torch.py:136): 512-key blocks with the
    probabilities rounded to bf16 reproduce torch's output far more often than fp32 probabilities
    or an unblocked softmax do. The residue is the fp32 accumulation order of its GEMMs."""
    import torch.nn.functional as F
    from oracle.attention_cpu import attend_row
    torch.manual_seed(0)
    torch.set_num_threads(4)
    S = 700
    q = torch.randn(1, 16, 1, 128).to(torch.bfloat16)
    k = torch.randn(1, 4, S, 128).to(torch.bfloat16)
    v = torch.randn(1, 4, S, 128).to(torch.bfloat16)
    ref = F.scaled_dot_product_attention(q, k, v, enable_gqa=True)[0, :, 0]

    def frac(**kw):
        got = torch.stack([attend_row(q[0, h, 0], k[0, h // 4], v[0, h // 4], **kw) for h in range(16)])
        return (got == ref).float().mean().item()

    blocked = frac()
    assert blocked > 0.78
    assert blocked > frac(round_p=False) + 0.1
    assert blocked > frac(block=1 << 20) + 0.02
    # causal prefill rows follow the same per-query structure
    Sp = 540
    qp = torch.randn(1, 4, Sp, 128).to(torch.bfloat16)
    kp = torch.randn(1, 1, Sp, 128).to(torch.bfloat16)
    vp = torch.randn(1, 1, Sp, 128).to(torch.bfloat16)
    refp = F.scaled_dot_product_attention(qp, kp, vp, is_causal=True, enable_gqa=True)[0]
    same = tot = 0
    for p in (0, 1, 77, 511, 512, 539):
        for h in range(4):
            got = attend_row(qp[0, h, p], kp[0, 0, : p + 1], vp[0, 0, : p + 1])
            same += int((got == refp[h, p]).sum())
            tot += 128
    assert same / tot > 0.8
