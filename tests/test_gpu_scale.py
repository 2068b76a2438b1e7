"""Batch sizes and context lengths of the BASELINE configs beyond C2 (MI355X only).

  * C3-style continuous batching: generate_batch at 8, 16 and 64 slots gives, per utterance, the
    codes generate() gives alone (the reference decodes batch_size=1, model.py:194;
    every decode kernel's per-row arithmetic is independent of the row count).
  * C5-style long context: a 430-frame audio prefix and 1,000 new frames (positions to ~1,470, four
    512-key softmax blocks merged) through a reduced-depth model at full width, teacher-forced along
    the oracle's own greedy trajectory (oracle/zonos_cpu.py restates model.py:218-315).
  * C5 KV capacity: 8 slots x 5,784 positions at the full 26-layer dims, one graph-captured decode
    step at positions ~5,770.
"""
import json
import os

import pytest
import torch

from zonos_vibes_amd.config import tiny_transformer, transformer_config, zonos_v01_transformer

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cond(seed, lc, d):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(2, lc, d, generator=g) * 0.5).to(torch.bfloat16)


def test_generate_batch_many_slots_equals_single():
    from zonos_vibes_amd.model import Zonos
    cfg = tiny_transformer(2)
    m = Zonos.synthetic(cfg, DEV, zero_eos=True, max_seqlen=96, max_prefill=32)
    n_utt = 70
    conds = [_cond(100 + i, 6 + i % 11, cfg.backbone.d_model).to(DEV) for i in range(n_utt)]
    lens = [8 + (7 * i) % 33 for i in range(n_utt)]
    params = dict(temperature=0.0)
    single = [m.generate(c, max_new_tokens=n, sampling_params=params, progress_bar=False) for c, n in zip(conds, lens)]
    for slots in (8, 16, 64):
        batch = m.generate_batch(conds, max_new_tokens=lens, sampling_params=params, max_slots=slots)
        for i, (a, b) in enumerate(zip(single, batch)):
            assert torch.equal(a, b), (slots, i)
    # generate() after the engine grew to 64 slots still decodes one slot pair the same way
    again = m.generate(conds[5], max_new_tokens=lens[5], sampling_params=params, progress_bar=False)
    assert torch.equal(again, single[5])


def test_generate_batch_full_dims_64_slots_equals_single():
    """C3 at the headline dims (Zonos-v0.1-transformer: 26 layers, d 2048, FFN 8192): 64 slots of short
    mixed-length utterances run the production many-row GEMV shapes (N = 3072 / 16384 / 2048 / 9248 at
    K = 2048 with 4 column groups, fc2 at K = 8192, several row tiles per workgroup, the LayerNorm
    pre-pass) and the chunked attention kernel at 128 rows; 8 of the utterances, decoded alone by
    generate() (2 rows: the fused decode block and the single-tile GEMVs), must give the same codes."""
    from zonos_vibes_amd.model import Zonos
    cfg = zonos_v01_transformer()
    n_utt, slots = 64, 64
    lcs = [8 + (5 * i) % 23 for i in range(n_utt)]
    lens = [6 + (11 * i) % 27 for i in range(n_utt)]
    m = Zonos.synthetic(cfg, DEV, zero_eos=True, max_slots=slots, max_seqlen=max(lcs) + max(lens) + 16,
                        max_prefill=max(lcs) + 8)
    conds = [_cond(300 + i, lc, cfg.backbone.d_model).to(DEV) for i, lc in enumerate(lcs)]
    params = dict(temperature=0.0)
    batch = m.generate_batch(conds, max_new_tokens=lens, sampling_params=params, max_slots=slots)
    m.engine.check_errors()
    for i in (0, 5, 17, 23, 38, 41, 56, 63):
        one = m.generate(conds[i], max_new_tokens=lens[i], sampling_params=params, progress_bar=False)
        assert one.shape[-1] == lens[i]
        assert torch.equal(one, batch[i]), i


def test_attention_form_switch_keeps_codes():
    """generate() whose positions cross the fused forms' reach (the chunk-split form to position 1023, then the
    24-chunk split form; or, with that form off, the score-exchange form to 1279 and separate launches beyond):
    the engine switches graphs at those positions inside one utterance, and the codes equal those of the
    separate launches throughout."""
    from zonos_vibes_amd.model import Zonos
    cfg = transformer_config(2048, 2, 16, 4, 8192)
    lc, n = 1000, 300  # positions 1001 .. 1308
    m = Zonos.synthetic(cfg, DEV, zero_eos=True, max_seqlen=lc + n + 16, max_prefill=lc + 8)
    cond = _cond(77, lc, 2048).to(DEV)
    params = dict(temperature=0.0)
    e = m.engine
    assert [f for f, _ in e._forms(2)] == ["split", "split24", "xs", "none"]
    e.attn_block = False
    e._build_plan()
    plain = m.generate(cond, max_new_tokens=n, sampling_params=params, progress_bar=False, chunk=128)
    for forms, want in ((("split", "xs"), {"split", "xs", "none"}), (("split", "split24", "xs"), {"split", "split24"})):
        e.attn_block, e.attn_forms = True, forms
        e._build_plan()
        fused = m.generate(cond, max_new_tokens=n, sampling_params=params, progress_bar=False, chunk=128)
        e.check_errors()
        used = {k[1] for k in e._graphs}
        assert want <= used, (forms, sorted(used))
        assert torch.equal(fused, plain), forms
