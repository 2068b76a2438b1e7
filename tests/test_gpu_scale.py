"""Batch sizes and context lengths of the BASELINE configs beyond C2 (MI355X only).

  * C3-style continuous batching: generate_batch at 8, 16 and 64 slots gives, per utterance, the
    codes generate() gives alone (the reference decodes batch_size=1, model.py:194;
    every decode kernel's per-row arithmetic is independent of the row count).
  * C3 at its own lengths (full 26-layer dims): the first 64 utterances of bench.c3_job() (2-30 s, positions
    to ~3,000 at 128 rows, the busy-slot bucket shrinking 64 -> 1 as they finish); generate_batch equals
    generate() per utterance, bit for bit, for the longest ones and a few short ones.
  * C5-style long context: 8 slots (16 rows: the separate QKV GEMV + the 512-key block-form attention with its
    prefetch role, asserted), each with a 430-frame audio prefix, 1,000 new frames (positions to ~1,470, three
    512-key softmax blocks merged) at full width, 2 layers; slot 0 teacher-forced along the oracle's own greedy
    trajectory (oracle/zonos_cpu.py restates model.py:218-315).
  * C5 KV capacity: 8 slots x 5,784 positions at the full 26-layer dims, one graph-captured decode
    step at positions ~5,770 through the block-form attention, its last layer checked against the blocking
    oracle and fp32 SDPA.
These two C5 tests were dropped in round 4 (commit aa697ec) when the block form became the library's choice for
16-row steps; round 5 restored them on that form.
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


def _ulp(x):
    return torch.ldexp(torch.ones_like(x), torch.frexp(x.abs().clamp_min(1e-30))[1] - 8)


LONG_BOUND_ULPS = 6.0  # allowed |GPU - oracle| score of the oracle's choice, bf16 ulps of its top score


def _assert_block_form_plan(e, rows):
    """The decode plan of `rows` rows runs the separate QKV GEMV + zmi_attention_pf with a prefetch role, and the
    library resolves that launch to the 512-key block form (variant 5)."""
    form = e._segments(1, rows // 2)[0][1]
    assert form == "none", form
    attn = [it for kind, it in e._plan(rows, form) if kind == "attn"]
    assert len(attn) == e.L, len(attn)
    assert all(pf is not None and pf.blocks > 0 and pf.bytes[0] > 0 for _, pf in attn)
    assert e.lib.zmi_attention_pick(rows, e.Hkv, e.attn_variant) == 5


def test_c5_prefix_430_generate_1000_teacher_forced_8_slots():
    """C5 shape at full width (d 2048, 16 / 4 heads x 128), 2 layers: 8 slots of Lc 32 + a 430-frame prefix,
    1,000 new frames, greedy with the repetition penalty, EOS suppressed. Every step decodes 16 rows through the
    block-form attention. Along the oracle's trajectory (slot 0 teacher-forced; slots 1-7 decode their own
    prefixes freely beside it) every decision's GPU score of the oracle's token is within LONG_BOUND_ULPS of the
    oracle's top score, and the GPU picks the oracle's token wherever the oracle's margin exceeds twice that."""
    from oracle.zonos_cpu import OracleZonos, apply_delay_pattern, repetition_penalty
    from tests.helpers import synthetic_weights
    from zonos_vibes_amd.engine import SamplingParams
    from zonos_vibes_amd.model import Zonos
    cfg = transformer_config(2048, 2, 16, 4, 8192)
    lc, p, n, slots = 32, 430, 1000, 8
    conds = [_cond(7 + i, lc, cfg.backbone.d_model) for i in range(slots)]
    g = torch.Generator().manual_seed(8)
    prefixes = [torch.randint(0, 1024, (1, 9, p), generator=g) for _ in range(slots)]
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    om = OracleZonos(cfg, synthetic_weights(cfg, zero_eos=True))
    trace = []
    om.generate(conds[0], prefixes[0], max_new_tokens=n, sampling_params=dict(temperature=0.0), trace=trace)
    dl = om.last_delayed[0].long()
    m = Zonos.synthetic(cfg, DEV, zero_eos=True, max_slots=slots, max_seqlen=lc + p + n + 24, max_prefill=lc + p + 8)
    e = m.engine
    for s in range(slots):
        e.prefill(s, conds[s].to(DEV), prefixes[s], n, SamplingParams(temperature=0.0))
    e.stream.synchronize()
    _assert_block_form_plan(e, 2 * slots)

    def cfg_logits(rows):
        c, u = rows[0].float().cpu(), rows[1].float().cpu()
        lg = u + (c - u) * 2.0
        lg[..., 1025:] = -torch.inf
        return lg

    bias = torch.zeros(9, 1026)
    bias[1:, 1024] = -torch.inf
    scores = [cfg_logits(e.logits_pre)]  # the last prefill's logits: slot 7's, so decision 0 is not compared
    dl_dev = dl.to(DEV, torch.int32)
    for _ in range(len(trace) - 1):
        with torch.cuda.stream(e.stream):  # the oracle's frames in slot 0, whatever the GPU sampler chose
            e.delayed[0, :, : dl.shape[-1]] = dl_dev
            for k, v in (("active", 1), ("stopping", 0), ("remaining", 2000)):
                e.st[k][0] = v
            e.refresh_inputs()
        o = int(e.st["offset"][0].item())
        e.step(1, use_graph=False, slots=slots)
        e.stream.synchronize()
        lg = cfg_logits(e.logits[0:2]) + bias
        scores.append(repetition_penalty(lg.unsqueeze(0), dl[None, :, : o + 1], 3.0, 2)[0])
    e.check_errors()
    assert max(e.pos_hi[:slots]) >= lc + p + n, e.pos_hi[:slots]
    init = apply_delay_pattern(torch.cat([prefixes[0], torch.full((1, 9, n), -1)], -1), 1025)[0]
    rows = []
    for i in range(1, min(len(trace), init.shape[1] - p - 1)):
        f = p + 1 + i  # decision i fills the unknown codebooks of delayed frame f, in order
        ref = trace[i][0]
        for mm, k in enumerate((init[:, f] == -1).nonzero().flatten().tolist()):
            tok = int(dl[k, f])
            if tok >= 1024:
                continue
            t2 = ref[mm].topk(2).values
            u = float(_ulp(t2[0]))
            rows.append(dict(err=abs(float(scores[i][mm, tok]) - float(t2[0])) / u,
                             margin=float(t2[0] - t2[1]) / u, agree=int(scores[i][mm].argmax()) == tok))
    det = [r for r in rows if r["margin"] > 2 * LONG_BOUND_ULPS]
    stats = dict(slots=slots, decisions=len(rows), agree=sum(r["agree"] for r in rows), determined=len(det),
                 determined_agree=sum(r["agree"] for r in det), max_err_ulps=max(r["err"] for r in rows),
                 mean_err_ulps=sum(r["err"] for r in rows) / len(rows), last_position=lc + p + len(trace),
                 attention="block form (variant 5) + prefetch role, 16 rows")
    if os.path.isdir("gpurun_out"):
        json.dump(stats, open("gpurun_out/c5_teacher_forced.json", "w"), indent=1)
    assert stats["decisions"] > 8000
    assert stats["determined_agree"] == stats["determined"], stats
    assert stats["max_err_ulps"] <= LONG_BOUND_ULPS, stats


def test_c5_kv_capacity_8_slots_5784_positions():
    """The C5 engine at the full 26-layer dims: 8 slots x 5,784 KV positions allocated; one graph-captured 16-row
    decode step at positions 5,760-5,775 through the block-form attention (asserted); the last layer's attention of
    three rows checked against the blocking oracle and fp32 SDPA."""
    from zonos_vibes_amd.model import Zonos
    cfg = zonos_v01_transformer()
    smax_req = 5784
    m = Zonos.synthetic(cfg, DEV, zero_eos=True, max_seqlen=smax_req, max_prefill=16, max_slots=8)
    e = m.engine
    assert e.smax >= smax_req
    kv_bytes = (e.kc.numel() + e.vc.numel()) * e.kc.element_size()
    assert kv_bytes == 2 * cfg.backbone.n_layer * 16 * 4 * e.smax * 128 * 2  # 16 rows = 8 CFG slot pairs
    rows = 16
    with torch.cuda.stream(e.stream):
        e.row_pos[:rows] = torch.arange(5760, 5760 + rows, dtype=torch.int32, device=DEV)
        e.row_kv[:rows] = torch.arange(rows, dtype=torch.int32, device=DEV)
        e.x[:rows].normal_()
        e.kc.normal_()
        e.vc.normal_()
    e.stream.synchronize()
    e.pos_hi[:8] = [5760 + rows - 1] * 8  # host position bound (set by a prefill in generate())
    _assert_block_form_plan(e, rows)
    e.step(1, use_graph=True, slots=8)
    e.stream.synchronize()
    e.check_errors()
    assert torch.isfinite(e.logits[:rows]).all()
    # the last layer's attention of three rows at ~5.77k keys against the blocking oracle and fp32 SDPA
    from tests.test_gpu_kernels import _check_attention
    last = cfg.backbone.n_layer - 1
    pick = [0, 7, 15]
    _check_attention(e.attn[pick], e.q[pick], e.kc[last][pick], e.vc[last][pick].transpose(-1, -2).contiguous(),
                     [5760 + r for r in pick])


def test_c3_real_lengths_64_slots_equals_single():
    """C3 at its own lengths and the headline dims: utterances 0..63 of bench.c3_job() (2-30 s, Lc 8 + 15 s, the
    conditioning bench.time_c3_sharded uses) through 64 slots; the steps shrink to the busy slots' bucket
    (64 -> ... -> 1) as utterances finish. generate() alone must give, bit for bit, the codes of the six longest
    utterances (each over 20 s, finishing in the small buckets) and of two short ones."""
    import bench
    from zonos_vibes_amd.model import Zonos
    cfg = zonos_v01_transformer()
    lcs, n_all = bench.c3_job()
    lcs, n_new = lcs[:64], n_all[:64]
    long_ = sorted(range(64), key=lambda i: -n_new[i])[:6]
    short = sorted(range(64), key=lambda i: n_new[i])[:2]
    assert all(n_new[i] > 20 * 86 for i in long_), [n_new[i] for i in long_]
    m = Zonos.synthetic(cfg, DEV, zero_eos=True, max_slots=64, max_seqlen=max(lcs) + max(n_new) + 16,
                        max_prefill=max(lcs) + 8)
    conds = [bench.cond_tensor(1000 + i, cfg.backbone.d_model, DEV, lc) for i, lc in enumerate(lcs)]
    params = dict(temperature=0.0)
    batch = m.generate_batch(conds, max_new_tokens=n_new, sampling_params=params, max_slots=64)
    m.engine.check_errors()
    assert [int(c.shape[-1]) for c in batch] == n_new
    for i in long_ + short:
        one = m.generate(conds[i], max_new_tokens=n_new[i], sampling_params=params, progress_bar=False, chunk=128)
        assert torch.equal(one, batch[i]), (i, n_new[i])
