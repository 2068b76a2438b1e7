"""Headline benchmark: real-time factor of Zonos-v0.1-transformer generate() + DAC decode on MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): one utterance per GPU per step —
batch=1, Lc=160 synthetic prefix-conditioning rows, 861 new frames (10 s of 44.1 kHz audio),
greedy decode with the reference's default repetition penalty, EOS suppressed (row 1024 of
heads.0 zeroed) so every step decodes exactly 869 backbone steps, then DAC decode of the 861
frames. Synthetic hash-PRNG weights at the full 1.6 B-parameter transformer dims.
A "step" = one full utterance (prefill + 869 decode steps + DAC decode).
value = total audio seconds over all ranks / max-over-ranks wall time of the K timed steps.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from zonos_vibes_amd import _lib  # noqa: E402
from zonos_vibes_amd import synthetic as syn  # noqa: E402
from zonos_vibes_amd.config import DAC_HOP, DAC_SAMPLE_RATE, zonos_v01_transformer  # noqa: E402

LC, N_NEW = 160, 861
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
BASELINE_RTF = 2.0     # "~2x" real-time on RTX 4090 (README.md:84)


def cond_tensor(seed: int, d: int, dev, lc: int = LC):
    import numpy as np
    a = syn.synthetic_conditioning_np(seed, 2, lc, d)
    return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16).to(dev)


def _live_state(model, cond):
    """Prefill slot 0 with the bench conditioning and decode to the C2 mean position; returns the position."""
    from zonos_vibes_amd.engine import SamplingParams
    e = model.engine
    s_len = e.prefill(0, cond, None, N_NEW, SamplingParams(temperature=0.0, cfg_scale=2.0))
    lead = (N_NEW + 8) // 2
    e.step(lead, slots=1)
    return s_len + lead


# the committed FETCH_SIZE pass of each dominant-kernel candidate, newest round first (tools/gpu.sh round)
PMC_FILES = {"attn_block_kernel<8, 1, 2, true>": ["r06_pmc_attnblk_fetch.json", "r05_pmc_attnblk_fetch.json"],
             "attn_block_kernel<24, 1, 2, true>": ["r06_pmc_attnblk24_fetch.json"],
             "gemv_kernel<2, 4, 8, 16, 1, 3, 1>": ["r06_pmc_fc1_fetch.json", "r05_pmc_fc1_fetch.json"],
             "gemv_kernel<1, 8, 16, 8, 0, 1, 1>": ["r06_pmc_fc2_fetch.json"]}


def roofline_entry(name: str, ent: dict) -> dict:
    """The bench line's roofline object for one kernel of the C2 step table: algorithmic bytes per launch / its mean
    launch time (HIP events on the engine stream in this run) against the HBM peak, traffic from the committed
    FETCH_SIZE pass of the same instantiation."""
    traffic, src = pmc_traffic(ent["kernel"])
    return {"kernel": f"{ent['kernel']} ({name})", "bound": "hbm", "achieved": ent["GBps"], "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ent["GBps"] / HBM_PEAK_GBS, 3), "traffic": traffic,
            "traffic_source": f"{src} (rocprofv3 FETCH_SIZE x2, bytes/launch)" if src else None,
            "avg_us": ent["us"], "bytes_per_launch": ent["bytes"], "launches_per_step": ent["launches_per_step"],
            "us_per_step": round(ent["us"] * ent["launches_per_step"], 1)}


def dominant_kernels(ktab: dict) -> tuple[dict, dict | None]:
    """(dominant, runner-up) roofline objects from the C2 step's kernel table: the dominant kernel is the one with the
    most GPU time per step (launch time x launches per step), as rocprof's --stats ranks it; the runner-up rides along
    (since round 6 the fused attention block and fc1 are within ~1 % of each other, so either can lead a run)."""
    ks = {k: v for k, v in ktab["kernels"].items() if "bytes" in v and "GBps" in v and "kernel" in v}
    if not ks:
        return None, None
    order = sorted(ks, key=lambda k: ks[k]["us"] * ks[k]["launches_per_step"], reverse=True)
    return roofline_entry(order[0], ks[order[0]]), (roofline_entry(order[1], ks[order[1]]) if len(order) > 1 else None)


def _time_fused(e, items, gran, run, reps: int) -> float:
    """us per launch of a fused launch kind (hand-off granules per layer): the 26 layers' launches back to
    back on the engine stream, each layer's granule area zeroed before the run (outside the events), so
    every launch waits for its own producers as in the decode step."""
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot = 0.0
    with torch.cuda.stream(e.stream):
        for r in range(reps + 1):
            gran.zero_()
            st.record(e.stream)
            for it in items:
                run(it)
            en.record(e.stream)
            en.synchronize()
            if r:
                tot += st.elapsed_time(en) * 1000.0
    return tot / (reps * len(items))


def pmc_traffic(kernel: str):
    """HBM bytes per launch of a kernel from the newest committed FETCH_SIZE pass of THIS instantiation
    (tools/gpu.sh round: rocprofv3 --pmc FETCH_SIZE over tools/pmc_driver.py, x2 gfx950 correction; a counter
    pass serialises dispatches, so it is not repeated inside the timed run). (None, None) when no profile of
    that instantiation is committed."""
    for name in PMC_FILES.get(kernel, []):
        path = os.path.join(REPO, "profiles", name)
        if not os.path.exists(path):
            continue
        with open(path) as f:
            d = json.load(f)
        if d.get("kernels") and all(kernel in k for k in d["kernels"]):
            return int(d["FETCH_SIZE_bytes_per_launch"]), f"profiles/{name}"
    return None, None


def time_decode_step(model, cond, steps: int = 64, n_new: int = N_NEW, at: int | None = None):
    """Decode-step time of a LIVE utterance (both CFG rows active) around its mean position.

    Prefills slot 0 with the bench conditioning (an n_new-frame utterance), runs to position Lc + at - steps/2
    (at = n_new / 2 by default), then times `steps` graph replays on the engine stream with HIP events. Returns
    (us per step, mean position).
    """
    from zonos_vibes_amd.engine import SamplingParams
    e = model.engine
    params = SamplingParams(temperature=0.0, cfg_scale=2.0)
    s_len = e.prefill(0, cond, None, n_new, params)
    lead = max(0, (n_new // 2 if at is None else at) - steps // 2)
    e.step(lead, slots=1)
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(e.stream):
        start.record(e.stream)
        e.step(steps, slots=1)
        end.record(e.stream)
    end.synchronize()
    assert e.slot_state(0)["active"], "slot finished inside the timed decode window"
    e.release(0)
    return start.elapsed_time(end) * 1000.0 / steps, s_len + lead + steps // 2


def kernel_table(model, cond, reps: int = 3) -> dict:
    """Every kernel of the C2 decode step at the utterance's mean position, timed on the engine stream
    with HIP events, each kind as all 26 layers' launches back to back (each weight from HBM, as in the
    step; a launch's time includes its boundary with the previous one); the fused launches with every
    layer's hand-off granules zeroed before the run (a re-run at the same position would otherwise find
    its own granules and skip the wait); heads and sampler as repeated single launches. Per kernel: avg
    us per launch, algorithmic bytes per launch, GB/s and fraction of HBM peak."""
    from zonos_vibes_amd.engine import SamplingParams
    e = model.engine
    s_len = e.prefill(0, cond, None, N_NEW, SamplingParams(temperature=0.0, cfg_scale=2.0))
    lead = (N_NEW + 8) // 2
    e.step(lead, slots=1)
    pos = s_len + lead
    form = e._segments(1, 1)[0][1]
    plan = e._plan(2, form)
    d, F, qkv_n = e.d, e.F, (e.H + 2 * e.Hkv) * e.hd
    kv = 2 * e.Hkv * e.hd * 2 * 2 * (pos + 1)  # K + V of both CFG rows, one layer
    gem = [it for kd, it in plan if kd == "gemv"]
    res = [it for it in gem if it[1] == _lib.EPI_RESIDUAL]
    kinds = {  # name: (launch items, algorithmic bytes per launch, rocprof instantiation)
        "out_proj": ([it for it in res if it[0].K == e.H * e.hd], d * d * 2, "gemv_kernel (out_proj)"),
        "fc1 (LN + SwiGLU)": ([it for it in gem if it[1] == _lib.EPI_SWIGLU], 2 * F * d * 2,
                              "gemv_kernel<2, 4, 8, 16, 1, 3, 1>"),
        "fc2": ([it for it in res if it[0].K == F], d * F * 2, "gemv_kernel<1, 8, 16, 8, 0, 1, 1>"),
        "heads (LN + logits)": ([it for it in gem if it[1] == _lib.EPI_LOGITS], 9 * 1025 * d * 2,
                                "gemv_kernel<2, 4, 8, 16, 1, 4, 1>"),
    }
    kinds = {k: v for k, v in kinds.items() if v[0]}
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {}
    with torch.cuda.stream(e.stream):
        for name, (items, nbytes, kname) in kinds.items():
            for it in items:
                e._run_gemv(it)
            st.record(e.stream)
            for _ in range(reps):
                for it in items:
                    e._run_gemv(it)
            en.record(e.stream)
            en.synchronize()
            us = st.elapsed_time(en) * 1000.0 / (reps * len(items))
            out[name] = dict(us=round(us, 2), bytes=nbytes, GBps=round(nbytes / us / 1e3, 1),
                             hbm_frac=round(nbytes / us / 1e3 / HBM_PEAK_GBS, 3), launches_per_step=len(items),
                             kernel=kname)
        blk = [it for kd, it in plan if kd == "attnblk"]
        if blk:
            us = _time_fused(e, blk, e.blk_gran, e._run_attn_block, reps)
            oproj = len(blk[0]) > 4 and blk[0][4] is not None
            nbytes = qkv_n * d * 2 + kv + (d * d * 2 if oproj else 0)
            what = "LN + QKV + RoPE + KV write + attention" + (" + out_proj + residual" if oproj else "")
            note = ("QKV and out_proj weights + the layer's K/V of both rows; the launch also prefetches fc1's head"
                    if oproj else "QKV weights + the layer's K/V of both rows; the launch also prefetches out_proj's weights")
            sl = blk[0][3]
            fm = 2 if sl & _lib.ATTNBLK_SPLIT else (1 if sl & _lib.ATTNBLK_SELF else 0)
            kname = f"attn_block_kernel<{sl & 255}, 1, {fm}, {'true' if oproj else 'false'}>"
            out[f"attn_block ({form}: {what})"] = dict(
                us=round(us, 2), bytes=nbytes, GBps=round(nbytes / us / 1e3, 1),
                hbm_frac=round(nbytes / us / 1e3 / HBM_PEAK_GBS, 3), launches_per_step=len(blk), note=note,
                kernel=kname)
        us, kind = _sampler_us(e, reps)
        out[f"sampler (CFG + penalty + argmax + FSM + next embedding; {kind})"] = dict(
            us=round(us, 2), bytes=2 * 9 * 1026 * 4, launches_per_step=1)
    e.check_errors()
    e.release(0)
    return {"pos": pos, "kernels": out}


def _sampler_us(e, reps: int) -> tuple[float, str]:
    """The sampler launches captured in one graph (a Python-side launch costs more than the kernel, so
    back-to-back launches from the host would time the host)."""
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n_s = 8 * reps
    _lib.check(e.lib.zmi_graph_begin(e.sptr), "graph_begin")
    try:
        for _ in range(n_s):
            e._sample(e.logits, None, 0, 0, 1)
    finally:
        g = ctypes.c_void_p()
        _lib.check(e.lib.zmi_graph_end(e.sptr, ctypes.byref(g)), "graph_end")
    _lib.check(e.lib.zmi_graph_launch(g.value, 1, e.sptr), "graph_launch")  # warm
    st.record(e.stream)
    _lib.check(e.lib.zmi_graph_launch(g.value, 1, e.sptr), "graph_launch")
    en.record(e.stream)
    en.synchronize()
    _lib.check(e.lib.zmi_graph_destroy(g.value))
    kind = "greedy: one workgroup per slot" if e._greedy_step(0, 1) else "per-codebook workgroups"
    return st.elapsed_time(en) * 1000.0 / n_s, kind


MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense fp16/bf16 MFMA
DAC_FLOP_PER_FRAME = 1_608_302_592  # DacDecoder MACs x 2 per frame (hooks), 44.1 kHz dims


def dac_encode_flop_per_frame() -> int:
    """Algorithmic FLOP of DacEncoder per 512-sample frame (2 x MACs of modeling_dac.py:444-475 at the
    44.1 kHz dims; the build's 3-tap polyphase strided convs do 1.5x the MACs of those convs)."""
    macs, t, c = 512 * 64 * 7, 512, 64
    for s in syn.DAC_ENC_STRIDES:
        macs += 3 * (c * c * 7 + c * c) * t      # 3 residual units
        macs += (2 * c) * c * (2 * s) * (t // s)  # strided conv
        t //= s
        c *= 2
    macs += 1024 * c * 3 * t
    return 2 * macs


def time_widened_rows(model, dev):
    """SURVEY.md §8f rows built this round, measured with HIP events on their own streams (not part of
    `value`): the prefix conditioner (v0.1 conditioner list, d = 2048, a 40-phoneme utterance) and DAC
    encode of a 5 s voice-clone prefix (430 frames, BASELINE configs[4])."""
    from zonos_vibes_amd.conditioning import PrefixConditioner, make_cond_dict, v01_transformer_conditioners
    d = model.config.backbone.d_model
    pc = PrefixConditioner(v01_transformer_conditioners(), d, dev)
    g = torch.Generator().manual_seed(0)
    pc.load_state_dict({k: (0.02 * torch.randn(sh, generator=g)).to(torch.bfloat16)
                        for k, sh in pc.param_shapes().items()})
    cd = make_cond_dict(phonemes="ðɪs ɪz ə bɛntʃmɑːk sɛntəns fɔːɹ ðə pɹɛfɪks kəndɪʃənɚ.",
                        speaker=torch.zeros(1, 128, dtype=torch.bfloat16), device=dev)
    out = pc.prepare_conditioning(cd)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    st.record()
    for _ in range(reps):
        pc.prepare_conditioning(cd)
    en.record()
    en.synchronize()
    cond_us = st.elapsed_time(en) * 1000.0 / reps
    ae = model.autoencoder
    frames = 430
    wav = (0.1 * torch.randn(1, 1, frames * DAC_HOP, generator=g)).to(dev)
    ae.encode(wav)
    torch.cuda.synchronize()
    st.record()
    for _ in range(3):
        ae.encode(wav)
    en.record()
    en.synchronize()
    enc_s = st.elapsed_time(en) / 1000.0 / 3
    tflops = dac_encode_flop_per_frame() * frames / enc_s / 1e12
    return {"prefix_conditioner": {"us_per_utterance": round(cond_us, 1), "rows": int(out.shape[0] * out.shape[1]),
                                   "note": "host row-table build + one zmi_prefix_condition launch"},
            "dac_encode": {"frames": frames, "ms": round(enc_s * 1e3, 2),
                           "frames_per_s": round(frames / enc_s, 1),
                           "roofline": {"bound": "mfma", "achieved": round(tflops, 1), "peak": MFMA_PEAK_TFLOPS,
                                        "unit": "TFLOP/s", "frac": round(tflops / MFMA_PEAK_TFLOPS, 4),
                                        "flop_per_frame": dac_encode_flop_per_frame()}}}


def utterance_breakdown(model, cond, n_new: int, chunk: int = 128) -> dict:
    """Wall time of one more C2 utterance split into phases (host clock, each phase bracketed by a
    stream synchronisation; not part of `value`)."""
    from zonos_vibes_amd.engine import SamplingParams
    e = model.engine
    params = SamplingParams(temperature=0.0, cfg_scale=2.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.prefill(0, cond, None, n_new, params)
    e.stream.synchronize()
    t1 = time.perf_counter()
    steps = 0
    while steps < n_new + 8:
        n = min(chunk, n_new + 8 - steps)
        e.step(n, slots=1)
        steps += n
        if not e.slot_state(0)["active"]:
            break
    t2 = time.perf_counter()
    codes = e.read_codes(0)
    e.release(0)
    t3 = time.perf_counter()
    model.autoencoder.decode(codes)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    return {"prefill_ms": round((t1 - t0) * 1e3, 2), "decode_loop_ms": round((t2 - t1) * 1e3, 2),
            "readback_ms": round((t3 - t2) * 1e3, 2), "dac_decode_ms": round((t4 - t3) * 1e3, 2)}


def step_bytes(model, pos: int) -> int:
    e = model.engine
    qkv = (e.H + 2 * e.Hkv) * e.hd
    w = e.L * 2 * (qkv * e.d + e.d * e.H * e.hd + 2 * e.F * e.d + e.d * e.F) + 9 * 1025 * e.d * 2
    kv = 2 * e.L * e.Hkv * e.hd * 2 * 2 * (pos + 1)
    return w + kv


def hybrid_step_bytes(e, pos: int) -> int:
    """Algorithmic HBM bytes of one hybrid decode step (2 CFG rows): every weight once, each Mamba2 layer's
    SSM state read + written (2 rows x nheads x 64 x 128 bf16) and conv ring slot traffic, the attention
    layers' K / V up to pos."""
    md, d = e.md, e.d
    n_attn = len(e.attn_idx)
    n_mamba = e.L - n_attn
    qkv = (e.H + 2 * e.Hkv) * e.hd
    w_m = md["d_in_proj"] * d + d * md["d_ssm"] + md["conv_dim"] * (md["d_conv"] + 1) + md["d_ssm"]
    w_a = qkv * d + d * e.H * e.hd
    w = 2 * (n_mamba * w_m + n_attn * w_a + e.L * 2 * d) + 9 * 1025 * d * 2
    state = n_mamba * 2 * (2 * md["nheads"] * md["headdim"] * md["d_state"] * 2 + 4 * md["conv_dim"] * 2)
    kv = n_attn * 2 * e.Hkv * e.hd * 2 * 2 * (pos + 1)
    return w + state + kv


def time_default_capacity(dev, n_new: int, ref_codes) -> dict:
    """The C2 utterance through a model whose engine is sized for the reference's default
    generate(max_new_tokens=86 * 30) (reference zonos/model.py:223): the decode forms are picked per step from
    the rows' positions, not from the capacity, so the step and the codes must match the C2 line's."""
    from zonos_vibes_amd.model import Zonos
    cfg = zonos_v01_transformer()
    cap = 86 * 30
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=LC + cap + 9, max_prefill=LC + 1)
    cond = cond_tensor(1, cfg.backbone.d_model, dev)

    def one():
        codes = m.generate(cond, max_new_tokens=n_new, sampling_params=dict(temperature=0.0), progress_bar=False,
                           chunk=128)
        return codes, m.autoencoder.decode(codes)

    one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    codes, _ = one()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    us, pos = time_decode_step(m, cond)
    out = {"config": f"C2 utterance ({n_new} frames, greedy, EOS suppressed) through an engine sized for the reference "
                     f"default max_new_tokens={cap} (KV capacity {m.engine.smax} positions)",
           "rtf": round(n_new * DAC_HOP / DAC_SAMPLE_RATE / el, 3), "utterance_ms": round(el * 1e3, 1),
           "decode_step_us": round(us, 1), "decode_step_pos": pos,
           "codes_equal_c2": bool(torch.equal(codes, ref_codes))}
    del m
    torch.cuda.empty_cache()
    return out


def time_long_utterance(dev, n_new: int = 86 * 30, engine_opts: dict | None = None) -> dict:
    """One batch-1 utterance at the reference's default generate(max_new_tokens=86 * 30) (model.py:223: 30 s of
    audio, contexts to Lc + 2580 positions): wall-clock RTF of generate() + DAC decode, and the decode step at
    positions across the utterance (HIP events, 64 steps each) with the attention form the plan picks there."""
    import hashlib
    from zonos_vibes_amd.model import Zonos
    cfg = zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=LC + n_new + 9, max_prefill=LC + 1)
    for k, v in (engine_opts or {}).items():  # A/B knobs (tools/bench_long.py)
        if k.startswith("opt_"):  # library launch knobs: opt_attnblk_spread -> zmi_set_option(OPT_ATTNBLK_SPREAD)
            _lib.check(m.engine.lib.zmi_set_option(getattr(_lib, "OPT_" + k[4:].upper()), int(v)), k)
        else:
            setattr(m.engine, k, tuple(v) if isinstance(v, list) else v)
    m.engine._build_plan()
    cond = cond_tensor(1, cfg.backbone.d_model, dev)

    def one():
        codes = m.generate(cond, max_new_tokens=n_new, sampling_params=dict(temperature=0.0), progress_bar=False,
                           chunk=128)
        return codes, m.autoencoder.decode(codes)

    one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    codes, _ = one()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    steps = {}
    for at in (430, 1000, 1200, 1600, 2000, 2500):
        us, pos = time_decode_step(m, cond, n_new=n_new, at=at)
        m.engine.pos_hi[0] = pos
        steps[str(pos)] = {"us": round(us, 1), "form": m.engine._segments(1, 1)[0][1]}
    out = {"config": f"batch 1, Lc {LC}, {n_new} new frames (30 s: the reference default max_new_tokens), greedy, EOS "
                     f"suppressed, + DAC decode", "rtf": round(n_new * DAC_HOP / DAC_SAMPLE_RATE / el, 3),
           "utterance_ms": round(el * 1e3, 1), "frames": int(codes.shape[-1]),
           "codes_sha256_16": hashlib.sha256(codes.cpu().numpy().tobytes()).hexdigest()[:16],
           "decode_step_us_by_position": steps}
    del m
    torch.cuda.empty_cache()
    return out


def time_hybrid(dev, n_new: int) -> dict:
    """BASELINE config C4 (Zonos-v0.1-hybrid, batch 1, one GPU): one C2-shaped utterance (Lc 160, n_new
    frames, greedy, EOS suppressed) through generate() + DAC decode, wall-clock RTF, and the decode step
    at the utterance's mean position (HIP events) against the step's algorithmic HBM bytes."""
    from zonos_vibes_amd.config import zonos_v01_hybrid
    from zonos_vibes_amd.engine import SamplingParams
    from zonos_vibes_amd.model import Zonos
    cfg = zonos_v01_hybrid()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=LC + n_new + 9, max_prefill=LC + 1)
    cond = cond_tensor(1, cfg.backbone.d_model, dev)

    def one():
        codes = m.generate(cond, max_new_tokens=n_new, sampling_params=dict(temperature=0.0), progress_bar=False,
                           chunk=128)
        return codes, m.autoencoder.decode(codes)

    one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    codes, wav = one()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert codes.shape[-1] == n_new
    e = m.engine
    e.prefill(0, cond, None, n_new, SamplingParams(temperature=0.0))
    e.release(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s_len = e.prefill(0, cond, None, n_new, SamplingParams(temperature=0.0))  # the Lc + 1 = 161-row prefill
    torch.cuda.synchronize()
    prefill_ms = (time.perf_counter() - t0) * 1e3
    lead, steps = max(0, n_new // 2 - 32), 64
    e.step(lead, slots=1)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(e.stream):
        st.record(e.stream)
        e.step(steps, slots=1)
        en.record(e.stream)
    en.synchronize()
    e.release(0)
    us = st.elapsed_time(en) * 1000.0 / steps
    pos = s_len + lead + steps // 2
    b = hybrid_step_bytes(e, pos)
    out = {"config": f"C4: Zonos-v0.1-hybrid dims (46 layers: 41 Mamba2 + MHA at 9/18/27/36/45), batch 1, Lc={LC}, "
                     f"{n_new} frames, greedy, EOS suppressed, + DAC decode",
           "rtf": round(n_new * DAC_HOP / DAC_SAMPLE_RATE / el, 3), "utterance_ms": round(el * 1e3, 1),
           "prefill_ms": round(prefill_ms, 2), "prefill_rows": 2 * s_len,
           "decode_step_us": round(us, 1), "decode_step_pos": pos, "step_bytes": b,
           "decode_step_hbm_frac": round(b / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 3),
           "parity": "unpinned (mamba-ssm absent); held to oracle/hybrid_cpu.py by tests/test_gpu_hybrid.py"}
    del m, e
    torch.cuda.empty_cache()
    return out


def time_batch(model, dev, n_utt: int = 64, slots: int = 64) -> dict:
    """A bounded C3-shaped sample on one GPU: n_utt independent utterances of 2-6 s (Lc = 8 + 15 s, as
    SURVEY.md §8d C3 draws them, shorter so the run stays short) through `slots` continuous-batching
    slots (generate_batch: LPT order, slot refill at chunk boundaries), greedy, EOS suppressed, + DAC
    decode of every utterance. Aggregate real-time factor = total audio s / wall s. Runs last: it grows
    the engine to `slots` slots."""
    g = torch.Generator().manual_seed(7)
    secs = (2.0 + 4.0 * torch.rand(n_utt, generator=g)).tolist()
    d = model.config.backbone.d_model
    conds = [cond_tensor(100 + i, d, dev)[:, : 8 + round(15 * s)].contiguous() for i, s in enumerate(secs)]
    n_new = [max(1, round(s * DAC_SAMPLE_RATE / DAC_HOP)) for s in secs]
    sp = dict(temperature=0.0)
    model.generate_batch(conds[:2], max_new_tokens=[16, 16], sampling_params=sp, seeds=[0, 1], max_slots=slots)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = model.generate_batch(conds, max_new_tokens=n_new, sampling_params=sp, seeds=list(range(n_utt)),
                               max_slots=slots)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for c in out:
        model.autoencoder.decode(c)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    frames = sum(int(c.shape[-1]) for c in out)
    assert frames == sum(n_new)
    audio = frames * DAC_HOP / DAC_SAMPLE_RATE
    return {"config": f"C3 sample: {n_utt} utterances of 2-6 s (Lc 8 + 15 s), {slots} slots on one GPU, greedy, "
                      f"EOS suppressed, + DAC decode per utterance",
            "rtf": round(audio / (t2 - t0), 2), "audio_s": round(audio, 1), "generate_s": round(t1 - t0, 3),
            "dac_s": round(t2 - t1, 3), "frames_per_s": round(frames / (t2 - t0), 1)}


def c3_job(n_utt: int = 512) -> tuple[list[int], list[int]]:
    """BASELINE config C3: 512 utterances, utterance i seeded by i: length uniform 2-30 s
    (N = round(s * 44100 / 512) frames), Lc = 8 + round(15 s) conditioning rows. Returns (Lc, N) lists."""
    lcs, n_new = [], []
    for i in range(n_utt):
        sec = 2.0 + 28.0 * float(torch.rand(1, generator=torch.Generator().manual_seed(i)))
        lcs.append(8 + round(15 * sec))
        n_new.append(max(1, round(sec * DAC_SAMPLE_RATE / DAC_HOP)))
    return lcs, n_new


def time_c3_sharded(model, dev, rank: int, world: int, dist, per_gpu: int = 64, cdev=None) -> dict:
    """C3 batch-sharded throughput (north_star): the first per_gpu x world of
    the 512 C3 utterances (all 512 at 8 GPUs; per-GPU work fixed as the rank count grows), LPT-sharded
    over the ranks with no communication (shard.generate_sharded: 64 continuous-batching slots per GPU),
    DAC decode of every utterance on its rank, then the end-of-batch gather of the codes to rank 0
    (int16 over RCCL). Aggregate real time = total audio s / max-over-ranks wall."""
    from zonos_vibes_amd.shard import estimated_frames, generate_sharded, lpt_assign
    d = model.config.backbone.d_model
    lcs, n_all = c3_job()
    n_utt = min(len(lcs), per_gpu * world)
    lcs, n_new = lcs[:n_utt], n_all[:n_utt]
    conds = [cond_tensor(1000 + i, d, dev, lc) for i, lc in enumerate(lcs)]
    mine_plan = lpt_assign(estimated_frames(conds, [None] * n_utt, n_new), world)[rank]
    # grow the engine to this job's capacity and capture its 64-slot graph outside the timed region
    model._ensure_capacity(per_gpu, max(lcs) + max(n_new) + 9, max(lcs) + 1)
    warm = min(per_gpu, n_utt)
    model.generate_batch(conds[:warm], max_new_tokens=[4] * warm, sampling_params=dict(temperature=0.0),
                         seeds=list(range(warm)), max_slots=per_gpu)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    mine, local, _ = generate_sharded(model, conds, max_new_tokens=n_new, sampling_params=dict(temperature=0.0),
                                      seeds=list(range(n_utt)), gather=False, max_slots=per_gpu)
    for c in local:
        model.autoencoder.decode(c)
    torch.cuda.synchronize()
    busy = time.perf_counter() - t0
    g0 = time.perf_counter()
    gathered = None
    if dist:
        # a failure here is fatal: a rank that raises leaves the others inside a collective, so the run ends and
        # torch.distributed.run reports it, rather than the ranks meeting at a barrier that never completes
        from zonos_vibes_amd.shard import gather_codes
        gathered = gather_codes(local, mine, n_utt, 0, None, cdev or dev)
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gather_ms = (time.perf_counter() - g0) * 1e3
    assert mine == mine_plan
    frames = sum(int(c.shape[-1]) for c in local)
    assert frames == sum(n_new[i] for i in mine)
    stats = torch.tensor([wall, busy, frames], dtype=torch.float64, device=cdev or dev)
    if dist:
        allv = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allv, stats)
    else:
        allv = [stats]
    walls = [float(v[0]) for v in allv]
    busys = [float(v[1]) for v in allv]
    audio = sum(float(v[2]) for v in allv) * DAC_HOP / DAC_SAMPLE_RATE
    res = {"config": f"C3: utterances 0..{n_utt - 1} of the 512-utterance C3 set (2-30 s, Lc 8 + 15 s, seed i), "
                     f"LPT over {world} GPU(s), {per_gpu} slots per GPU, greedy, EOS suppressed, + DAC decode; "
                     f"end-of-batch code gather to rank 0 ({'int16 over RCCL' if dist else 'none: one rank'})",
           "utterances": n_utt, "audio_s": round(audio, 1), "rtf": round(audio / max(walls), 2),
           "rtf_per_gpu": round(audio / max(walls) / world, 2),
           "wall_s": round(max(walls), 3), "busy_s_per_rank": [round(b, 3) for b in busys],
           "lpt_tail": round(max(busys) / (sum(busys) / len(busys)), 3), "gather_ms": round(gather_ms, 1)}
    if rank == 0 and dist:
        res["gathered_utterances"] = len(gathered) if gathered is not None else 0
    return res


def time_c5(dev, slots: int = 8, n_new: int = 5168, prefix: int = 430, engine_opts: dict | None = None) -> dict:
    """One GPU's share of BASELINE config C5 (voice clone, long form): `slots` utterances of n_new frames
    (60 s) after a `prefix`-frame audio prompt (random codes), Lc = 160, greedy, EOS suppressed, through
    `slots` slots (contexts grow to Lc + prefix + n_new ~ 5.8k positions), then DAC decode of every
    utterance's prefix + new frames. A fresh engine sized for the job."""
    from zonos_vibes_amd.model import Zonos
    cfg = zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_slots=slots, max_seqlen=LC + prefix + n_new + 9,
                        max_prefill=LC + prefix + 1)
    for k, v in (engine_opts or {}).items():  # A/B knobs (tools/bench_c5.py)
        if k.startswith("opt_"):  # library launch knobs: opt_gemm_rows -> zmi_set_option(OPT_GEMM_ROWS)
            _lib.check(m.engine.lib.zmi_set_option(getattr(_lib, "OPT_" + k[4:].upper()), int(v)), k)
        else:
            setattr(m.engine, k, v)
    m.engine._build_plan()
    g = torch.Generator().manual_seed(11)
    conds = [cond_tensor(200 + i, cfg.backbone.d_model, dev) for i in range(slots)]
    prefixes = [torch.randint(0, 1024, (1, 9, prefix), generator=g).to(dev) for _ in range(slots)]
    sp = dict(temperature=0.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = m.generate_batch(conds, prefixes, max_new_tokens=n_new, sampling_params=sp, seeds=list(range(slots)),
                           max_slots=slots)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for c in out:
        m.autoencoder.decode(c)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    frames = sum(int(c.shape[-1]) for c in out)
    assert frames == slots * (prefix + n_new)
    new_audio = slots * n_new * DAC_HOP / DAC_SAMPLE_RATE
    res = {"config": f"C5 share of one GPU: {slots} voice-clone utterances, {prefix}-frame audio prefix + {n_new} new "
                     f"frames (60 s), Lc {LC}, {slots} slots, greedy, EOS suppressed, + DAC decode of "
                     f"{slots} x {prefix + n_new} frames",
           "rtf_new_audio": round(new_audio / (t2 - t0), 2), "generate_s": round(t1 - t0, 2),
           "dac_s": round(t2 - t1, 3), "dac_frames_per_s": round(frames / (t2 - t1), 1),
           "decode_steps": n_new + 8, "ms_per_step": round((t1 - t0) / (n_new + 8) * 1e3, 3)}
    del m
    torch.cuda.empty_cache()
    return res


def cpu_cores() -> int:
    """CPU threads this process may use: its affinity set, capped by OMP_NUM_THREADS when the host sets one
    (the GPU box gives each GPU process a 16-thread share of its host CPUs and sets OMP_NUM_THREADS=16)."""
    n = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


def cpu_info() -> dict:
    """Host CPU model and counts, for the CPU-baseline line."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "host_logical_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(dev_weights: dict, cfg, budget_s: float = 20.0):
    """The oracle (PyTorch eager CPU, same op order as the reference) on a bounded sample of C2: the
    prefill (2 x 161 rows), decode steps around the C2 mean position (p ~ 591) with the KV cache
    filled to there, and DAC decode frames; extrapolated to the whole utterance."""
    from oracle.dac_cpu import OracleDAC
    from oracle.zonos_cpu import OracleZonos, apply_delay_pattern
    threads = cpu_cores()
    torch.set_num_threads(threads)
    w = {k: v.cpu() for k, v in dev_weights.items()}
    m = OracleZonos(cfg, w)
    cond = cond_tensor(1, cfg.backbone.d_model, "cpu")
    mean_pos = LC + 1 + (N_NEW + 8) // 2
    with torch.inference_mode():
        cache = m.new_cache(2, LC + N_NEW + 9)
        delayed = apply_delay_pattern(torch.full((1, 9, N_NEW), -1), 1025)
        t0 = time.perf_counter()
        m.prefill(cond, delayed[..., :1], cache, 2.0)
        t_pre = time.perf_counter() - t0
        for kv in cache["kv"]:  # positions up to the sample window hold cache values (cost is data-independent)
            kv[:, LC + 1: mean_pos + 32].normal_()
        n_pre = mean_pos - 100  # decode steps centred on the mean position: 100 either side at most
        cache["offset"] = n_pre
        cache["lengths"][:] = n_pre
        n, t0 = 0, time.perf_counter()
        ids = torch.randint(0, 1024, (1, 9, 1))
        while n < 8 or (time.perf_counter() - t0 < budget_s * 0.6 and n < 200):
            m.decode_one(ids, cache, torch.tensor(2.0))
            cache["offset"] += 1
            cache["lengths"][:] += 1
            n += 1
        t_step = (time.perf_counter() - t0) / n
        p_lo, p_hi = n_pre, n_pre + n - 1
        dac = OracleDAC({k: v for k, v in _dac_weights_cpu().items()})
        nf = 215
        t0 = time.perf_counter()
        dac.decode(torch.randint(0, 1024, (1, 9, nf)))
        t_dac = (time.perf_counter() - t0) / nf
    total = t_pre + (N_NEW + 8) * t_step + N_NEW * t_dac
    audio = N_NEW * DAC_HOP / DAC_SAMPLE_RATE
    return {"value": round(audio / total, 4), "unit": "x realtime (audio s / CPU s), extrapolated",
            "cores": threads, "kind": "port",
            "sample": f"C2 prefill (2x{LC + 1} rows) {t_pre:.2f}s + {n} decode steps at positions {p_lo}..{p_hi} "
                      f"(C2 mean {mean_pos}; {t_step * 1e3:.1f} ms/step, x{N_NEW + 8}) + DAC decode of {nf} of "
                      f"{N_NEW} frames ({t_dac * 1e3:.1f} ms/frame), extrapolated to the full utterance; "
                      f"{threads} threads = this GPU process's share of the host CPUs (the box runs one GPU per "
                      f"16-thread share and sets OMP_NUM_THREADS=16)", **cpu_info()}


def _dac_weights_cpu():
    return dict(syn.iter_torch_cpu(syn.dac_specs(), 0))


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher around it: run N ranks of this same command line under
    torch.distributed.run (127.0.0.1 rendezvous, a free port) as a child process; returns its exit status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dry_run(args, rank: int, world: int) -> None:
    """The multi-rank harness without a GPU (gloo, CPU tensors): the C3 set's LPT plan over `world` ranks
    (shard.lpt_assign, as time_c3_sharded uses it), a stand-in generator that emits placeholder codes of each
    utterance's length (no kernel, no oracle: this checks the plumbing, not the decode), the barrier-bracketed
    timing reduced as the max over ranks, and the end-of-batch gather (shard.gather_codes) to rank 0. Rank 0
    prints one JSON line with the world it saw and the gathered utterance count."""
    import datetime

    import torch.distributed as dist

    from zonos_vibes_amd.shard import gather_codes, lpt_assign
    dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=5))
    try:
        per_gpu = 8
        lcs, n_all = c3_job()
        n_utt = min(len(lcs), per_gpu * world)
        costs = [n + 8 + lc + 1 for lc, n in zip(lcs[:n_utt], n_all[:n_utt])]
        mine = lpt_assign(costs, world)[rank]
        dist.barrier()
        t0 = time.perf_counter()
        local = [torch.full((1, 9, n_all[i]), i % 1024, dtype=torch.long) for i in mine]
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        fr = torch.tensor([sum(int(c.shape[-1]) for c in local)], dtype=torch.float64)
        dist.all_reduce(fr)
        got = gather_codes(local, mine, n_utt, 0)
        if rank == 0:
            ok = got is not None and all(int(c[0, 0, 0]) == i % 1024 and c.shape[-1] == n_all[i] for i, c in enumerate(got))
            print(json.dumps({"dry_run": True, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                              "backend": "gloo", "wall_s_max_over_ranks": round(float(t.item()), 6),
                              "c3_sharded": {"utterances": n_utt, "frames": int(fr.item()),
                                             "gathered_utterances": 0 if got is None else len(got),
                                             "gathered_in_order": bool(ok)}}), flush=True)
    finally:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--new-tokens", type=int, default=N_NEW)
    ap.add_argument("--no-hybrid", action="store_true", help="skip the C4 hybrid-backbone line in `widened`")
    ap.add_argument("--no-batch", action="store_true", help="skip the C3-sample batch line in `widened`")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 (voice clone, 60 s, 8 slots) line in `widened`")
    ap.add_argument("--no-default-cap", action="store_true",
                    help="skip the line with the engine sized for the reference default max_new_tokens")
    ap.add_argument("--c3-per-gpu", type=int, default=64, help="C3 utterances (and slots) per GPU in `c3_sharded`")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="rehearsal of the N-rank GPU run on a one-GPU box: every rank on cuda:0, gloo collectives on "
                         "CPU tensors (timings are not per-GPU numbers)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU / gloo rehearsal of the multi-rank harness (launcher, world check, LPT plan of the C3 "
                         "set, timing reductions, end-of-batch gather) with placeholder codes; runs no kernel")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: start the N ranks as a child torch.distributed.run (this parent touches no GPU) and
        # exit with its status
        raise SystemExit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started {world} rank(s)")
    if args.dry_run:
        return dry_run(args, rank, world)
    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu") if args.rehearse_one_gpu else dev  # where the collectives' tensors live
    dist = None
    if world > 1:
        import datetime

        import torch.distributed as dist
        # rank 0 alone runs the widened lines; the other ranks wait at the next barrier for that long
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=45))
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(minutes=45))

    from zonos_vibes_amd.model import Zonos
    cfg = zonos_v01_transformer()
    n_new = args.new_tokens
    model = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=LC + n_new + 9, max_prefill=LC + 1)
    cond = cond_tensor(1 + rank, cfg.backbone.d_model, dev)
    params = dict(temperature=0.0)

    def one_utterance():
        codes = model.generate(cond, max_new_tokens=n_new, sampling_params=params, progress_bar=False, chunk=128)
        wav = model.autoencoder.decode(codes)
        return codes, wav

    for _ in range(max(1, args.warmup)):
        codes, wav = one_utterance()
    torch.cuda.synchronize()
    ref_codes = codes.clone()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    frames = 0
    timed_codes = []
    for _ in range(args.steps):
        codes, wav = one_utterance()
        frames += codes.shape[-1]
        timed_codes.append(codes)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    assert codes.shape[-1] == n_new and wav.shape[-1] == n_new * DAC_HOP, (codes.shape, wav.shape)
    # every timed utterance decoded exactly the warm-up's codes (greedy: a silent change fails the run)
    for c in timed_codes:
        if not torch.equal(c, ref_codes):
            raise SystemExit("bench: a timed utterance's codes differ from the warm-up's (non-deterministic decode)")
    import hashlib
    codes_sha = hashlib.sha256(ref_codes.cpu().numpy().tobytes()).hexdigest()[:16]
    if dist:
        t = torch.tensor([elapsed], device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        fr = torch.tensor([frames], device=cdev, dtype=torch.float64)
        dist.all_reduce(fr)
        frames = int(fr.item())
    audio_s = frames * DAC_HOP / DAC_SAMPLE_RATE
    rtf = audio_s / elapsed

    # optional end-of-batch gather of every rank's codes to rank 0 (outside the timed
    # region): int16 payload over RCCL/xGMI
    gather = None
    if dist:
        from zonos_vibes_amd.shard import gather_codes
        g0 = time.perf_counter()  # fatal on failure (see time_c3_sharded)
        got = gather_codes([codes], [rank], world, device=cdev)
        torch.cuda.synchronize()
        gather = {"ok": True, "ms": round((time.perf_counter() - g0) * 1e3, 2)}
        if rank == 0:
            gather["frames_gathered"] = int(sum(c.shape[-1] for c in got))

    # kernel-level measurement (outside the timed region)
    step_us, step_pos = time_decode_step(model, cond)
    ktab = kernel_table(model, cond)
    roof, roof_next = dominant_kernels(ktab)
    widened = time_widened_rows(model, dev)
    if rank == 0 and not args.no_default_cap:
        widened["default_capacity"] = time_default_capacity(dev, n_new, ref_codes)
        widened["batch1_30s"] = time_long_utterance(dev)
    if rank == 0 and not args.no_hybrid:
        widened["hybrid_c4"] = time_hybrid(dev, n_new)
    if rank == 0 and not args.no_c5:
        widened["c5_share"] = time_c5(dev)
    breakdown = utterance_breakdown(model, cond, n_new)
    dac_tf = DAC_FLOP_PER_FRAME * n_new / (breakdown["dac_decode_ms"] * 1e-3) / 1e12
    c3 = None
    if not args.no_batch:
        c3 = time_c3_sharded(model, dev, rank, world, dist, per_gpu=args.c3_per_gpu, cdev=cdev)  # last: grows the engine
    out = None
    if rank == 0:
        out = {
            "metric": "real-time factor (44kHz audio s/compute s) + DAC tokens/s/GPU, Zonos-transformer",
            "value": round(rtf, 3), "unit": "x realtime (audio s / wall s, all GPUs)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(rtf / BASELINE_RTF, 3),
            "dtype": "bf16", "data": "synthetic",
            "config": {"workload": f"C2: batch=1 per GPU, Lc={LC}, {n_new} frames ({n_new * DAC_HOP / DAC_SAMPLE_RATE:.2f}"
                                   f" s audio), greedy + rep. penalty, EOS suppressed, + DAC decode",
                       "global_batch": world, "seq_len": LC + n_new + 9, "parallelism": f"dp{world} (utterance-sharded)",
                       "decode_steps": n_new + 8},
            "dac_tokens_per_s_per_gpu": round(frames * 9 / elapsed / world, 1),
            "frames_per_s_per_gpu": round(frames / elapsed / world, 1),
            "decode_step_us": round(step_us, 1), "decode_step_pos": step_pos,
            "decode_step_hbm_frac": round(step_bytes(model, step_pos) / (step_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 3),
            "roofline": roof,
            "roofline_next": roof_next,
            "codes_sha256_16": codes_sha,
            "c2_step_kernels": ktab,
            "utterance_breakdown": breakdown,
            "dac_decode_roofline": {"bound": "mfma", "achieved": round(dac_tf, 1), "peak": MFMA_PEAK_TFLOPS,
                                    "unit": "TFLOP/s", "frac": round(dac_tf / MFMA_PEAK_TFLOPS, 4),
                                    "flop_per_frame": DAC_FLOP_PER_FRAME, "frames": n_new,
                                    "ms": breakdown["dac_decode_ms"],
                                    "mfma_busy_source": "profiles/r06_dac_mfma_pmc.json (SQ_VALU_MFMA_BUSY_CYCLES pass)"},
            "c3_sharded": c3,
            "widened": widened,
            "end_of_batch_gather": gather,
        }
        if world == 1 and not args.no_cpu_baseline:
            sd = {}
            for sp in syn.zonos_specs(cfg):
                t = torch.empty(sp.shape, dtype=torch.bfloat16, device=dev)
                _lib.check(_lib.lib().zmi_fill_uniform(t.data_ptr(), sp.numel, syn.tensor_key(0, sp.name), sp.scale,
                                                       sp.offset, 0, torch.cuda.current_stream().cuda_stream))
                sd[sp.name] = t
            sd["heads.0.weight"][1024] = 0
            torch.cuda.synchronize()
            out["cpu_baseline"] = cpu_baseline(sd, cfg)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
