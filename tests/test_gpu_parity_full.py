"""Full-depth parity at the headline model: Zonos-v0.1-transformer dims (26 layers, d 2048, 16/4
heads, FFN 8192), C2 conditioning (Lc = 160), synthetic weights — the HIP path against the
REFERENCE's own outputs (tests/golden/full_model.safetensors, make_golden_full.py).

At these dims the reference is not reproducible against itself: its greedy trajectory at 1 or 3
CPU threads leaves the 8-thread one at delayed frame 3, and its teacher-forced logits differ
between thread counts by up to ~10 bf16 ulps of the top score (fixture metadata `self_noise`:
its GEMM blocking changes the fp32 accumulation order); the same model with exact (fp64) GEMMs differs
from it by 7.5 ulps mean, 11.9 max (fixture metadata `exact_gemm_noise`). The HIP path is held to the
larger of the two scales:

  * teacher-forced logits (prefill + 16 steps): error in bf16 ulps of each decision's top score,
    mean and max no larger than the reference's own thread-count noise allows;
  * every greedy decision along the reference trajectory whose margin exceeds twice the
    reference's self-noise must be identical (teacher-forced, so one near-tie cannot hide the rest);
  * free-running generate(): identical codes up to the first decision the reference itself leaves
    undetermined (margin within its self-noise), never a divergence at a determined decision.
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from tests.helpers import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ulp(x: torch.Tensor) -> torch.Tensor:
    return torch.ldexp(torch.ones_like(x), torch.frexp(x.abs().clamp_min(1e-30))[1] - 8)


def _cfg_logits(rows):
    c, u = rows[0].float().cpu(), rows[1].float().cpu()
    lg = u + (c - u) * 2.0
    lg[..., 1025:] = -torch.inf
    return lg


@pytest.fixture(scope="module")
def full():
    from zonos_vibes_amd import synthetic as syn
    from zonos_vibes_amd.config import ZonosConfig
    from zonos_vibes_amd.model import Zonos
    t, meta = load_golden("full_model")
    cfg = ZonosConfig.from_dict(meta["cfg"])
    lc, n = meta["lc"], meta["n"]
    cond = torch.from_numpy(syn.synthetic_conditioning_np(meta["cond_seed"], 2, lc, cfg.backbone.d_model)
                            .view(np.int16).copy()).view(torch.bfloat16)
    model = Zonos.synthetic(cfg, DEV, seed=meta["weights_seed"], zero_eos=meta["zero_eos"],
                            max_seqlen=lc + n + 24, max_prefill=lc + 8)
    yield model, t, meta, cond
    del model
    torch.cuda.empty_cache()


def test_full_depth_teacher_forced_logits_and_decisions(full):
    from oracle.zonos_cpu import apply_delay_pattern, repetition_penalty
    from zonos_vibes_amd.engine import SamplingParams
    model, t, meta, cond = full
    e = model.engine
    n = meta["n"]
    noise = meta["self_noise"]
    e.prefill(0, cond.to(DEV), None, n, SamplingParams(temperature=0.0))
    e.stream.synchronize()
    delayed = apply_delay_pattern(t["codes"], 1025)[0]
    with torch.cuda.stream(e.stream):
        e.delayed[0, :, : delayed.shape[-1]] = delayed.to(DEV, torch.int32)
        e.refresh_inputs()
    logits = [_cfg_logits(e.logits_pre)]
    scores = [logits[0]]
    bias = torch.zeros(9, 1026)
    bias[1:, 1024] = -torch.inf
    for s in range(n + 8):
        o = int(e.st["offset"][0].item())
        e.step(1, use_graph=False, slots=1)
        e.stream.synchronize()
        lg = _cfg_logits(e.logits[0:2])
        if s < meta["teacher_forced_steps"]:
            logits.append(lg)
        scores.append(repetition_penalty((lg + bias).unsqueeze(0), delayed[None, :, : o + 1], 3.0, 2)[0])
    e.check_errors()
    # the yardstick: the reference's own thread-count noise, or (if larger) the noise of the same model
    # with exact fp64 GEMMs — what a different GEMM accumulation order alone does to these logits
    if "exact_gemm_noise" in meta and meta["exact_gemm_noise"]["max_ulps"] > noise["max_ulps"]:
        noise = dict(meta["exact_gemm_noise"], source="exact_gemm")
    ref = [t["prefill"]] + list(t["steps"])
    errs = []
    for got, r in zip(logits, ref):
        fin = torch.isfinite(r)
        assert torch.equal(fin, torch.isfinite(got))
        top = r.masked_fill(~fin, -torch.inf).max(-1).values
        errs.append((got - r).masked_fill(~fin, 0).abs().max(-1).values / _ulp(top))
    errs = torch.cat(errs)
    floor = 2 * noise["max_ulps"]
    det = t["margin"] > floor * _ulp(t["top"])
    got_arg = torch.stack([sc.argmax(-1) for sc in scores])  # [decisions, 9]
    # the reference's choices along its trajectory: decision i wrote frame i + 1 by
    # masked_scatter_ into the codebooks still unknown there (model.py:258-260,296-297), in order
    init = apply_delay_pattern(torch.full((1, 9, n), -1), 1025)[0]
    agree = torch.ones_like(det)
    used = torch.zeros_like(det)
    for i in range(min(got_arg.shape[0], init.shape[1] - 1)):  # the last decision writes no frame
        unk = (init[:, i + 1] == -1).nonzero().flatten().tolist()
        for m, k in enumerate(unk):
            used[i, m] = True
            agree[i, m] = bool(got_arg[i, m] == delayed[k, i + 1])
    det = det & used
    stats = dict(mean_err_ulps=float(errs.mean()), max_err_ulps=float(errs.max()),
                 ref_self_noise=meta["self_noise"], ref_exact_gemm_noise=meta.get("exact_gemm_noise"),
                 yardstick=noise, decisions=int(used.sum()), agree=int((agree & used).sum()),
                 determined=int(det.sum()), determined_disagreements=int((det & ~agree).sum()))
    if os.path.isdir("gpurun_out"):
        json.dump(stats, open("gpurun_out/full_parity.json", "w"), indent=1)
    assert stats["determined_disagreements"] == 0, stats
    assert errs.mean() <= 1.5 * noise["mean_ulps"], stats
    assert errs.max() <= 2 * noise["max_ulps"], stats
    # regression guard against the HIP path's own recorded error (deterministic kernels; see
    # test_full_depth_per_layer_error): tighter than the reference-noise yardstick above
    base = _hip_baseline()
    if base is not None:
        assert errs.mean() <= base["logits_mean_err_ulps"] + 0.25, (stats, base["logits_mean_err_ulps"])
        assert errs.max() <= base["logits_max_err_ulps"] + 1.0, (stats, base["logits_max_err_ulps"])


def test_full_depth_greedy_trajectory(full):
    from oracle.zonos_cpu import apply_delay_pattern
    model, t, meta, cond = full
    n = meta["n"]
    out = model.generate(cond.to(DEV), max_new_tokens=n, sampling_params=dict(temperature=0.0), progress_bar=False)
    got = apply_delay_pattern(out.cpu(), 1025)[0]
    ref = apply_delay_pattern(t["codes"], 1025)[0]
    diff = (got != ref)
    if not diff.any():
        return
    f = int(diff.any(0).nonzero()[0])  # first diverging delayed frame; decision index f - 1
    k = int(diff[:, f].nonzero()[0])
    margin, top = float(t["margin"][f - 1, k]), float(t["top"][f - 1, k])
    ref_noise = max(meta["self_noise"]["max_ulps"], meta.get("exact_gemm_noise", {}).get("max_ulps", 0.0))
    floor = 2 * ref_noise * float(_ulp(torch.tensor(top)))
    info = dict(first_diverging_frame=f, codebook=k, ref_margin=margin, floor=floor,
                ref_1_thread_first_divergence=meta["stable_1_3_8"]["1"]["first_diverging_delayed_frame"])
    if os.path.isdir("gpurun_out"):
        json.dump(info, open("gpurun_out/full_trajectory.json", "w"), indent=1)
    assert margin <= floor, f"divergence at a decision the reference determines: {info}"


def _row_ulps(ref, got):
    ref, got = ref.float().cpu(), got.float().cpu()
    return (ref - got).abs().amax(-1) / _ulp(ref.abs().amax(-1))


def _hip_baseline():
    """The HIP path's own measured error on the Zonos-v0.1 fixture (MI355X, round 4), or None."""
    p = os.path.join(os.path.dirname(__file__), "golden", "full_layers_hip_baseline.json")
    return json.load(open(p)) if os.path.exists(p) else None


def test_full_depth_per_layer_error(full):
    """Where the logit noise builds up: the first teacher-forced decode step run launch by launch, the
    residual stream after every block (and the attention-block / FFN outputs at the fixture's probe
    layers) against the reference's, in bf16 ulps of each row's max |x|, next to the same deviation of
    the reference's own 1-thread run and of the reference with exact (fp64) GEMMs (fixture metadata).
    Written to gpurun_out/full_layers.json; the HIP path must stay within 4x the larger of the two
    yardsticks (+ 2 ulps) at every block, and within 1 ulp of its own recorded baseline."""
    from oracle.zonos_cpu import apply_delay_pattern
    from zonos_vibes_amd import _lib
    from zonos_vibes_amd.engine import SamplingParams
    model, t, meta = full[:3]
    if "layer_out" not in t:
        pytest.skip("fixture without per-layer probes")
    e = model.engine
    probes = meta["layer_probes"]
    e.prefill(0, full[3].to(DEV), None, meta["n"], SamplingParams(temperature=0.0))
    delayed = apply_delay_pattern(t["codes"], 1025)[0]
    with torch.cuda.stream(e.stream):
        e.delayed[0, :, : delayed.shape[-1]] = delayed.to(DEV, torch.int32)
        e.refresh_inputs()
    e.stream.synchronize()
    plan = e._plan(2, "none")  # launch by launch: QKV, attention, out_proj, fc1, fc2 as their own launches
    layer_out, mixer, mlp = [], {}, {}
    scratch = torch.zeros(2, e.d, dtype=torch.bfloat16, device=DEV)
    res_i = 0
    with torch.cuda.stream(e.stream):
        for kind, item in plan:
            if kind == "gemv" and item[1] == _lib.EPI_RESIDUAL:
                layer = res_i // 2
                if layer in probes:  # the same GEMV with a plain bf16 store: the block's mixer / FFN output
                    a, _ = item
                    keep = (a.out, a.ldo)
                    a.out, a.ldo = scratch.data_ptr(), e.d
                    _lib.check(e.lib.zmi_gemv_launch(ctypes.byref(a), _lib.EPI_STORE, e.sptr))
                    a.out, a.ldo = keep
                    (mixer if res_i % 2 == 0 else mlp)[layer] = scratch.clone()
                e._run_gemv(item)
                if res_i % 2 == 1:
                    layer_out.append(e.x[:2].clone())
                res_i += 1
            elif kind == "gemv":
                e._run_gemv(item)
            elif kind == "attn":
                i, pf = item if isinstance(item, tuple) else (item, None)  # (layer, prefetch ranges)
                e._attention(i, e.q, 2, None, e.row_pos, e.smax - 1, e.attn, pf)
            else:
                raise AssertionError(kind)
    e.stream.synchronize()
    e.check_errors()
    e.release(0)
    hip = _row_ulps(t["layer_out"], torch.stack(layer_out))  # [26, 2]
    ln = meta["layer_noise"]
    thr, exact = torch.tensor(ln["threads_1_vs_8"]), torch.tensor(ln["exact_gemm"])
    rows = []
    for i in range(hip.shape[0]):
        r = dict(layer=i, hip=hip[i].tolist(), ref_1_thread=thr[i].tolist(), ref_exact_gemm=exact[i].tolist())
        if i in probes:
            r["hip_mixer"] = _row_ulps(t[f"mixer_out/{i}"], mixer[i]).tolist()
            r["hip_mlp"] = _row_ulps(t[f"mlp_out/{i}"], mlp[i]).tolist()
        rows.append(r)
    if os.path.isdir("gpurun_out"):
        json.dump(rows, open("gpurun_out/full_layers.json", "w"), indent=1)
    yard = torch.maximum(thr, exact)
    assert (hip <= 4 * yard + 2).all(), rows
    # regression guard, tighter than the yardstick: the HIP kernels are deterministic, so this step's per-block
    # error is a fixed number for the committed code (tests/golden/full_layers_hip_baseline.json, measured on
    # MI355X); a change that moves any block by more than 1 ulp must refresh the baseline on purpose
    base = _hip_baseline()
    if base is not None:
        base = torch.tensor(base["hip_row_ulps"])
        assert base.shape == hip.shape
        assert (hip <= base + 1.0).all(), dict(hip=hip.tolist(), baseline=base.tolist())
