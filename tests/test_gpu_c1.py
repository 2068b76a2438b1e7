"""C1 end to end at the headline dims: the reference's sample.py flow (sample.py:13-20) — make_cond_dict
-> prepare_conditioning -> generate -> autoencoder.decode — on the HIP path against the REFERENCE's own
outputs (tests/golden/c1_hello.safetensors, make_golden_c1.py: Zonos-v0.1-transformer dims, the
v0.1-transformer conditioner list, "Hello, world!" as phonemes, Lc = 23, 86 greedy frames, synthetic
weights).

  * conditioning: every element within one bf16 ulp of the reference's prepare_conditioning output, at
    least 98 % bit-identical (test_conditioning.py's criterion);
  * the seam: teacher-forced on the reference's conditioning and codes, the logits stay within the
    noise scale of the reference (the larger of its 1-vs-8-thread noise and the noise of the same model
    with exact fp64 GEMMs; at Lc 23 the thread counts can agree bit for bit) and every decision the
    reference determines (margin above twice that scale) is identical (test_gpu_parity_full.py's criteria);
  * free running from the HIP conditioning: identical codes up to the first decision the reference
    leaves undetermined;
  * DAC decode of the reference codes: max-abs < 2e-3 and SNR > 50 dB against the reference waveform.
"""
import os

import json
import numpy as np
import pytest
import torch

from tests.helpers import load_golden
from tests.test_conditioning import assert_bf16_close
from tests.test_gpu_parity_full import _cfg_logits, _ulp

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def c1():
    from zonos_vibes_amd.config import ZonosConfig
    from zonos_vibes_amd.model import Zonos
    t, meta = load_golden("c1_hello")
    cfg = ZonosConfig.from_dict(meta["cfg"])
    model = Zonos.synthetic(cfg, DEV, seed=meta["weights_seed"], zero_eos=meta["zero_eos"],
                            max_seqlen=meta["lc"] + meta["n"] + 24, max_prefill=meta["lc"] + 8)
    yield model, t, meta
    del model
    torch.cuda.empty_cache()


def _hip_conditioning(model, t, meta):
    from zonos_vibes_amd.conditioning import make_cond_dict
    cd = make_cond_dict(phonemes=meta["phonemes"], speaker=t["speaker"].to(DEV), language=meta["language"],
                        device=DEV)
    return model.prepare_conditioning(cd)


def test_c1_conditioning(c1):
    model, t, meta = c1
    cond = _hip_conditioning(model, t, meta)
    assert tuple(cond.shape) == (2, 23, 2048) == tuple(t["cond"].shape)
    assert_bf16_close(cond, t["cond"])


def test_c1_teacher_forced_decisions(c1):
    from oracle.zonos_cpu import apply_delay_pattern, repetition_penalty
    from zonos_vibes_amd.engine import SamplingParams
    model, t, meta = c1
    e = model.engine
    n = meta["n"]
    # the yardstick: the larger of the reference's thread-count noise and the noise of exact GEMMs against it
    noise = max((meta["self_noise"], meta["exact_gemm_noise"]), key=lambda d: d["max_ulps"])
    e.prefill(0, t["cond"].to(DEV), None, n, SamplingParams(temperature=0.0))
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
        e.step(1, slots=1)
        e.stream.synchronize()
        lg = _cfg_logits(e.logits[0:2])
        if s < meta["teacher_forced_steps"]:
            logits.append(lg)
        scores.append(repetition_penalty((lg + bias).unsqueeze(0), delayed[None, :, : o + 1], 3.0, 2)[0])
    e.check_errors()
    e.release(0)
    errs = []
    for got, r in zip(logits, [t["prefill"]] + list(t["steps"])):
        fin = torch.isfinite(r)
        assert torch.equal(fin, torch.isfinite(got))
        top = r.masked_fill(~fin, -torch.inf).max(-1).values
        errs.append((got - r).masked_fill(~fin, 0).abs().max(-1).values / _ulp(top))
    errs = torch.cat(errs)
    floor = 2 * noise["max_ulps"]
    det = t["margin"] > floor * _ulp(t["top"])
    got_arg = torch.stack([sc.argmax(-1) for sc in scores])
    init = apply_delay_pattern(torch.full((1, 9, n), -1), 1025)[0]
    agree, used = torch.ones_like(det), torch.zeros_like(det)
    for i in range(min(got_arg.shape[0], init.shape[1] - 1)):
        for m, k in enumerate((init[:, i + 1] == -1).nonzero().flatten().tolist()):
            used[i, m] = True
            agree[i, m] = bool(got_arg[i, m] == delayed[k, i + 1])
    det = det & used
    stats = dict(mean_err_ulps=float(errs.mean()), max_err_ulps=float(errs.max()), ref_self_noise=noise,
                 decisions=int(used.sum()), agree=int((agree & used).sum()), determined=int(det.sum()),
                 determined_disagreements=int((det & ~agree).sum()))
    if os.path.isdir("gpurun_out"):
        json.dump(stats, open("gpurun_out/c1_parity.json", "w"), indent=1)
    assert stats["determined_disagreements"] == 0, stats
    assert errs.mean() <= 1.5 * noise["mean_ulps"], stats
    assert errs.max() <= 2 * noise["max_ulps"], stats


def test_c1_free_running_from_hip_conditioning(c1):
    from oracle.zonos_cpu import apply_delay_pattern
    model, t, meta = c1
    cond = _hip_conditioning(model, t, meta)
    out = model.generate(cond, max_new_tokens=meta["n"], sampling_params=dict(temperature=0.0), progress_bar=False)
    got = apply_delay_pattern(out.cpu(), 1025)[0]
    ref = apply_delay_pattern(t["codes"], 1025)[0]
    assert got.shape == ref.shape
    diff = got != ref
    if not diff.any():
        return
    f = int(diff.any(0).nonzero()[0])
    k = int(diff[:, f].nonzero()[0])
    margin, top = float(t["margin"][f - 1, k]), float(t["top"][f - 1, k])
    ref_noise = max(meta["self_noise"]["max_ulps"], meta["exact_gemm_noise"]["max_ulps"])
    floor = 2 * ref_noise * float(_ulp(torch.tensor(top)))
    assert margin <= floor, dict(first_diverging_frame=f, codebook=k, ref_margin=margin, floor=floor)


def test_c1_dac_decode(c1):
    model, t, meta = c1
    wav = model.autoencoder.decode(t["codes"].to(DEV)).float().cpu()
    ref = t["wav"].float()
    assert wav.shape == ref.shape
    err = (wav - ref).abs()
    snr = 10 * torch.log10(ref.pow(2).mean() / (wav - ref).pow(2).mean())
    assert err.max() < 2e-3 and snr > 50, (err.max().item(), snr.item())
