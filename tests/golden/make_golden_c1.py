"""C1 golden fixture: the reference's sample.py flow (sample.py:13-20) at the Zonos-v0.1-transformer dims,
produced by the REFERENCE in this container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c1.py

make_cond_dict("Hello, world!", speaker, "en-us") -> Zonos.prepare_conditioning -> generate(86 frames,
greedy) -> autoencoder.decode, with the v0.1-transformer conditioner list (espeak, speaker, emotion, fmax,
pitch_std, speaking_rate, language_id). The eSpeak front-end is absent, so `phonemize` is the identity and
the "text" is the phoneme string espeak gives for "Hello, world!" (15 symbols; 17 ids with BOS / EOS, so
Lc = 17 + 6 conditioner tokens = 23). Every weight (backbone, heads, prefix conditioner,
DAC) is the counter-based synthetic value of zonos_vibes_amd.synthetic (seed 0, EOS row of heads.0 zeroed
so the run lasts 86 frames, as the bench does), so the fixture holds no weights. It records
(tests/golden/c1_hello.safetensors):

  speaker        the [1, 128] speaker embedding fed to make_cond_dict (synthetic)
  cond           prepare_conditioning output [2, 23, 2048] bf16 (model.py:204-212)
  codes          the greedy generate() codes [1, 9, 86], eager mode, 8 threads
  prefill/steps  CFG'd logits of the prefill and of the first N_TF decode steps, teacher-forced on codes
  top / margin   per decision (prefill + 94 steps, 9 codebooks): top score after EOS bias + penalty, and
                 its top-1 minus top-2 margin
  wav            autoencoder.decode(codes) [1, 1, 44032] f32 (transformers DacModel, fp32 CPU)
metadata: the reference's thread-count self-noise of the teacher-forced logits (1 vs 8 threads), the noise
of the same model with exact (fp64) GEMMs against it, and whether its 1- / 3-thread trajectories equal the
8-thread one.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from make_golden import Fp64Linear, build_ref_model, import_reference, run_generate, save, ulp  # noqa: E402
from zonos_vibes_amd import synthetic as syn  # noqa: E402
from zonos_vibes_amd.conditioning import v01_transformer_conditioners  # noqa: E402
from zonos_vibes_amd.config import PrefixConditionerConfig, ZonosConfig, zonos_v01_transformer  # noqa: E402

PHONEMES = "həlˈoʊ, wˈɜːld!"  # espeak-ng en-us for "Hello, world!"
N, N_TF = 86, 8


def c1_config() -> ZonosConfig:
    cfg = zonos_v01_transformer()
    return ZonosConfig(cfg.backbone, PrefixConditionerConfig(v01_transformer_conditioners(), "none"))


def teacher_forced(model, zs, zc, cond, codes, n_keep):
    """Reference CFG'd logits / decisions along `codes` (model.py:240-307 with the sampled tokens replaced)."""
    lc = cond.shape[1]
    out_logits, tops, margins = [], [], []
    with torch.inference_mode():
        delayed = zc.apply_delay_pattern(codes, 1025)
        n_frames = codes.shape[-1]
        ip = model.setup_cache(batch_size=2, max_seqlen=lc + n_frames + 9)
        lg = model._prefill(cond, delayed[..., :1], ip, 2.0)
        out_logits.append(lg[0].clone())

        def record(scores):
            t2 = scores[0].topk(2, dim=-1).values
            tops.append(t2[:, 0].clone())
            margins.append((t2[:, 0] - t2[:, 1]).clone())

        record(lg)
        ip.seqlen_offset += lc + 1
        ip.lengths_per_sample[:] += lc + 1
        bias = torch.zeros_like(lg)
        bias[:, 1:, 1024] = -torch.inf
        offset = 1
        for s in range(n_frames + 8):
            offset += 1
            lg = model._decode_one_token(delayed[..., offset - 1:offset], ip, torch.tensor(2.0),
                                         allow_cudagraphs=False).clone()
            if s < n_keep:
                out_logits.append(lg[0].clone())
            record(zs.modify_logit_for_repetition_penalty(lg + bias, delayed[..., :offset], 3.0, 2))
            ip.seqlen_offset += 1
            ip.lengths_per_sample[:] += 1
    return out_logits, torch.stack(tops), torch.stack(margins)


def main():
    zm, zs, zc, RefZonosConfig, BACKBONES = import_reference()
    cond_mod = sys.modules["zonos.conditioning"]
    cond_mod.phonemize = lambda texts, languages: list(texts)
    cfg = c1_config()
    t0 = time.time()
    model, _ = build_ref_model(zm, RefZonosConfig, BACKBONES, cfg, zero_eos=True)
    # the conditioner's own state dict (a second Zonos-level load would re-run the head-padding hook)
    pcsd = model.prefix_conditioner.state_dict()
    for k, v in syn.iter_torch_cpu(syn.prefix_conditioner_specs(cfg.prefix_conditioner.conditioners,
                                                                cfg.backbone.d_model), 0):
        k = k[len("prefix_conditioner."):]
        assert pcsd[k].shape == v.shape, (k, pcsd[k].shape, v.shape)
        pcsd[k].copy_(v)
    model.prefix_conditioner.load_state_dict(pcsd)
    assert model.heads[0].weight.shape[0] == 1026
    # the DAC: random-init transformers DacModel overwritten with the synthetic weights (make_golden.py §7)
    dsd = model.autoencoder.dac.state_dict()
    for k, v in syn.iter_torch_cpu(syn.dac_specs(), 0):
        dsd[k].copy_(v)
    model.autoencoder.dac.load_state_dict(dsd)
    model.autoencoder.dac.eval()
    print(f"model built in {time.time() - t0:.0f}s", flush=True)

    speaker = torch.from_numpy(syn.synthetic_speaker_np(0).view(np.int16).copy()).view(torch.bfloat16)
    torch.set_num_threads(8)
    cond_dict = cond_mod.make_cond_dict(text=PHONEMES, speaker=speaker, language="en-us")
    with torch.inference_mode():
        cond = model.prepare_conditioning(cond_dict)
    print("conditioning", tuple(cond.shape), flush=True)
    greedy = dict(temperature=0.0)
    runs = {}
    for th in (8, 3, 1):
        t0 = time.time()
        runs[th] = run_generate(model, cond, None, N, greedy, th, 0)
        print(f"threads {th}: {tuple(runs[th].shape)} in {time.time() - t0:.0f}s", flush=True)
    codes = runs[8]
    stable = {}
    for th in (3, 1):
        same = torch.equal(runs[th], codes)
        first = None
        if not same and runs[th].shape == codes.shape:
            d = (zc.apply_delay_pattern(runs[th], 1025) != zc.apply_delay_pattern(codes, 1025)).any(1)[0]
            first = int(d.nonzero()[0])
        stable[str(th)] = dict(same=same, first_diverging_delayed_frame=first)
    torch.set_num_threads(8)
    logits, tops, margins = teacher_forced(model, zs, zc, cond, codes, N + 8)
    torch.set_num_threads(1)
    logits1, _, _ = teacher_forced(model, zs, zc, cond, codes, N + 8)
    errs, flips = [], 0
    for a, b in zip(logits, logits1):
        fin = torch.isfinite(a)
        top = a.masked_fill(~fin, -torch.inf).max(-1).values
        errs.append((a - b).masked_fill(~fin, 0).abs().max(-1).values / ulp(top))
        flips += int((a.argmax(-1) != b.argmax(-1)).sum())
    errs = torch.cat(errs)
    self_noise = dict(threads=(1, 8), max_ulps=float(errs.max()), mean_ulps=float(errs.mean()),
                      raw_argmax_disagreements=flips, decisions=int(errs.numel()))
    print("self noise", self_noise, flush=True)
    # at Lc 23 the reference's thread counts may agree bit for bit; the yardstick for an implementation
    # whose GEMMs accumulate in another order is then the same model with every linear exact (fp64,
    # rounded once): the logit noise a different accumulation order alone causes
    torch.set_num_threads(8)
    with Fp64Linear():
        logits64, _, _ = teacher_forced(model, zs, zc, cond, codes, N + 8)
    errs = []
    for a, b in zip(logits, logits64):
        fin = torch.isfinite(a)
        top = a.masked_fill(~fin, -torch.inf).max(-1).values
        errs.append((a - b).masked_fill(~fin, 0).abs().max(-1).values / ulp(top))
    errs = torch.cat(errs)
    exact_gemm_noise = dict(max_ulps=float(errs.max()), mean_ulps=float(errs.mean()), decisions=int(errs.numel()))
    print("exact-GEMM noise", exact_gemm_noise, flush=True)
    torch.set_num_threads(8)
    with torch.inference_mode():
        wav = model.autoencoder.decode(codes)
    logits = logits[: N_TF + 1]
    save("c1_hello", {"speaker": speaker, "cond": cond, "codes": codes, "prefill": logits[0],
                      "steps": torch.stack(logits[1:]), "top": tops, "margin": margins, "wav": wav.float()},
         {"cfg": cfg.to_dict(), "phonemes": PHONEMES, "language": "en-us", "lc": int(cond.shape[1]), "n": N,
          "weights_seed": 0, "zero_eos": True, "threads": 8, "stable_1_3_8": stable, "teacher_forced_steps": N_TF,
          "self_noise": self_noise, "exact_gemm_noise": exact_gemm_noise})
    print(json.dumps(stable))


if __name__ == "__main__":
    main()
