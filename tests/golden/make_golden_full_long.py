"""Full-depth golden fixture at the positions C2 and longer batch-1 utterances reach: the REFERENCE
Zonos-v0.1-transformer dims (26 layers, d 2048) on the synthetic weights, C2's conditioning (Lc = 160),
greedy, EOS suppressed. Run in this container only (CPU, ~30 min):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_full_long.py

Imports /root/reference exactly as make_golden.py does; all weights are the counter-based synthetic values of
zonos_vibes_amd.synthetic (seed 0, EOS row of heads.0 zeroed), so the fixture holds no weights. It records
(tests/golden/full_model_long.safetensors):

  codes         the reference's greedy generate() trajectory, N frames (8 threads, eager)
  top / margin  per decision along that trajectory (prefill + N + 8 decode steps, 9 codebooks), teacher-forced:
                the top score the greedy argmax sees (after the EOS bias and the repetition penalty) and its
                top-1 minus top-2 margin
  win_logits    CFG'd logits of the decode steps in WINDOWS (positions around 591 = the C2 mean, 1020-1028 and
                1278-1292), teacher-forced
  win_steps     their decode-step indices (the step at index s runs at position Lc + 1 + s)
  self_noise    the same teacher-forced logits at 1 thread against 8, in bf16 ulps of each decision's top score
                (metadata): the reference's own scale of GEMM accumulation-order noise at these positions
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from make_golden import build_ref_model, cond_tensor, import_reference, run_generate, save, ulp  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402

LC, N = 160, 1125
WINDOWS = [(427, 436), (857, 868), (1117, 1132)]  # decode steps (positions 588-596, 1018-1028, 1278-1292)


def in_window(s):
    return any(a <= s < b for a, b in WINDOWS)


def teacher_forced(model, zs, zc, cond, codes):
    """Reference logits along `codes` (model.py:240-307 with the sampled tokens replaced)."""
    win, tops, margins = [], [], []
    with torch.inference_mode():
        delayed = zc.apply_delay_pattern(codes, 1025)
        n_frames = codes.shape[-1]
        ip = model.setup_cache(batch_size=2, max_seqlen=LC + n_frames + 9)
        lg = model._prefill(cond, delayed[..., :1], ip, 2.0)

        def record(scores):
            t2 = scores[0].topk(2, dim=-1).values
            tops.append(t2[:, 0].clone())
            margins.append((t2[:, 0] - t2[:, 1]).clone())

        record(lg)
        ip.seqlen_offset += LC + 1
        ip.lengths_per_sample[:] += LC + 1
        bias = torch.zeros_like(lg)
        bias[:, 1:, 1024] = -torch.inf
        offset = 1
        for s in range(n_frames + 8):
            offset += 1
            lg = model._decode_one_token(delayed[..., offset - 1:offset], ip, torch.tensor(2.0),
                                         allow_cudagraphs=False).clone()
            if in_window(s):
                win.append(lg[0].clone())
            fin = zs.modify_logit_for_repetition_penalty(lg + bias, delayed[..., :offset], 3.0, 2)
            record(fin)
            ip.seqlen_offset += 1
            ip.lengths_per_sample[:] += 1
            if s % 100 == 0:
                print(f"  teacher-forced step {s}", flush=True)
    return torch.stack(win), torch.stack(tops), torch.stack(margins)


def main():
    zm, zs, zc, ZonosConfig, BACKBONES = import_reference()
    cfg = zonos_v01_transformer()
    t0 = time.time()
    model, _ = build_ref_model(zm, ZonosConfig, BACKBONES, cfg, zero_eos=True)
    print(f"model built in {time.time() - t0:.0f}s", flush=True)
    cond = cond_tensor(1, 2, LC, cfg.backbone.d_model)
    t0 = time.time()
    codes = run_generate(model, cond, None, N, dict(temperature=0.0), 8, 0)
    print(f"generate: {tuple(codes.shape)} in {time.time() - t0:.0f}s", flush=True)
    torch.set_num_threads(8)
    t0 = time.time()
    win, tops, margins = teacher_forced(model, zs, zc, cond, codes)
    print(f"teacher-forced (8 threads) in {time.time() - t0:.0f}s", flush=True)
    torch.set_num_threads(1)
    t0 = time.time()
    win1, _, _ = teacher_forced(model, zs, zc, cond, codes)
    print(f"teacher-forced (1 thread) in {time.time() - t0:.0f}s", flush=True)
    errs, flips = [], 0
    for a, b in zip(win, win1):
        fin = torch.isfinite(a)
        top = a.masked_fill(~fin, -torch.inf).max(-1).values
        errs.append((a - b).masked_fill(~fin, 0).abs().max(-1).values / ulp(top))
        flips += int((a.argmax(-1) != b.argmax(-1)).sum())
    errs = torch.cat(errs)
    self_noise = dict(threads=(1, 8), max_ulps=float(errs.max()), mean_ulps=float(errs.mean()),
                      raw_argmax_disagreements=flips, decisions=int(errs.numel()))
    print("self noise", self_noise, flush=True)
    steps = [s for a, b in WINDOWS for s in range(a, b)]
    save("full_model_long", {"codes": codes, "top": tops, "margin": margins, "win_logits": win,
                             "win_steps": torch.tensor(steps, dtype=torch.int32)},
         {"cfg": cfg.to_dict(), "lc": LC, "cond_seed": 1, "n": N, "weights_seed": 0, "zero_eos": True,
          "threads": 8, "windows": WINDOWS, "self_noise": self_noise})


if __name__ == "__main__":
    main()
