"""Full-depth golden fixture: the REFERENCE Zonos-v0.1-transformer dims (26 layers, d 2048) on
the synthetic weights, C2's conditioning (Lc = 160). Run in this container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_full.py

Imports /root/reference exactly as make_golden.py does (stubs for the absent text/audio front-end
packages, random-init DacModel); all weights are then overwritten with the counter-based synthetic
values of zonos_vibes_amd.synthetic (seed 0, EOS row of heads.0 zeroed as the bench does), so the
fixture holds no weights. It records (tests/golden/full_model.safetensors):

  codes          the greedy generate() trajectory, 64 new frames, reference eager mode, 8 threads
  stable_1_3_8   whether 1- and 3-thread runs give the same codes (and, if not, the first
                 diverging delayed frame index)
  prefill        CFG'd logits of the prefill ([9, 1026] f32, model.py:255)
  steps          CFG'd logits of the first 16 decode steps, teacher-forced on `codes`
  top / margin   per decision (prefill + 72 steps, 9 codebooks): the top score the greedy argmax
                 sees (after EOS bias + repetition penalty) and its top-1 minus top-2 margin
  self_noise     the reference against itself: the same teacher-forced logits at 1 thread vs 8
                 threads, in bf16 ulps of each decision's top score (metadata)
  exact_gemm_noise  the same logits of the reference with every linear exact (fp64, rounded once)
                 against the 8-thread run: the noise a different GEMM accumulation order alone causes
  layer_out      the first decode step's residual stream after every block [26, 2, 2048] bf16
  mixer_out/mlp_out  that step's attention-block (after out_proj) and FFN outputs at LAYER_PROBES
  layer_noise    per block, the 1-thread and exact-GEMM variants' deviation from layer_out in bf16 ulps
                 of each row's max |x| (metadata; localises where logit noise builds up)
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

from make_golden import Fp64Linear, build_ref_model, cond_tensor, import_reference, run_generate, save  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402

LC, N, N_TF = 160, 64, 16
LAYER_PROBES = (0, 1, 12, 25)


def probe_step(model, zc, cond, codes):
    """Reference block / mixer / mlp outputs of the first teacher-forced decode step (forward hooks)."""
    outs = {"layer": [], "mixer": {}, "mlp": {}}
    hooks = []
    capture = [False]

    def grab(kind, i):
        def f(mod, inp, out):
            if capture[0]:
                v = out[0].detach().clone() if isinstance(out, tuple) else out.detach().clone()
                if kind == "layer":
                    outs["layer"].append(v.reshape(2, -1))
                else:
                    outs[kind][i] = v.reshape(2, -1)
        return f

    for i, layer in enumerate(model.backbone.layers):
        hooks.append(layer.register_forward_hook(grab("layer", i)))
        if i in LAYER_PROBES:
            hooks.append(layer.mixer.register_forward_hook(grab("mixer", i)))
            hooks.append(layer.mlp.register_forward_hook(grab("mlp", i)))
    try:
        with torch.inference_mode():
            delayed = zc.apply_delay_pattern(codes, 1025)
            ip = model.setup_cache(batch_size=2, max_seqlen=LC + codes.shape[-1] + 9)
            model._prefill(cond, delayed[..., :1], ip, 2.0)
            ip.seqlen_offset += LC + 1
            ip.lengths_per_sample[:] += LC + 1
            capture[0] = True
            model._decode_one_token(delayed[..., 1:2], ip, torch.tensor(2.0), allow_cudagraphs=False)
    finally:
        for h in hooks:
            h.remove()
    return torch.stack(outs["layer"]), outs["mixer"], outs["mlp"]


def row_ulps(a, b):
    """|a - b| in bf16 ulps of each row's max |a| (max over the row), per leading index."""
    a, b = a.float(), b.float()
    return ((a - b).abs().amax(-1) / ulp(a.abs().amax(-1)))


def ulp(x: torch.Tensor) -> torch.Tensor:
    return torch.ldexp(torch.ones_like(x), torch.frexp(x.abs().clamp_min(1e-30))[1] - 8)


def teacher_forced(model, zs, zc, cond, codes, keep_all=False):
    """Reference logits along `codes` (model.py:240-307 with the sampled tokens replaced)."""
    out_logits, tops, margins = [], [], []
    with torch.inference_mode():
        delayed = zc.apply_delay_pattern(torch.cat([codes, torch.full((1, 9, 0), -1)], -1), 1025)
        n_frames = codes.shape[-1]
        ip = model.setup_cache(batch_size=2, max_seqlen=LC + n_frames + 9)
        lg = model._prefill(cond, delayed[..., :1], ip, 2.0)
        out_logits.append(lg[0].clone())

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
            if s < N_TF or keep_all:
                out_logits.append(lg[0].clone())
            fin = zs.modify_logit_for_repetition_penalty(lg + bias, delayed[..., :offset], 3.0, 2)
            record(fin)
            ip.seqlen_offset += 1
            ip.lengths_per_sample[:] += 1
    return out_logits, torch.stack(tops), torch.stack(margins)


def main():
    zm, zs, zc, ZonosConfig, BACKBONES = import_reference()
    cfg = zonos_v01_transformer()
    t0 = time.time()
    model, _ = build_ref_model(zm, ZonosConfig, BACKBONES, cfg, zero_eos=True)
    print(f"model built in {time.time() - t0:.0f}s", flush=True)
    cond = cond_tensor(1, 2, LC, cfg.backbone.d_model)
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
        if not same:
            d = (zc.apply_delay_pattern(runs[th], 1025) != zc.apply_delay_pattern(codes, 1025)).any(1)[0]
            first = int(d.nonzero()[0])
        stable[str(th)] = dict(same=same, first_diverging_delayed_frame=first)
    torch.set_num_threads(8)
    logits, tops, margins = teacher_forced(model, zs, zc, cond, codes, keep_all=True)
    torch.set_num_threads(1)
    logits1, tops1, _ = teacher_forced(model, zs, zc, cond, codes, keep_all=True)
    errs, flips = [], 0
    for a, b in zip(logits, logits1):
        fin = torch.isfinite(a)
        top = a.masked_fill(~fin, -torch.inf).max(-1).values
        e = ((a - b).masked_fill(~fin, 0).abs().max(-1).values / ulp(top))
        errs.append(e)
        flips += int((a.argmax(-1) != b.argmax(-1)).sum())
    errs = torch.cat(errs)
    self_noise = dict(threads=(1, 8), max_ulps=float(errs.max()), mean_ulps=float(errs.mean()),
                      raw_argmax_disagreements=flips, decisions=int(errs.numel()))
    print("self noise", self_noise, flush=True)
    torch.set_num_threads(8)
    with Fp64Linear():
        logits64, _, _ = teacher_forced(model, zs, zc, cond, codes, keep_all=True)
    errs = []
    for a, b in zip(logits, logits64):
        fin = torch.isfinite(a)
        top = a.masked_fill(~fin, -torch.inf).max(-1).values
        errs.append((a - b).masked_fill(~fin, 0).abs().max(-1).values / ulp(top))
    errs = torch.cat(errs)
    exact_gemm_noise = dict(max_ulps=float(errs.max()), mean_ulps=float(errs.mean()), decisions=int(errs.numel()))
    print("exact-GEMM noise", exact_gemm_noise, flush=True)
    # where the noise builds up: per-block deviations of the 1-thread and exact-GEMM variants
    lay8, mix8, mlp8 = probe_step(model, zc, cond, codes)
    torch.set_num_threads(1)
    lay1, _, _ = probe_step(model, zc, cond, codes)
    torch.set_num_threads(8)
    with Fp64Linear():
        lay64, _, _ = probe_step(model, zc, cond, codes)
    layer_noise = dict(threads_1_vs_8=row_ulps(lay8, lay1).tolist(), exact_gemm=row_ulps(lay8, lay64).tolist())
    logits = logits[: N_TF + 1]
    probes = {f"mixer_out/{i}": mix8[i] for i in LAYER_PROBES}
    probes.update({f"mlp_out/{i}": mlp8[i] for i in LAYER_PROBES})
    save("full_model", {"codes": codes, "prefill": logits[0], "steps": torch.stack(logits[1:]), "top": tops,
                        "margin": margins, "layer_out": lay8, **probes},
         {"cfg": cfg.to_dict(), "lc": LC, "cond_seed": 1, "n": N, "weights_seed": 0, "zero_eos": True,
          "threads": 8, "stable_1_3_8": stable, "teacher_forced_steps": N_TF, "self_noise": self_noise,
          "exact_gemm_noise": exact_gemm_noise, "layer_probes": list(LAYER_PROBES), "layer_noise": layer_noise})
    print(json.dumps(stable))


if __name__ == "__main__":
    main()
