"""Generate the golden fixtures by running the REFERENCE implementation (in this container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference (`/root/reference`, read-only) is imported with stub modules for the
text/audio front-end packages that are absent here (torchaudio, inflect, kanjize, phonemizer,
sudachipy); none of them is on the generate()/decode() path (SURVEY.md §8c recipe).
`DacModel.from_pretrained` is replaced by a random-init `DacModel(DacConfig(sampling_rate=44100))`
because the real checkpoint needs the network. All weights are then overwritten with the
counter-based synthetic values of `zonos_vibes_amd.synthetic` so any consumer can regenerate
them without committing weights.

Outputs (small, committed): tests/golden/*.safetensors — inputs and reference outputs only.
Trajectory fixtures are "stable": identical under torch.set_num_threads(1, 3, 8).
"""
from __future__ import annotations

import importlib.machinery
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from safetensors.torch import save_file  # noqa: E402

from zonos_vibes_amd import synthetic as syn  # noqa: E402
from zonos_vibes_amd.config import tiny_transformer, transformer_config  # noqa: E402

REF = "/root/reference"


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def import_reference():
    import transformers  # noqa: F401  (probes find_spec('torchaudio') before the stub exists)

    class _Any:
        def __init__(self, *a, **k):
            pass

        def create(self, *a, **k):
            return self

    ta = _stub("torchaudio")
    ta.functional = _stub("torchaudio.functional")
    ta.transforms = _stub("torchaudio.transforms")
    _stub("inflect", engine=_Any)
    _stub("kanjize", number2kanji=str)
    _stub("phonemizer")
    _stub("phonemizer.backend", EspeakBackend=_Any)
    _stub("sudachipy", Dictionary=_Any, SplitMode=types.SimpleNamespace(A=0))
    from transformers import DacConfig, DacModel
    DacModel.from_pretrained = classmethod(lambda cls, *a, **k: DacModel(DacConfig(sampling_rate=44100)))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import zonos.model as zm
    import zonos.sampling as zs
    import zonos.codebook_pattern as zc
    from zonos.config import ZonosConfig
    from zonos.backbone import BACKBONES
    return zm, zs, zc, ZonosConfig, BACKBONES


def build_ref_model(zm, ZonosConfig, BACKBONES, cfg, seed=0, eos_row_scale=None, zero_eos=False):
    rcfg = ZonosConfig.from_dict(json.loads(json.dumps(cfg.to_dict())))
    model = zm.Zonos(rcfg, BACKBONES["torch"]).to(torch.bfloat16)
    sd = model.state_dict()  # heads are [1025, d] here; the load hook pads them to 1026 (model.py:46-51)
    w = dict(syn.iter_torch_cpu(syn.zonos_specs(cfg), seed))
    tweak_heads(w, eos_row_scale, zero_eos)
    for k, v in w.items():
        sd[k].copy_(v)
    model.load_state_dict(sd)
    assert model.heads[0].weight.shape[0] == 1026
    model.eval()
    return model, w


def tweak_heads(w, eos_row_scale=None, zero_eos=False):
    """EOS control: zero row 1024 of heads.0 (suppress) or scale it (make EOS likely)."""
    h0 = w["heads.0.weight"].clone()
    if zero_eos:
        h0[1024] = 0
    if eos_row_scale is not None:
        h0[1024] = (h0[1024].float() * eos_row_scale).to(torch.bfloat16)
    w["heads.0.weight"] = h0


def cond_tensor(seed, rows, length, d):
    a = syn.synthetic_conditioning_np(seed, rows, length, d)
    return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)


def save(name, tensors, meta):
    path = os.path.join(HERE, name + ".safetensors")
    save_file({k: v.contiguous() for k, v in tensors.items()}, path, metadata={"json": json.dumps(meta)})
    print("wrote", path, {k: tuple(v.shape) for k, v in tensors.items()})


def run_generate(model, cond, prefix, n, params, threads, seed):
    torch.set_num_threads(threads)
    torch.manual_seed(seed)
    return model.generate(cond, audio_prefix_codes=prefix, max_new_tokens=n, cfg_scale=2.0,
                          sampling_params=params, progress_bar=False, disable_torch_compile=True)


def ulp(x: torch.Tensor) -> torch.Tensor:
    return torch.ldexp(torch.ones_like(x), torch.frexp(x.abs().clamp_min(1e-30))[1] - 8)


class Fp64Linear:
    """Context: every nn.Linear / F.linear of the reference computed exactly (fp64) and rounded to
    its dtype once -- an implementation that differs from the reference only in the GEMMs'
    accumulation order, to measure the logit noise such a difference alone causes."""
    def __enter__(self):
        import torch.nn.functional as F
        self.orig = F.linear
        F.linear = lambda x, w, b=None: ((x.double() @ w.double().t()) + (0 if b is None else b.double())).to(x.dtype)
        return self

    def __exit__(self, *a):
        import torch.nn.functional as F
        F.linear = self.orig


def teacher_forced_scores(model, zs, cond, prefix_len, delayed, n_decisions):
    """Reference decisions along a known delayed trajectory (model.py:240-307 with the sampled tokens
    fixed): per decision the CFG'd logits and the scores greedy argmax sees (EOS bias + penalty)."""
    lc = cond.shape[1]
    logits, scores = [], []
    with torch.inference_mode():
        ip = model.setup_cache(batch_size=2, max_seqlen=lc + delayed.shape[-1])
        lg = model._prefill(cond, delayed[..., : prefix_len + 1], ip, 2.0)
        logits.append(lg[0].clone())
        scores.append(lg[0].clone())
        ip.seqlen_offset += lc + prefix_len + 1
        ip.lengths_per_sample[:] += lc + prefix_len + 1
        bias = torch.zeros_like(lg)
        bias[:, 1:, 1024] = -torch.inf
        offset = prefix_len + 1
        for _ in range(n_decisions - 1):
            offset += 1
            lg = model._decode_one_token(delayed[..., offset - 1:offset], ip, torch.tensor(2.0),
                                         allow_cudagraphs=False).clone()
            logits.append(lg[0].clone())
            scores.append(zs.modify_logit_for_repetition_penalty(lg + bias, delayed[..., :offset], 3.0, 2)[0])
            ip.seqlen_offset += 1
            ip.lengths_per_sample[:] += 1
    return logits, scores


def noise_ulps(a_list, b_list):
    """Max |a - b| per decision and codebook, in bf16 ulps of a's top score."""
    out = []
    for a, b in zip(a_list, b_list):
        fin = torch.isfinite(a)
        top = a.masked_fill(~fin, -torch.inf).max(-1).values
        out.append((a - b).masked_fill(~fin, 0).abs().max(-1).values / ulp(top))
    return torch.stack(out)


def stable(model, cond, prefix, n, params, seed=0):
    outs = [run_generate(model, cond, prefix, n, params, t, seed) for t in (1, 3, 8)]
    same = all(o.shape == outs[0].shape and torch.equal(o, outs[0]) for o in outs)
    return outs[0], same


def main():
    zm, zs, zc, ZonosConfig, BACKBONES = import_reference()
    torch.set_num_threads(8)

    # 1. delay pattern --------------------------------------------------------------
    g = torch.Generator().manual_seed(0)
    codes = torch.randint(0, 1024, (2, 9, 12), generator=g)
    codes[:, :, 9:] = -1
    dl = zc.apply_delay_pattern(codes, 1025)
    save("delay_pattern", {"codes": codes, "delayed": dl, "reverted": zc.revert_delay_pattern(dl)}, {})

    # 2. penalty + greedy on bf16-valued logits (ties occur) -------------------------
    lg = (torch.randn(3, 9, 1026, generator=g) * 2).to(torch.bfloat16).float()
    lg[..., 1025] = -torch.inf
    lg[:, 1:, 1024] = -torch.inf
    gen = torch.randint(0, 1026, (3, 9, 6), generator=g)
    gen[0, :, -1] = gen[0, :, -2]  # repeated token -> factor 9
    pen = zs.modify_logit_for_repetition_penalty(lg.clone(), gen, 3.0, 2)
    greedy = zs.sample_from_logits(lg.clone(), temperature=0.0, generated_tokens=gen)
    save("penalty_greedy", {"logits": lg, "generated": gen, "penalized": pen, "greedy": greedy}, {})

    # 3. stochastic samplers with the reference's own exponential draw ------------------
    psets = [dict(min_p=0.1), dict(top_p=0.8), dict(top_k=30), dict(linear=0.5, conf=0.4, quad=0.0),
             dict(temperature=0.7, top_p=0.95, min_p=0.05), dict(temperature=1.3, top_k=50, top_p=0.9)]
    tens, meta = {"logits": lg, "generated": gen}, {"params": psets}
    for i, ps in enumerate(psets):
        torch.manual_seed(100 + i)
        out = zs.sample_from_logits(lg.clone(), generated_tokens=gen, **ps)
        torch.manual_seed(100 + i)
        q = torch.empty(lg.shape).exponential_(1)
        tens[f"q{i}"], tens[f"out{i}"] = q, out
    save("samplers", tens, meta)

    # 4. rope table digest (the table is recomputed by consumers, 8 MB is not committed) ---
    import hashlib
    from zonos.backbone._torch import precompute_freqs_cis
    fc = precompute_freqs_cis(16384, 128)
    save("rope", {"rows_0_8": fc[:8].clone(), "rows_last": fc[-4:].clone()},
         {"sha256": hashlib.sha256(fc.numpy().tobytes()).hexdigest()})

    # 5. tiny-model trajectories -------------------------------------------------------
    cfg = tiny_transformer(2)
    traj_t, traj_meta = {}, {"cfg": cfg.to_dict(), "cases": []}

    def add_case(tag, model_kw, cond_seed, lc, n, params, prefix_len=0, seed=0, require_stable=True):
        model, w_case = build_ref_model(zm, ZonosConfig, BACKBONES, cfg, **model_kw)
        cond = cond_tensor(cond_seed, 2, lc, cfg.backbone.d_model)
        prefix = None
        if prefix_len:
            prefix = torch.randint(0, 1024, (1, 9, prefix_len), generator=torch.Generator().manual_seed(cond_seed))
        out, ok = stable(model, cond, prefix, n, params, seed)
        print(tag, "stable" if ok else "UNSTABLE", tuple(out.shape))
        if require_stable and not ok:
            return False
        traj_t[tag + "/cond"] = cond
        traj_t[tag + "/codes"] = out
        if prefix is not None:
            traj_t[tag + "/prefix"] = prefix
        extra = {}
        if params.get("temperature", 1.0) == 0.0:
            # the reference's decisions along its own trajectory (its delayed frames from the oracle,
            # which is bit-identical here), and the noise an exact-GEMM implementation shows on them
            from oracle.zonos_cpu import OracleZonos
            torch.set_num_threads(8)
            om = OracleZonos(cfg, w_case)
            raw = []
            o_codes = om.generate(cond, prefix, max_new_tokens=n, sampling_params=params, raw_trace=raw)
            assert torch.equal(o_codes, out)
            dl = om.last_delayed
            lg, sc = teacher_forced_scores(model, zs, cond, prefix_len, dl, len(raw))
            with Fp64Linear():
                lg64, _ = teacher_forced_scores(model, zs, cond, prefix_len, dl, len(raw))
            t2 = torch.stack([x.topk(2, dim=-1).values for x in sc])
            traj_t[tag + "/delayed"] = dl.to(torch.int16).contiguous()
            traj_t[tag + "/top"] = t2[..., 0].contiguous()
            traj_t[tag + "/margin"] = (t2[..., 0] - t2[..., 1]).contiguous()
            nz = noise_ulps(lg, lg64)
            extra = dict(exact_gemm_noise=dict(max_ulps=float(nz.max()), mean_ulps=float(nz.mean())))
            print(tag, extra)
        traj_meta["cases"].append(dict(tag=tag, model_kw=model_kw, cond_seed=cond_seed, lc=lc, n=n, params=params,
                                       prefix_len=prefix_len, seed=seed, threads_checked=[1, 3, 8], stable=ok,
                                       **extra))
        return True

    greedy_p = dict(temperature=0.0)
    add_case("greedy_maxlen", dict(zero_eos=True), 11, 12, 24, greedy_p)
    add_case("greedy_prefix", dict(zero_eos=True), 12, 9, 20, greedy_p, prefix_len=5)
    # EOS-forced runs: scale the EOS row until a stable trajectory ends early
    found = 0
    for sc in (6.0, 8.0, 10.0, 12.0, 16.0):
        for cs in range(20, 40):
            model, _ = build_ref_model(zm, ZonosConfig, BACKBONES, cfg, eos_row_scale=sc)
            cond = cond_tensor(cs, 2, 10, cfg.backbone.d_model)
            out = run_generate(model, cond, None, 40, greedy_p, 8, 0)
            if 3 <= out.shape[2] < 30:
                if add_case(f"greedy_eos_{found}", dict(eos_row_scale=sc), cs, 10, 40, greedy_p):
                    found += 1
            if found >= 2:
                break
        if found >= 2:
            break
    add_case("minp_seeded", dict(zero_eos=True), 13, 8, 16, dict(min_p=0.1), seed=421, require_stable=False)
    save("tiny_trajectories", traj_t, traj_meta)

    # 6. full-dims single layer: prefill + 3 teacher-forced decode logits ----------------
    cfg1 = transformer_config(2048, 1, 16, 4, 8192)
    model, _ = build_ref_model(zm, ZonosConfig, BACKBONES, cfg1, zero_eos=True)
    cond = cond_tensor(7, 2, 16, 2048)
    torch.set_num_threads(8)
    with torch.inference_mode():
        ip = model.setup_cache(batch_size=2, max_seqlen=16 + 8 + 9)
        delayed = zc.apply_delay_pattern(torch.full((1, 9, 8), -1), 1025)
        pl = model._prefill(cond, delayed[..., :1], ip, 2.0)
        ip.seqlen_offset += 17
        ip.lengths_per_sample[:] += 17
        feed = torch.randint(0, 1024, (3, 1, 9, 1), generator=torch.Generator().manual_seed(3))
        steps = []
        for t in range(3):
            steps.append(model._decode_one_token(feed[t], ip, torch.tensor(2.0), allow_cudagraphs=False).clone())
            ip.seqlen_offset += 1
            ip.lengths_per_sample[:] += 1
    save("full_layer", {"cond": cond, "prefill_logits": pl, "feed": feed, "step_logits": torch.stack(steps)},
         {"cfg": cfg1.to_dict(), "threads": 8})

    # 7. DAC decode of 16 frames at full 44.1 kHz dims ------------------------------------
    from transformers import DacConfig, DacModel
    dac = DacModel(DacConfig(sampling_rate=44100)).eval()
    dsd = dac.state_dict()
    for k, v in syn.iter_torch_cpu(syn.dac_specs(), 0):
        assert dsd[k].shape == v.shape, (k, dsd[k].shape, v.shape)
        dsd[k].copy_(v)
    dac.load_state_dict(dsd)
    from zonos.autoencoder import DACAutoencoder
    ae = DACAutoencoder.__new__(DACAutoencoder)
    ae.dac = dac
    codes = torch.randint(0, 1024, (2, 9, 16), generator=torch.Generator().manual_seed(5))
    with torch.inference_mode():
        wav = ae.decode(codes)
    save("dac_decode", {"codes": codes, "wav": wav}, {"threads": 8})


if __name__ == "__main__":
    main()
