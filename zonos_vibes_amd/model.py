"""Zonos with the reference's generate() surface (zonos/model.py:218-315), on the HIP engine.

    model = Zonos.synthetic(zonos_v01_transformer(), device="cuda")      # or Zonos.from_local(...)
    codes = model.generate(prefix_conditioning)                          # [1, 9, T] int64
    wav = model.autoencoder.decode(codes)                                # [1, 1, 512 T] fp32

`generate` keeps the reference's arguments and batch_size=1 semantics; `generate_batch`
runs many independent utterances through the slots of one engine (continuous batching at
chunk granularity), each with exactly the per-utterance result of `generate`.
"""
from __future__ import annotations

import json
from typing import Callable, Sequence

import torch

from . import _lib  # noqa: F401  (fail loudly at import if the HIP library is missing)
from .autoencoder import DACAutoencoder
from .conditioning import PrefixConditioner
from .config import N_CODEBOOKS, ZonosConfig
from .engine import SamplingParams, make_engine


def _draw_seed() -> int:
    # the reference draws its noise from torch's global RNG (sampling.py:20); derive our
    # counter-based stream from the same generator so torch.manual_seed() controls it
    return int(torch.randint(0, 2 ** 62, (1,)).item())


class Zonos:
    def __init__(self, config: ZonosConfig, device="cuda", max_slots: int = 1, max_seqlen: int = 2048,
                 max_prefill: int = 512, autoencoder: DACAutoencoder | None = None):
        self.config = config
        self.eos_token_id = config.eos_token_id
        self.masked_token_id = config.masked_token_id
        self._device = torch.device(device)
        self.engine = make_engine(config, device, max_slots, max_seqlen, max_prefill)
        self.autoencoder = autoencoder if autoencoder is not None else DACAutoencoder(device)
        pcc = config.prefix_conditioner
        self.prefix_conditioner = (PrefixConditioner(pcc.conditioners, config.backbone.d_model, device, pcc.projection)
                                   if pcc.conditioners else None)

    @property
    def device(self) -> torch.device:
        return self._device

    # ------------------------------------------------------------------ construction
    @classmethod
    def synthetic(cls, config: ZonosConfig, device="cuda", seed: int = 0, zero_eos: bool = False,
                  eos_row_scale: float | None = None, dac_seed: int = 0, **kw) -> "Zonos":
        m = cls(config, device, autoencoder=DACAutoencoder(device, seed=dac_seed), **kw)
        m.engine.init_synthetic(seed, zero_eos=zero_eos, eos_row_scale=eos_row_scale)
        if m.prefix_conditioner is not None:
            from . import synthetic as syn
            pcc = config.prefix_conditioner
            sd = dict(syn.iter_torch_cpu(syn.prefix_conditioner_specs(pcc.conditioners, config.backbone.d_model), seed))
            m.prefix_conditioner.load_state_dict(sd, prefix="prefix_conditioner.")
        return m

    @classmethod
    def from_local(cls, config_path: str, model_path: str, device="cuda", backbone: str | None = None,
                   dac_path: str | None = None, **kw) -> "Zonos":
        """model.py:65-88 with local files only (safetensors, no pickle)."""
        from safetensors.torch import load_file
        if backbone not in (None, "hip"):
            raise ValueError(f"backbone {backbone!r}: the HIP build registers BACKBONES['hip'] only "
                             "(transformer and hybrid)")
        config = ZonosConfig.from_dict(json.load(open(config_path)))
        dac = DACAutoencoder(device, state_dict=load_file(dac_path) if dac_path else None)
        m = cls(config, device, autoencoder=dac, **kw)
        sd = load_file(model_path)
        m.engine.load_state_dict(sd)
        if m.prefix_conditioner is not None:
            m.prefix_conditioner.load_state_dict(sd, prefix="prefix_conditioner.")
        return m

    @classmethod
    def from_pretrained(cls, repo_id: str, revision: str | None = None, device="cuda", **kw) -> "Zonos":
        """model.py:57-63: resolves files through the local HF cache (no network in this build)."""
        from huggingface_hub import hf_hub_download
        cfg = hf_hub_download(repo_id=repo_id, filename="config.json", revision=revision)
        mdl = hf_hub_download(repo_id=repo_id, filename="model.safetensors", revision=revision)
        return cls.from_local(cfg, mdl, device, **kw)

    def _ensure_capacity(self, slots: int, seqlen: int, prefill: int):
        e = self.engine
        if slots > e.S or seqlen > e.smax or prefill > e.max_prefill:
            w = e.w
            self.engine = make_engine(self.config, self._device, max(slots, e.S), max(seqlen, e.smax),
                                      max(prefill, e.max_prefill))
            self.engine.w = w
            self.engine._build_plan()

    # ------------------------------------------------------------------ conditioning
    def prepare_conditioning(self, cond_dict: dict, uncond_dict: dict | None = None) -> torch.Tensor:
        """model.py:204-212: [2, Lc, d] bf16 (conditional rows, then unconditional), one HIP launch."""
        if self.prefix_conditioner is None:
            raise ValueError("this config has no prefix conditioners")
        return self.prefix_conditioner.prepare_conditioning(cond_dict, uncond_dict)

    # ------------------------------------------------------------------ generation
    @torch.inference_mode()
    def generate(self, prefix_conditioning: torch.Tensor, audio_prefix_codes: torch.Tensor | None = None,
                 max_new_tokens: int = 86 * 30, cfg_scale: float = 2.0, batch_size: int = 1,
                 sampling_params: dict = dict(min_p=0.1), progress_bar: bool = True,
                 disable_torch_compile: bool = False,
                 callback: Callable[[torch.Tensor, int, int], bool] | None = None,
                 chunk: int = 64) -> torch.Tensor:
        """Reference model.py:218-315 (batch_size=1). `disable_torch_compile` is accepted and ignored:
        the decode step is a hipGraph of hand-written kernels in every mode."""
        assert cfg_scale != 1, "TODO: add support for cfg_scale=1"
        if batch_size != 1 or prefix_conditioning.shape[0] != 2:
            raise ValueError("the reference generate() supports batch_size=1 only (SURVEY.md §0.3); "
                             "use generate_batch() for many utterances")
        lc = prefix_conditioning.shape[1]
        p = 0 if audio_prefix_codes is None else audio_prefix_codes.shape[2]
        self._ensure_capacity(1, lc + p + max_new_tokens + 9, lc + p + 1)
        e = self.engine
        params = SamplingParams.from_dict(dict(sampling_params), cfg_scale, _draw_seed())
        slot = 0
        e.prefill(slot, prefix_conditioning, audio_prefix_codes, max_new_tokens, params)
        max_steps = max_new_tokens + 8
        bar = None
        if progress_bar:
            from tqdm import tqdm
            bar = tqdm(total=max_steps, desc="Generating")
        step = 0
        if callback is None:
            while step < max_steps:
                n = min(chunk, max_steps - step)
                e.step(n, slots=1)
                step += n
                if bar is not None:
                    bar.update(n)
                if not e.slot_state(slot)["active"]:
                    break
        else:
            # exact reference semantics: the callback sees every frame and may stop the loop
            while step < max_steps:
                e.step(1, slots=1)
                step += 1
                if bar is not None:
                    bar.update(1)
                stt = e.slot_state(slot)
                o = stt["offset"]
                frame = e.delayed[slot, :, o:o + 1].to(torch.int64).unsqueeze(0)
                if not callback(frame, step, max_steps) or not stt["active"]:
                    break
        if bar is not None:
            bar.close()
        e.check_errors()  # a hand-off that gave up (or a position past a form's reach) must not pass silently
        out = e.read_codes(slot)
        e.release(slot)
        return out

    @torch.inference_mode()
    def generate_batch(self, conds: Sequence[torch.Tensor], prefixes: Sequence[torch.Tensor | None] | None = None,
                       max_new_tokens: Sequence[int] | int = 86 * 30, cfg_scale: float = 2.0,
                       sampling_params: dict = dict(min_p=0.1), seeds: Sequence[int] | None = None,
                       max_slots: int | None = None, chunk: int = 32) -> list[torch.Tensor]:
        """Many independent utterances through the engine's slots; result i equals generate() on utterance i."""
        n = len(conds)
        prefixes = list(prefixes) if prefixes is not None else [None] * n
        mnt = [max_new_tokens] * n if isinstance(max_new_tokens, int) else list(max_new_tokens)
        seeds = list(seeds) if seeds is not None else [_draw_seed() for _ in range(n)]
        need_seq = max(c.shape[1] + (0 if p is None else p.shape[2]) + m + 9 for c, p, m in zip(conds, prefixes, mnt))
        need_pre = max(c.shape[1] + (0 if p is None else p.shape[2]) + 1 for c, p in zip(conds, prefixes))
        slots = min(max_slots or n, n)
        self._ensure_capacity(slots, need_seq, need_pre)
        e = self.engine
        # longest-processing-time first, so the tail is short
        order = sorted(range(n), key=lambda i: -mnt[i])
        queue = list(order)
        owner = [-1] * slots
        results: list[torch.Tensor | None] = [None] * n
        remaining = [0] * slots

        def fill():
            items = []
            for s in range(slots):
                if owner[s] < 0 and queue:
                    i = queue.pop(0)
                    params = SamplingParams.from_dict(dict(sampling_params), cfg_scale, seeds[i])
                    items.append((s, conds[i], prefixes[i], mnt[i], params))
                    owner[s] = i
                    remaining[s] = mnt[i] + 8
            e.prefill_many(items)  # the free slots' prefills in as few passes through the layers as fit

        # a step runs slots 0 .. the highest busy one (rounded up to a few sizes, one decode graph each): LPT
        # fills the low slots with the longest utterances, so the tail of a job steps a handful of rows instead
        # of every slot's (every kernel is row-invariant: the codes do not depend on the row count)
        sizes = sorted({slots} | {b for b in (1, 2, 4, 8, 16, 24, 32, 40, 48, 56) if b < slots})

        fill()
        while any(o >= 0 for o in owner):
            k = min(chunk, max(r for s, r in enumerate(remaining) if owner[s] >= 0))
            hi = max(s for s in range(slots) if owner[s] >= 0) + 1 if e.batch_shrink else slots
            e.step(k, slots=next(b for b in sizes if b >= hi))
            e.stream.synchronize()
            e.check_errors()
            act = e.st["active"].cpu()
            for s in range(slots):
                if owner[s] >= 0:
                    remaining[s] -= k
                    if not act[s]:
                        results[owner[s]] = e.read_codes(s)
                        owner[s] = -1
                        e.pos_hi[s] = 0  # its rows are inactive (position -1): no bound on the attention form
            fill()
        return results

    def __repr__(self):
        bb = self.config.backbone
        kind = "hybrid" if bb.is_hybrid else "transformer"
        return f"Zonos(hip {kind}, d={bb.d_model}, layers={bb.n_layer}, heads={bb.num_heads}/{bb.num_heads_kv})"


__all__ = ["Zonos", "DACAutoencoder", "N_CODEBOOKS"]
