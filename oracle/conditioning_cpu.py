"""ORACLE — CPU restatement of the reference prefix conditioner. TEST INFRASTRUCTURE ONLY.

Only `tests/` may import this module, as the checker of zonos_vibes_amd.conditioning (the HIP path).
Pinned by tests/golden/prefix_cond.safetensors, produced by the reference itself
(tests/golden/make_golden_cond.py).

  Conditioner.forward          reference zonos/conditioning.py:43-50
  EspeakPhonemeConditioner     :219-235 (phonemize is the out-of-scope eSpeak front-end: this
                               restatement takes the phoneme strings it would return)
  tokenize_phonemes            :148-154
  FourierConditioner           :241-258
  IntegerConditioner           :261-270
  PassthroughConditioner       :273-279
  PrefixConditioner.forward    :293-310
  make_cond_dict               :326-395 (minus phonemization)
  Zonos.prepare_conditioning   reference zonos/model.py:204-212

The same ATen ops in the same order as the reference, on bf16 parameters (the reference model is
`.to(torch.bfloat16)` as a whole, Fourier buffers included).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from zonos_vibes_amd.conditioning import tokenize_phonemes


class OracleConditioner:
    def __init__(self, conditioners: list[dict], d: int, weights: dict, projection: str = "none"):
        """`weights`: reference state-dict names relative to `prefix_conditioner.`, bf16 CPU tensors."""
        if projection != "none":
            raise NotImplementedError("prefix projection other than 'none'")
        self.cfgs = [dict(c) for c in conditioners]
        self.d = d
        self.w = weights
        self.required_keys = {c["name"] for c in self.cfgs if c.get("uncond_type", "none") != "learned"}

    def _project(self, i, cfg, x):
        if cfg.get("projection", "none") == "linear":
            return F.linear(x, self.w[f"conditioners.{i}.project.weight"], self.w[f"conditioners.{i}.project.bias"])
        if cfg.get("projection", "none") == "mlp":
            raise NotImplementedError("conditioner projection 'mlp'")
        return x

    def _apply(self, i, cfg, *inputs):
        t = cfg["type"]
        if t == "EspeakPhonemeConditioner":
            phonemes, _languages = inputs
            ids, _ = tokenize_phonemes(list(phonemes))
            return F.embedding(ids, self.w[f"conditioners.{i}.phoneme_embedder.weight"])
        if t == "FourierConditioner":
            (x,) = inputs
            wt = self.w[f"conditioners.{i}.weight"]
            assert x.shape[-1] == cfg.get("input_dim", 1)
            x = (x - cfg.get("min_val", 0.0)) / (cfg.get("max_val", 1.0) - cfg.get("min_val", 0.0))
            f = 2 * torch.pi * x.to(wt.dtype) @ wt.T
            return torch.cat([f.cos(), f.sin()], dim=-1)
        if t == "IntegerConditioner":
            (x,) = inputs
            assert x.shape[-1] == 1
            return F.embedding(x.squeeze(-1) - cfg.get("min_val", 0), self.w[f"conditioners.{i}.int_embedder.weight"])
        if t == "PassthroughConditioner":
            (x,) = inputs
            assert x.shape[-1] == (cfg.get("cond_dim") or self.d)
            return x
        raise ValueError(t)

    def _conditioner(self, i, cfg, inputs):
        if inputs is None:
            return self.w[f"conditioners.{i}.uncond_vector"].view(1, 1, -1)
        return self._project(i, cfg, self._apply(i, cfg, *inputs))

    def forward(self, cond_dict: dict) -> torch.Tensor:
        if not set(cond_dict).issuperset(self.required_keys):
            raise ValueError(f"Missing required keys: {self.required_keys - set(cond_dict)}")
        conds = [self._conditioner(i, c, cond_dict.get(c["name"])) for i, c in enumerate(self.cfgs)]
        max_bsz = max(map(len, conds))
        conds = [c.expand(max_bsz, -1, -1) for c in conds]
        x = torch.cat(conds, dim=-2)
        return F.layer_norm(x, (self.d,), self.w["norm.weight"], self.w["norm.bias"], 1e-5)

    def prepare_conditioning(self, cond_dict: dict, uncond_dict: dict | None = None) -> torch.Tensor:
        if uncond_dict is None:
            uncond_dict = {k: cond_dict[k] for k in self.required_keys}
        return torch.cat([self.forward(cond_dict), self.forward(uncond_dict)])
