"""Prefix conditioner on the HIP path: the caller side of generate().

Mirrors the reference's conditioning surface so a caller of `Zonos.prepare_conditioning` switches
unchanged:

  make_cond_dict              reference zonos/conditioning.py:326-395
  tokenize_phonemes           :148-154 (phoneme string -> [BOS, ids..., EOS], left-padded)
  PrefixConditioner.forward   :293-310 (conditioner rows concatenated, then LayerNorm)
  Zonos.prepare_conditioning  reference zonos/model.py:204-212 (cond rows, then uncond rows)

All rows (cond and uncond) are produced by ONE launch of `zmi_prefix_condition`
(csrc/zmi_cond.hip): per row an embedding / learned-vector copy, a Fourier feature or a linear
projection, then the LayerNorm, rounded to bf16 at the reference's rounding points.

The eSpeak phonemizer (text -> phonemes, conditioning.py:159-216) is out of scope:
the "espeak" entry carries phoneme strings, e.g. `make_cond_dict(phonemes="həloʊ")`.
"""
from __future__ import annotations

import ctypes
from typing import Iterable

import torch

from . import _lib

PAD_ID, UNK_ID, BOS_ID, EOS_ID = 0, 1, 2, 3
N_SPECIAL = 4
# phoneme vocabulary (the reference's symbol table, conditioning.py:134-143): ids start after the
# four special tokens, unknown symbols map to UNK_ID
_PUNCT = ';:,.!?¡¿—…"«»“”() *~-/\\&'
_LETTERS = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"
_IPA = ("ɑɐɒæɓʙβɔɕçɗɖðʤəɘɚɛɜɝɞɟʄɡɠɢʛɦɧħɥʜɨɪʝɭɬɫɮʟɱɯɰŋɳɲɴøɵɸθœɶʘɹɺɾɻʀʁɽʂʃʈʧʉʊʋⱱʌɣɤʍχʎʏʑʐʒʔʡʕʢǀǁǂǃˈˌːˑʼʴʰʱʲʷˠˤ˞↓↑→↗↘'̩'ᵻ")
SYMBOLS = [*_PUNCT, *_LETTERS, *_IPA]
PHONEME_VOCAB = N_SPECIAL + len(SYMBOLS)
_SYM_ID = {s: i for i, s in enumerate(SYMBOLS, start=N_SPECIAL)}  # last occurrence wins, as a dict literal does

SUPPORTED_LANGUAGE_CODES = [
    'af', 'am', 'an', 'ar', 'as', 'az', 'ba', 'bg', 'bn', 'bpy', 'bs', 'ca', 'cmn', 'cs', 'cy',
    'da', 'de', 'el', 'en-029', 'en-gb', 'en-gb-scotland', 'en-gb-x-gbclan', 'en-gb-x-gbcwmd',
    'en-gb-x-rp', 'en-us', 'eo', 'es', 'es-419', 'et', 'eu', 'fa', 'fa-latn', 'fi', 'fr-be',
    'fr-ch', 'fr-fr', 'ga', 'gd', 'gn', 'grc', 'gu', 'hak', 'hi', 'hr', 'ht', 'hu', 'hy', 'hyw',
    'ia', 'id', 'is', 'it', 'ja', 'jbo', 'ka', 'kk', 'kl', 'kn', 'ko', 'kok', 'ku', 'ky', 'la',
    'lfn', 'lt', 'lv', 'mi', 'mk', 'ml', 'mr', 'ms', 'mt', 'my', 'nb', 'nci', 'ne', 'nl', 'om',
    'or', 'pa', 'pap', 'pl', 'pt', 'pt-br', 'py', 'quc', 'ro', 'ru', 'ru-lv', 'sd', 'shn', 'si',
    'sk', 'sl', 'sq', 'sr', 'sv', 'sw', 'ta', 'te', 'tn', 'tr', 'tt', 'ur', 'uz', 'vi',
    'vi-vn-x-central', 'vi-vn-x-south', 'yue',
]
LANGUAGE_ID = {lang: i for i, lang in enumerate(SUPPORTED_LANGUAGE_CODES)}


def tokenize_phonemes(phonemes: list[str]) -> tuple[torch.Tensor, list[int]]:
    """[BOS, symbol ids..., EOS] per string, left-padded with PAD to the longest."""
    ids = [[BOS_ID, *(_SYM_ID.get(ch, UNK_ID) for ch in p), EOS_ID] for p in phonemes]
    lengths = [len(x) for x in ids]
    n = max(lengths)
    return torch.tensor([[PAD_ID] * (n - len(x)) + x for x in ids]), lengths


def v01_transformer_conditioners() -> list[dict]:
    """Conditioner list of Zonos-v0.1-transformer as documented in the reference's
    CONDITIONING_README.md (the checkpoint's config.json is not available offline)."""
    L = "learned"
    return [
        {"type": "EspeakPhonemeConditioner", "name": "espeak"},
        {"type": "PassthroughConditioner", "name": "speaker", "cond_dim": 128, "uncond_type": L,
         "projection": "linear"},
        {"type": "FourierConditioner", "name": "emotion", "input_dim": 8, "uncond_type": L},
        {"type": "FourierConditioner", "name": "fmax", "min_val": 0, "max_val": 24000, "uncond_type": L},
        {"type": "FourierConditioner", "name": "pitch_std", "min_val": 0, "max_val": 400, "uncond_type": L},
        {"type": "FourierConditioner", "name": "speaking_rate", "min_val": 0, "max_val": 40, "uncond_type": L},
        {"type": "IntegerConditioner", "name": "language_id", "min_val": -1, "max_val": 126, "uncond_type": L},
    ]


def make_cond_dict(phonemes: str | None = None, language: str = "en-us", speaker: torch.Tensor | None = None,
                   emotion: list[float] = [0.3077, 0.0256, 0.0256, 0.0256, 0.0256, 0.0256, 0.2564, 0.3077],
                   fmax: float = 22050.0, pitch_std: float = 20.0, speaking_rate: float = 15.0,
                   vqscore_8: list[float] = [0.78] * 8, ctc_loss: float = 0.0, dnsmos_ovrl: float = 4.0,
                   speaker_noised: bool = False, unconditional_keys: Iterable[str] = {"vqscore_8", "dnsmos_ovrl"},
                   device: torch.device | str = "cpu", text: str | None = None) -> dict:
    """conditioning.py:326-395 with phoneme input (`text` needs the out-of-scope eSpeak front-end)."""
    if phonemes is None:
        raise NotImplementedError("text -> phonemes needs eSpeak (out of scope): pass phonemes=")
    assert language.lower() in LANGUAGE_ID, "Please pick a supported language"
    d = {
        "espeak": ([phonemes], [language]),
        "speaker": speaker,
        "emotion": emotion,
        "fmax": fmax,
        "pitch_std": pitch_std,
        "speaking_rate": speaking_rate,
        "language_id": LANGUAGE_ID[language],
        "vqscore_8": vqscore_8,
        "ctc_loss": ctc_loss,
        "dnsmos_ovrl": dnsmos_ovrl,
        "speaker_noised": int(speaker_noised),
    }
    for k in unconditional_keys:
        d.pop(k, None)
    for k, v in d.items():
        if isinstance(v, (float, int, list)):
            v = torch.tensor(v)
        if isinstance(v, torch.Tensor):
            d[k] = v.view(1, 1, -1).to(device)
        if k == "emotion":
            d[k] /= d[k].sum(dim=-1)
    return d


_KIND_OF_TYPE = {"FourierConditioner": _lib.COND_FOURIER, "IntegerConditioner": _lib.COND_EMBED,
                 "EspeakPhonemeConditioner": _lib.COND_EMBED}


class PrefixConditioner:
    """HIP prefix conditioner. Parameters use the reference state-dict names under
    `prefix_conditioner.` (conditioning.py:284-291), bf16 on the device."""

    def __init__(self, conditioners: list[dict], d: int, device="cuda", projection: str = "none",
                 eps: float = 1e-5):
        if projection != "none":
            raise NotImplementedError("PrefixConditioner projection other than 'none'")
        self.cfgs = [dict(c) for c in conditioners]
        for c in self.cfgs:
            if c["type"] not in ("EspeakPhonemeConditioner", "FourierConditioner", "IntegerConditioner",
                                 "PassthroughConditioner"):
                raise ValueError(f"unknown conditioner type {c['type']}")
            if c.get("projection", "none") not in ("none", "linear"):
                raise NotImplementedError(f"conditioner projection {c.get('projection')!r}")
        self.d, self.dev, self.eps = d, torch.device(device), eps
        self.required_keys = {c["name"] for c in self.cfgs if c.get("uncond_type", "none") != "learned"}
        self.w: dict[str, torch.Tensor] = {}
        self._params = None

    # ------------------------------------------------------------------ parameters
    def param_shapes(self) -> dict[str, tuple]:
        d, out = self.d, {"norm.weight": (self.d,), "norm.bias": (self.d,)}
        for i, c in enumerate(self.cfgs):
            p = f"conditioners.{i}."
            t = c["type"]
            if t == "EspeakPhonemeConditioner":
                out[p + "phoneme_embedder.weight"] = (PHONEME_VOCAB, d)
            elif t == "FourierConditioner":
                out[p + "weight"] = (d // 2, c.get("input_dim", 1))
            elif t == "IntegerConditioner":
                out[p + "int_embedder.weight"] = (c.get("max_val", 512) - c.get("min_val", 0) + 1, d)
            cd = c.get("cond_dim") or d
            if c.get("projection", "none") == "linear":
                out[p + "project.weight"] = (d, cd)
                out[p + "project.bias"] = (d,)
            if c.get("uncond_type", "none") == "learned":
                out[p + "uncond_vector"] = (d,)
        return out

    def load_state_dict(self, sd: dict, prefix: str = ""):
        for name, shape in self.param_shapes().items():
            t = sd[prefix + name]
            if tuple(t.shape) != shape:
                raise ValueError(f"{name}: shape {tuple(t.shape)} != {shape}")
            self.w[name] = t.to(device=self.dev, dtype=torch.bfloat16).contiguous()
        self._params = None

    def _param_block(self) -> torch.Tensor:
        """Device array of ZmiCondParam: 2 entries per conditioner (conditional, learned uncond)."""
        if self._params is None:
            arr = (_lib.CondParam * (2 * len(self.cfgs)))()
            for i, c in enumerate(self.cfgs):
                p, t = f"conditioners.{i}.", c["type"]
                cp = arr[2 * i]
                cp.min_val, cp.max_val = float(c.get("min_val", 0.0)), float(c.get("max_val", 1.0))
                if t == "EspeakPhonemeConditioner":
                    cp.table = self.w[p + "phoneme_embedder.weight"].data_ptr()
                elif t == "IntegerConditioner":
                    cp.table = self.w[p + "int_embedder.weight"].data_ptr()
                elif t == "FourierConditioner":
                    cp.weight, cp.in_dim = self.w[p + "weight"].data_ptr(), c.get("input_dim", 1)
                    if cp.in_dim > 256:
                        raise ValueError("Fourier conditioner input wider than 256")
                elif t == "PassthroughConditioner":
                    cp.in_dim = c.get("cond_dim") or self.d
                    if c.get("projection", "none") == "linear":
                        cp.weight = self.w[p + "project.weight"].data_ptr()
                        cp.bias = self.w[p + "project.bias"].data_ptr()
                        if cp.in_dim > 256:
                            raise ValueError("linear conditioner input wider than 256")
                if c.get("uncond_type", "none") == "learned":
                    arr[2 * i + 1].table = self.w[p + "uncond_vector"].data_ptr()
            raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            self._params = raw.to(self.dev)
        return self._params

    # ------------------------------------------------------------------ rows
    def _rows(self, cond_dict: dict, rows: list, xs: list[float]):
        if not set(cond_dict).issuperset(self.required_keys):
            raise ValueError(f"Missing required keys: {self.required_keys - set(cond_dict)}")
        for i, c in enumerate(self.cfgs):
            v, t = cond_dict.get(c["name"]), c["type"]
            if v is None:
                if c.get("uncond_type", "none") != "learned":
                    raise ValueError(f"conditioner {c['name']} has no unconditional vector")
                rows.append((2 * i + 1, _lib.COND_VECTOR, 0, 0))
                continue
            if t == "EspeakPhonemeConditioner":
                phonemes, _langs = v
                if len(phonemes) != 1:
                    raise ValueError("one utterance per cond_dict (reference generate() is batch_size=1)")
                ids, _ = tokenize_phonemes(list(phonemes))
                rows.extend((2 * i, _lib.COND_EMBED, int(k), 0) for k in ids[0].tolist())
                continue
            x = v.reshape(v.shape[0], -1) if v.dim() >= 2 else v.reshape(1, -1)
            if x.shape[0] != 1:
                raise ValueError(f"{c['name']}: one utterance per cond_dict")
            x = x[0]
            if t == "IntegerConditioner":
                if x.numel() != 1:
                    raise ValueError(f"{c['name']}: expects one integer")
                idx = int(x.item()) - int(c.get("min_val", 0))
                n = int(c.get("max_val", 512)) - int(c.get("min_val", 0)) + 1
                if not 0 <= idx < n:
                    raise IndexError(f"{c['name']}: value out of range")
                rows.append((2 * i, _lib.COND_EMBED, idx, 0))
            elif t == "FourierConditioner":
                if x.numel() != c.get("input_dim", 1):
                    raise ValueError(f"{c['name']}: expects {c.get('input_dim', 1)} values")
                rows.append((2 * i, _lib.COND_FOURIER, 0, len(xs)))
                xs.extend(x.to(torch.float32).cpu().tolist())
            else:  # Passthrough
                cd = c.get("cond_dim") or self.d
                if x.numel() != cd:
                    raise ValueError(f"{c['name']}: expects {cd} values")
                if c.get("projection", "none") == "linear" and x.dtype != torch.bfloat16:
                    raise TypeError(f"{c['name']}: the bf16 projection needs a bf16 input (reference dtype rule)")
                kind = _lib.COND_LINEAR if c.get("projection", "none") == "linear" else _lib.COND_PASSTHROUGH
                rows.append((2 * i, kind, 0, len(xs)))
                xs.extend(x.to(torch.float32).cpu().tolist())

    def prepare_conditioning(self, cond_dict: dict, uncond_dict: dict | None = None, stream=None) -> torch.Tensor:
        """[2, Lc, d] bf16: the conditional rows, then the unconditional ones (model.py:204-212)."""
        if uncond_dict is None:
            uncond_dict = {k: cond_dict[k] for k in self.required_keys}
        rows_c: list = []
        rows_u: list = []
        xs: list[float] = []
        self._rows(cond_dict, rows_c, xs)
        self._rows(uncond_dict, rows_u, xs)
        if len(rows_c) != len(rows_u):
            raise ValueError("cond and uncond conditioning lengths differ")
        rows = torch.tensor(rows_c + rows_u, dtype=torch.int32).to(self.dev)
        x = torch.tensor(xs if xs else [0.0], dtype=torch.float32).to(self.dev)
        out = torch.empty(2, len(rows_c), self.d, dtype=torch.bfloat16, device=self.dev)
        s = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        _lib.check(_lib.lib().zmi_prefix_condition(self._param_block().data_ptr(), rows.data_ptr(), rows.shape[0],
                                                   x.data_ptr(), self.d, self.w["norm.weight"].data_ptr(),
                                                   self.w["norm.bias"].data_ptr(), self.eps, out.data_ptr(), s),
                   "prefix_condition")
        return out

    def __call__(self, cond_dict: dict) -> torch.Tensor:
        """PrefixConditioner.forward for one cond_dict: [1, Lc, d]."""
        rows: list = []
        xs: list[float] = []
        self._rows(cond_dict, rows, xs)
        r = torch.tensor(rows, dtype=torch.int32).to(self.dev)
        x = torch.tensor(xs if xs else [0.0], dtype=torch.float32).to(self.dev)
        out = torch.empty(1, len(rows), self.d, dtype=torch.bfloat16, device=self.dev)
        _lib.check(_lib.lib().zmi_prefix_condition(self._param_block().data_ptr(), r.data_ptr(), r.shape[0],
                                                   x.data_ptr(), self.d, self.w["norm.weight"].data_ptr(),
                                                   self.w["norm.bias"].data_ptr(), self.eps, out.data_ptr(),
                                                   torch.cuda.current_stream(self.dev).cuda_stream),
                   "prefix_condition")
        return out


__all__ = ["PrefixConditioner", "make_cond_dict", "tokenize_phonemes", "v01_transformer_conditioners",
           "SUPPORTED_LANGUAGE_CODES", "PHONEME_VOCAB"]
