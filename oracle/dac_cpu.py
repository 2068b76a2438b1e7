"""ORACLE — CPU restatement of DACAutoencoder.decode (44.1 kHz DAC decoder). TEST INFRASTRUCTURE ONLY.

Restates, with the same ATen ops, the third-party path the reference calls
(`zonos/autoencoder.py:25-27` -> transformers `DacModel.decode`):

  from_codes      modeling_dac.py:347-371  (codebook gather -> 1x1 out_proj, summed over 9 codebooks)
  DacDecoder      modeling_dac.py:407-441  (conv k7 -> 4 x DecoderBlock -> Snake -> conv k7 -> tanh)
  DacDecoderBlock modeling_dac.py:236-264  (Snake -> ConvTranspose(k=2s, s, p=ceil(s/2)) -> 3 x ResUnit)
  DacResidualUnit modeling_dac.py:175-209  (Snake -> conv k7 dil d -> Snake -> conv 1x1 -> + skip)
  Snake1d         modeling_dac.py:86-100   (x + 1/(a+1e-9) * sin(a x)^2)

and the encode path (`zonos/autoencoder.py:17-23` -> `DacModel.encode`, modeling_dac.py:583-608):

  DacEncoder      modeling_dac.py:444-475  (conv k7 -> 4 x EncoderBlock -> Snake -> conv k3)
  DacEncoderBlock modeling_dac.py:212-234  (3 x ResUnit -> Snake -> conv(k=2s, s, p=ceil(s/2)))
  DacResidualVectorQuantizer.forward :283-345, DacVectorQuantize :123-173 (in_proj, l2-normalised
                  nearest codebook entry, out_proj of p + (q - p), residual -= it)

The CPU reference runs fp32 (autocast is disabled on CPU, autoencoder.py:26), so this is the
fp32 oracle; the GPU path is compared to it with the tolerance stated in its test.
Pinned against transformers' own DacModel in tests/golden (make_golden.py, `dac_*` fixtures).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

STRIDES = (8, 8, 4, 2)
ENC_STRIDES = (2, 4, 8, 8)
DILATIONS = (1, 3, 9)


def snake(x: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    shp = x.shape
    x = x.reshape(shp[0], shp[1], -1)
    x = x + (alpha + 1e-9).reciprocal() * torch.sin(alpha * x).pow(2)
    return x.reshape(shp)


class OracleDAC:
    def __init__(self, weights: dict):
        self.w = weights

    def from_codes(self, codes: torch.Tensor) -> torch.Tensor:
        q = 0.0
        for i in range(codes.shape[1]):
            p = f"quantizer.quantizers.{i}."
            lat = F.embedding(codes[:, i, :], self.w[p + "codebook.weight"]).transpose(1, 2)
            q = q + F.conv1d(lat, self.w[p + "out_proj.weight"], self.w[p + "out_proj.bias"])
        return q

    def _res_unit(self, x, p, dil):
        y = F.conv1d(snake(x, self.w[p + "snake1.alpha"]), self.w[p + "conv1.weight"], self.w[p + "conv1.bias"],
                     dilation=dil, padding=3 * dil)
        y = F.conv1d(snake(y, self.w[p + "snake2.alpha"]), self.w[p + "conv2.weight"], self.w[p + "conv2.bias"])
        pad = (x.shape[-1] - y.shape[-1]) // 2
        if pad > 0:
            x = x[..., pad:-pad]
        return x + y

    def decoder(self, z: torch.Tensor) -> torch.Tensor:
        h = F.conv1d(z, self.w["decoder.conv1.weight"], self.w["decoder.conv1.bias"], padding=3)
        for j, s in enumerate(STRIDES):
            p = f"decoder.block.{j}."
            h = snake(h, self.w[p + "snake1.alpha"])
            h = F.conv_transpose1d(h, self.w[p + "conv_t1.weight"], self.w[p + "conv_t1.bias"], stride=s,
                                   padding=math.ceil(s / 2))
            for u, d in enumerate(DILATIONS):
                h = self._res_unit(h, p + f"res_unit{u + 1}.", d)
        h = snake(h, self.w["decoder.snake1.alpha"])
        h = F.conv1d(h, self.w["decoder.conv2.weight"], self.w["decoder.conv2.bias"], padding=3)
        return torch.tanh(h)

    @torch.inference_mode()
    def decode(self, codes: torch.Tensor) -> torch.Tensor:
        """autoencoder.py:25-27 on CPU: [B, 9, T] int64 -> [B, 1, 512 T] fp32."""
        return self.decoder(self.from_codes(codes)).squeeze(1).unsqueeze(1).float()

    # ------------------------------------------------------------------ encode
    def encoder(self, wav: torch.Tensor) -> torch.Tensor:
        """[B, 1, T] fp32 -> latents [B, 1024, T / 512] (modeling_dac.py:464-475)."""
        h = F.conv1d(wav, self.w["encoder.conv1.weight"], self.w["encoder.conv1.bias"], padding=3)
        for j, s in enumerate(ENC_STRIDES):
            p = f"encoder.block.{j}."
            for u, d in enumerate(DILATIONS):
                h = self._res_unit(h, p + f"res_unit{u + 1}.", d)
            h = snake(h, self.w[p + "snake1.alpha"])
            h = F.conv1d(h, self.w[p + "conv1.weight"], self.w[p + "conv1.bias"], stride=s, padding=math.ceil(s / 2))
        h = snake(h, self.w["encoder.snake1.alpha"])
        return F.conv1d(h, self.w["encoder.conv2.weight"], self.w["encoder.conv2.bias"], padding=1)

    def quantize(self, latents: torch.Tensor, n_q: int = 9):
        """Residual VQ (modeling_dac.py:283-345, :123-173) -> codes [B, 9, T] and, per decision, the gap
        between the best and second-best score (the near-tie margin)."""
        residual = latents
        codes, margins = [], []
        for i in range(n_q):
            p = f"quantizer.quantizers.{i}."
            proj = F.conv1d(residual, self.w[p + "in_proj.weight"], self.w[p + "in_proj.bias"])
            b, dim, t = proj.shape
            enc = F.normalize(proj.permute(0, 2, 1).reshape(b * t, dim))
            cb = F.normalize(self.w[p + "codebook.weight"])
            l2 = enc.pow(2).sum(1, keepdim=True)
            dist = -(l2 - 2 * enc @ cb.t()) + cb.pow(2).sum(1, keepdim=True).t()
            idx = dist.max(1)[1]
            top2 = dist.topk(2, dim=1).values
            margins.append((top2[:, 0] - top2[:, 1]).reshape(b, t))
            q = F.embedding(idx.reshape(b, t), self.w[p + "codebook.weight"]).transpose(1, 2)
            q = proj + (q - proj)
            residual = residual - F.conv1d(q, self.w[p + "out_proj.weight"], self.w[p + "out_proj.bias"])
            codes.append(idx.reshape(b, t))
        return torch.stack(codes, dim=1), torch.stack(margins, dim=1)

    @torch.inference_mode()
    def encode(self, wav: torch.Tensor) -> torch.Tensor:
        """autoencoder.py:22-23 on CPU: [B, 1, 512 T] fp32 -> codes [B, 9, T] int64."""
        return self.quantize(self.encoder(wav))[0]
