"""DACAutoencoder with the reference's decode() surface (zonos/autoencoder.py:8-27), on HIP kernels.

Only the decoder path is on the hot path: quantizer.from_codes +
DacDecoder. `encode`/`preprocess` (voice-clone prefix) are not built.

Weights use transformers' DacModel state_dict names (quantizer.quantizers.{i}.*, decoder.*);
weight-norm pairs (weight_g, weight_v) are folded to plain weights at load time.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from . import synthetic as syn
from .config import DAC_HOP, DAC_SAMPLE_RATE, N_CODEBOOKS

STRIDES = syn.DAC_STRIDES
DILATIONS = syn.DAC_DILATIONS


def _fold_weight_norm(sd: dict) -> dict:
    out = dict(sd)
    for k in list(sd):
        if k.endswith(".weight_g"):
            base = k[: -len(".weight_g")]
            g, v = sd[k].float(), sd[base + ".weight_v"].float()
            norm = v.flatten(1).norm(dim=1).view(-1, *([1] * (v.dim() - 1)))
            out[base + ".weight"] = g * v / norm
            del out[k], out[base + ".weight_v"]
    return out


class DACAutoencoder:
    codebook_size = 1024
    num_codebooks = N_CODEBOOKS
    sampling_rate = DAC_SAMPLE_RATE

    def __init__(self, device="cuda", state_dict: dict | None = None, seed: int = 0):
        self.dev = torch.device(device)
        self.lib = _lib.lib()
        self.stream = torch.cuda.Stream(self.dev)
        self.sptr = self.stream.cuda_stream
        if state_dict is None:
            state_dict = {}
            with torch.cuda.stream(self.stream):
                for sp in syn.dac_specs():
                    t = torch.empty(sp.shape, dtype=torch.float32, device=self.dev)
                    _lib.check(self.lib.zmi_fill_uniform(t.data_ptr(), sp.numel, syn.tensor_key(seed, sp.name),
                                                         sp.scale, sp.offset, 1, self.sptr), "fill")
                    state_dict[sp.name] = t
        self._prepare(_fold_weight_norm(state_dict))
        self._bufs = None

    # --------------------------------------------------------------- weight layout
    def _prepare(self, sd: dict):
        f32 = lambda t: t.to(self.dev, torch.float32).contiguous()  # noqa: E731

        def conv_w(w):  # [co][ci][k] -> [k][co][ci] fp16
            return w.to(self.dev, torch.float32).permute(2, 0, 1).contiguous().half()

        with torch.cuda.stream(self.stream):
            q = "quantizer.quantizers."
            self.codebooks = torch.stack([f32(sd[f"{q}{i}.codebook.weight"]) for i in range(N_CODEBOOKS)]).contiguous()
            self.proj_w = torch.stack([f32(sd[f"{q}{i}.out_proj.weight"]).reshape(-1, 8)
                                       for i in range(N_CODEBOOKS)]).contiguous()
            self.proj_b = torch.stack([f32(sd[f"{q}{i}.out_proj.bias"]) for i in range(N_CODEBOOKS)]).contiguous()
            self.c1_w, self.c1_b = conv_w(sd["decoder.conv1.weight"]), f32(sd["decoder.conv1.bias"])
            self.blocks = []
            for j, s in enumerate(STRIDES):
                p = f"decoder.block.{j}."
                wt = sd[p + "conv_t1.weight"].to(self.dev, torch.float32)  # [cin][cout][2s]
                pad = math.ceil(s / 2)
                phases = []
                for rho in range(s):
                    k0 = (rho + pad) % s
                    taps = torch.stack([wt[:, :, k0].t(), wt[:, :, k0 + s].t()])  # [2][cout][cin]
                    phases.append((taps.contiguous().half(), (rho + pad) // s))
                blk = dict(stride=s, cin=wt.shape[0], cout=wt.shape[1], alpha=f32(sd[p + "snake1.alpha"]).reshape(-1),
                           phases=phases, bt=f32(sd[p + "conv_t1.bias"]), res=[])
                for u in range(3):
                    r = p + f"res_unit{u + 1}."
                    blk["res"].append(dict(a1=f32(sd[r + "snake1.alpha"]).reshape(-1),
                                           w1=conv_w(sd[r + "conv1.weight"]), b1=f32(sd[r + "conv1.bias"]),
                                           a2=f32(sd[r + "snake2.alpha"]).reshape(-1),
                                           w2=conv_w(sd[r + "conv2.weight"]), b2=f32(sd[r + "conv2.bias"])))
                self.blocks.append(blk)
            self.final_alpha = f32(sd["decoder.snake1.alpha"]).reshape(-1)
            self.out_w = f32(sd["decoder.conv2.weight"]).reshape(-1)        # [96 * 7]
            self.out_b = float(sd["decoder.conv2.bias"].float().reshape(-1)[0])
        self.stream.synchronize()

    def _buffers(self, T: int):
        need = 49152 * T  # max over stages of C x time (blocks 3 and 4: 192 x 256T = 96 x 512T)
        if self._bufs is None or self._bufs[0].numel() < need:
            with torch.cuda.stream(self.stream):
                self._bufs = [torch.empty(need, dtype=torch.float16, device=self.dev) for _ in range(4)]
        return self._bufs

    # --------------------------------------------------------------- decode
    def _conv(self, x, t_in, c_in, w, b, c_out, taps, step, off, n_out, stride, phase, t_out, skip=None, raw=None,
              snake=None, alpha=None):
        p = _lib.ptr
        _lib.check(self.lib.zmi_dac_conv(p(x), t_in, c_in, p(w), p(b), c_out, taps, step, off, n_out, stride, phase,
                                         t_out, p(skip), p(raw), p(snake), p(alpha), self.sptr), "dac_conv")

    def _decode_one(self, codes: torch.Tensor, out: torch.Tensor):
        """codes [9, T] int64 (device) -> out [512 T] fp32 (modeling_dac.py:347-371, 407-441)."""
        T = codes.shape[-1]
        H, SA, SB, S2 = self._buffers(T)
        z = S2
        _lib.check(self.lib.zmi_dac_from_codes(codes.data_ptr(), T, self.codebooks.data_ptr(), self.proj_w.data_ptr(),
                                               self.proj_b.data_ptr(), z.data_ptr(), self.sptr), "from_codes")
        c = self.c1_w.shape[1]
        # conv1 (k7, pad 3) -> Snake of block 0 (its only consumer is block 0's ConvTranspose)
        self._conv(z, T, self.c1_w.shape[2], self.c1_w, self.c1_b, c, 7, 1, -3, T, 1, 0, T, snake=SA,
                   alpha=self.blocks[0]["alpha"])
        t = T
        xin, xalt = SA, SB
        for j, blk in enumerate(self.blocks):
            s, cin, cout = blk["stride"], blk["cin"], blk["cout"]
            tn = t * s
            res = blk["res"]
            for rho, (wp, coff) in enumerate(blk["phases"]):  # polyphase ConvTranspose1d(k=2s, s, pad=ceil(s/2))
                self._conv(xin, t, cin, wp, blk["bt"], cout, 2, -1, coff, t, s, rho, tn, raw=H, snake=xalt,
                           alpha=res[0]["a1"])
            for u, dil in enumerate(DILATIONS):
                ru = res[u]
                self._conv(xalt, tn, cout, ru["w1"], ru["b1"], cout, 7, dil, -3 * dil, tn, 1, 0, tn, snake=S2,
                           alpha=ru["a2"])
                last_unit = u == len(DILATIONS) - 1
                if not last_unit:
                    nxt = res[u + 1]["a1"]
                elif j + 1 < len(self.blocks):
                    nxt = self.blocks[j + 1]["alpha"]
                else:
                    nxt = self.final_alpha
                self._conv(S2, tn, cout, ru["w2"], ru["b2"], cout, 1, 0, 0, tn, 1, 0, tn, skip=H,
                           raw=None if last_unit else H, snake=xalt, alpha=nxt)
            t = tn
            xin, xalt = xalt, xin
        _lib.check(self.lib.zmi_dac_conv_out(xin.data_ptr(), t, self.blocks[-1]["cout"], self.out_w.data_ptr(),
                                             self.out_b, out.data_ptr(), self.sptr), "conv_out")

    @torch.inference_mode()
    def decode(self, codes: torch.Tensor) -> torch.Tensor:
        """[B, 9, T] codes -> [B, 1, 512 T] fp32 waveform (reference autoencoder.py:25-27)."""
        B, nq, T = codes.shape
        assert nq == N_CODEBOOKS
        out = torch.empty(B, 1, DAC_HOP * T, dtype=torch.float32, device=self.dev)
        cur = torch.cuda.current_stream(self.dev)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            codes = codes.to(self.dev, torch.int64).contiguous()
            for b in range(B):
                self._decode_one(codes[b], out[b, 0])
        cur.wait_stream(self.stream)
        return out
