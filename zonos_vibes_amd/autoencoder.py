"""DACAutoencoder with the reference's decode() surface (zonos/autoencoder.py:8-27), on HIP kernels.

The decoder path is on the hot path: quantizer.from_codes + DacDecoder.
`encode` (voice-clone audio prefix) runs DacEncoder + the residual VQ on the
same MFMA conv kernel (strided convs in polyphase form) plus a VQ kernel; `preprocess` pads to a
multiple of 512 samples (resampling needs torchaudio, absent here: only 44.1 kHz input is taken).

Weights use transformers' DacModel state_dict names (quantizer.quantizers.{i}.*, decoder.*);
weight-norm pairs (weight_g / weight_v, or parametrizations.weight.original0 / original1) are
folded to plain weights at load time.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from . import synthetic as syn
from .config import DAC_HOP, DAC_SAMPLE_RATE, N_CODEBOOKS

STRIDES = syn.DAC_STRIDES
ENC_STRIDES = syn.DAC_ENC_STRIDES
DILATIONS = syn.DAC_DILATIONS


def _fold_weight_norm(sd: dict) -> dict:
    """Plain conv weights from weight-norm pairs, in either of the two key styles a DAC state_dict
    can carry: `x.weight_g` / `x.weight_v` (torch.nn.utils.weight_norm, the published checkpoint)
    or `x.parametrizations.weight.original0` / `.original1` (torch.nn.utils.parametrizations.weight_norm,
    what transformers' DacModel.apply_weight_norm registers): weight = g * v / ||v|| over all dims
    but the first (dim=0, torch's default)."""
    out = dict(sd)
    for gk, vk, base in [(k, k[: -len("_g")] + "_v", k[: -len(".weight_g")]) for k in sd if k.endswith(".weight_g")] + \
            [(k, k[: -1] + "1", k[: -len(".parametrizations.weight.original0")])
             for k in sd if k.endswith(".parametrizations.weight.original0")]:
        g, v = sd[gk].float(), sd[vk].float()
        norm = v.flatten(1).norm(dim=1).view(-1, *([1] * (v.dim() - 1)))
        out[base + ".weight"] = g * v / norm
        del out[gk], out[vk]
    return out


def _blocked(w: torch.Tensor) -> torch.Tensor:
    """[..., co, ci] conv weights -> fp16 channel-blocked [..., ci / 32, co, 32]: the layout zmi_dac_conv* read for
    convs with more than one tap, in which one 32-channel step of 16 output channels (one LDS-DMA piece, 16 x 64 B)
    is 1 KiB contiguous (1x1 convs keep [co][ci], include/zonos_hip.h)."""
    co, ci = w.shape[-2], w.shape[-1]
    assert ci % 32 == 0, ci
    return w.reshape(*w.shape[:-1], ci // 32, 32).transpose(-3, -2).contiguous().half()


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
                for sp in syn.dac_specs() + syn.dac_encoder_specs():
                    t = torch.empty(sp.shape, dtype=torch.float32, device=self.dev)
                    _lib.check(self.lib.zmi_fill_uniform(t.data_ptr(), sp.numel, syn.tensor_key(seed, sp.name),
                                                         sp.scale, sp.offset, 1, self.sptr), "fill")
                    state_dict[sp.name] = t
        self._prepare(_fold_weight_norm(state_dict))
        self._bufs = None

    # --------------------------------------------------------------- weight layout
    def _prepare(self, sd: dict):
        f32 = lambda t: t.to(self.dev, torch.float32).contiguous()  # noqa: E731

        def conv_w(w):  # [co][ci][k] -> channel-blocked [k][ci / 32][co][32] fp16 (_blocked); 1x1: [1][co][ci]
            w = w.to(self.dev, torch.float32).permute(2, 0, 1)
            return w.contiguous().half() if w.shape[0] == 1 else _blocked(w)

        with torch.cuda.stream(self.stream):
            q = "quantizer.quantizers."
            self.codebooks = torch.stack([f32(sd[f"{q}{i}.codebook.weight"]) for i in range(N_CODEBOOKS)]).contiguous()
            self.proj_w = torch.stack([f32(sd[f"{q}{i}.out_proj.weight"]).reshape(-1, 8)
                                       for i in range(N_CODEBOOKS)]).contiguous()
            self.proj_b = torch.stack([f32(sd[f"{q}{i}.out_proj.bias"]) for i in range(N_CODEBOOKS)]).contiguous()
            self.c1_w, self.c1_b = conv_w(sd["decoder.conv1.weight"]), f32(sd["decoder.conv1.bias"])
            self.c1_cin, self.c1_cout = sd["decoder.conv1.weight"].shape[1], sd["decoder.conv1.weight"].shape[0]
            self.blocks = []
            for j, s in enumerate(STRIDES):
                p = f"decoder.block.{j}."
                wt = sd[p + "conv_t1.weight"].to(self.dev, torch.float32)  # [cin][cout][2s]
                pad = math.ceil(s / 2)
                phases = []
                for rho in range(s):  # polyphase: phase rho uses taps (rho + pad) % s and + s, transposed
                    k0 = (rho + pad) % s
                    phases.append(torch.stack([wt[:, :, k0].t(), wt[:, :, k0 + s].t()]))  # [2][cout][cin]
                blk = dict(stride=s, pad=pad, cin=wt.shape[0], cout=wt.shape[1],
                           alpha=f32(sd[p + "snake1.alpha"]).reshape(-1),
                           wt=_blocked(torch.stack(phases)), bt=f32(sd[p + "conv_t1.bias"]), res=[])
                for u in range(3):
                    r = p + f"res_unit{u + 1}."
                    blk["res"].append(dict(a1=f32(sd[r + "snake1.alpha"]).reshape(-1),
                                           w1=conv_w(sd[r + "conv1.weight"]), b1=f32(sd[r + "conv1.bias"]),
                                           a2=f32(sd[r + "snake2.alpha"]).reshape(-1),
                                           w2=conv_w(sd[r + "conv2.weight"]), b2=f32(sd[r + "conv2.bias"])))
                self.blocks.append(blk)
            self.final_alpha = f32(sd["decoder.snake1.alpha"]).reshape(-1)
            w2 = f32(sd["decoder.conv2.weight"])                              # [1][96][7]
            self.out_w = torch.zeros(7, 32, w2.shape[1], device=self.dev)     # [k][co padded to 32][ci]
            self.out_w[:, 0, :] = w2[0].t()
            self.out_w = _blocked(self.out_w)
            self.out_b = torch.zeros(32, device=self.dev)
            self.out_b[0] = f32(sd["decoder.conv2.bias"]).reshape(-1)[0]
            self.has_encoder = "encoder.conv1.weight" in sd
            if self.has_encoder:
                self._prepare_encoder(sd, f32, conv_w)
        self.stream.synchronize()

    def _prepare_encoder(self, sd, f32, conv_w):
        w1 = f32(sd["encoder.conv1.weight"])                                  # [64][1][7]
        col = torch.zeros(1, w1.shape[0], 32, device=self.dev)
        col[0, :, :7] = w1[:, 0, :]
        self.e1_w, self.e1_b = col.half().contiguous(), f32(sd["encoder.conv1.bias"])  # 1x1: [1][co][ci]
        self.eblocks = []
        c = w1.shape[0]
        for j, s in enumerate(ENC_STRIDES):
            p = f"encoder.block.{j}."
            res = [dict(a1=f32(sd[p + f"res_unit{u + 1}.snake1.alpha"]).reshape(-1),
                        w1=conv_w(sd[p + f"res_unit{u + 1}.conv1.weight"]), b1=f32(sd[p + f"res_unit{u + 1}.conv1.bias"]),
                        a2=f32(sd[p + f"res_unit{u + 1}.snake2.alpha"]).reshape(-1),
                        w2=conv_w(sd[p + f"res_unit{u + 1}.conv2.weight"]), b2=f32(sd[p + f"res_unit{u + 1}.conv2.bias"]))
                   for u in range(3)]
            # Conv1d(c, 2c, k=2s, stride s, pad ceil(s/2)) over the polyphase view x'[t][j*c + ci] = x[s t + j][ci]:
            # out[t] = sum_{a=-1..1} W'[a] x'[t + a] with W'[a][co][j*c + ci] = W[co][ci][s a + j + pad] (0 if
            # that tap is outside [0, 2s)) -- a stride-1, 3-tap conv with c_in = s*c
            wt = f32(sd[p + "conv1.weight"])                                   # [2c][c][2s]
            pad = math.ceil(s / 2)
            wp = torch.zeros(3, 2 * c, s, c, device=self.dev)
            for a in range(3):
                for jj in range(s):
                    k = s * (a - 1) + jj + pad
                    if 0 <= k < 2 * s:
                        wp[a, :, jj, :] = wt[:, :, k]
            self.eblocks.append(dict(stride=s, c=c, res=res, alpha=f32(sd[p + "snake1.alpha"]).reshape(-1),
                                     w=_blocked(wp.reshape(3, 2 * c, s * c)), b=f32(sd[p + "conv1.bias"])))
            c *= 2
        self.e_final_alpha = f32(sd["encoder.snake1.alpha"]).reshape(-1)
        self.e2_w, self.e2_b = conv_w(sd["encoder.conv2.weight"]), f32(sd["encoder.conv2.bias"])
        self.e2_cin, self.e2_cout = sd["encoder.conv2.weight"].shape[1], sd["encoder.conv2.weight"].shape[0]
        q = "quantizer.quantizers."
        self.vq_in_w = torch.stack([f32(sd[f"{q}{i}.in_proj.weight"]).reshape(8, -1) for i in range(N_CODEBOOKS)])
        self.vq_in_b = torch.stack([f32(sd[f"{q}{i}.in_proj.bias"]) for i in range(N_CODEBOOKS)]).contiguous()
        # l2-normalised codebooks and their squared norms: load-time weight preparation (modeling_dac.py:163-168)
        self.cb_n = torch.nn.functional.normalize(self.codebooks, dim=-1).contiguous()
        self.cb_n2 = self.cb_n.pow(2).sum(-1).contiguous()

    def _buffers(self, T: int):
        need = 49152 * T  # max over stages of C x time (blocks 3 and 4: 192 x 256T = 96 x 512T)
        if self._bufs is None or self._bufs[0].numel() < need:
            with torch.cuda.stream(self.stream):
                self._bufs = [torch.empty(need, dtype=torch.float16, device=self.dev) for _ in range(4)]
        return self._bufs

    # --------------------------------------------------------------- decode
    def _conv(self, x, t_in, c_in, w, b, c_out, taps, step, off, n_out, stride, phase, t_out, skip=None, raw=None,
              snake=None, alpha=None, f32=None):
        p = _lib.ptr
        _lib.check(self.lib.zmi_dac_conv(p(x), t_in, c_in, p(w), p(b), c_out, taps, step, off, n_out, stride, phase,
                                         t_out, p(skip), p(raw), p(snake), p(alpha), p(f32), self.sptr), "dac_conv")

    def _decode_one(self, codes: torch.Tensor, out: torch.Tensor):
        """codes [9, T] int64 (device) -> out [512 T] fp32 (modeling_dac.py:347-371, 407-441)."""
        T = codes.shape[-1]
        H, SA, SB, S2 = self._buffers(T)
        z = S2
        _lib.check(self.lib.zmi_dac_from_codes(codes.data_ptr(), T, self.codebooks.data_ptr(), self.proj_w.data_ptr(),
                                               self.proj_b.data_ptr(), z.data_ptr(), self.sptr), "from_codes")
        c = self.c1_cout
        # conv1 (k7, pad 3) -> Snake of block 0 (its only consumer is block 0's ConvTranspose)
        self._conv(z, T, self.c1_cin, self.c1_w, self.c1_b, c, 7, 1, -3, T, 1, 0, T, snake=SA,
                   alpha=self.blocks[0]["alpha"])
        t = T
        xin, xalt = SA, SB
        for j, blk in enumerate(self.blocks):
            s, cin, cout = blk["stride"], blk["cin"], blk["cout"]
            tn = t * s
            res = blk["res"]
            # ConvTranspose1d(k=2s, s, pad=ceil(s/2)), every phase in one launch
            _lib.check(self.lib.zmi_dac_conv_t(xin.data_ptr(), t, cin, blk["wt"].data_ptr(), blk["bt"].data_ptr(),
                                               cout, s, blk["pad"], H.data_ptr(), xalt.data_ptr(),
                                               res[0]["a1"].data_ptr(), self.sptr), "dac_conv_t")
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
                                             self.out_b.data_ptr(), out.data_ptr(), self.sptr), "conv_out")

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

    # --------------------------------------------------------------- encode
    def preprocess(self, wav: torch.Tensor, sr: int) -> torch.Tensor:
        """autoencoder.py:17-20: resample to 44.1 kHz (identity only: torchaudio is absent) and right-pad to
        a multiple of 512 samples."""
        if sr != DAC_SAMPLE_RATE:
            raise NotImplementedError(f"resampling {sr} Hz -> 44.1 kHz needs torchaudio (absent in this build)")
        right = math.ceil(wav.shape[-1] / DAC_HOP) * DAC_HOP - wav.shape[-1]
        return torch.nn.functional.pad(wav, (0, right))

    def _encoder_buffers(self, n: int):
        need = 64 * (n + 8)
        if getattr(self, "_ebufs", None) is None or self._ebufs[0].numel() < need:
            with torch.cuda.stream(self.stream):
                self._ebufs = [torch.empty(need, dtype=torch.float16, device=self.dev) for _ in range(3)]
        return self._ebufs

    def encode_latents(self, wav1: torch.Tensor, lat: torch.Tensor):
        """wav1 [n] fp32 (n % 512 == 0) -> lat [n / 512][1024] fp32 (DacEncoder, modeling_dac.py:464-475)."""
        n = wav1.shape[-1]
        H, SA, S2 = self._encoder_buffers(n)
        col = S2  # [n][32] fp16, consumed by conv1 before S2 is reused
        _lib.check(self.lib.zmi_dac_im2col7(wav1.data_ptr(), n, col.data_ptr(), self.sptr), "im2col7")
        b0 = self.eblocks[0]
        self._conv(col, n, 32, self.e1_w, self.e1_b, b0["c"], 1, 0, 0, n, 1, 0, n, raw=H, snake=SA,
                   alpha=b0["res"][0]["a1"])
        t = n
        for j, blk in enumerate(self.eblocks):
            c, s, res = blk["c"], blk["stride"], blk["res"]
            for u, dil in enumerate(DILATIONS):
                ru = res[u]
                self._conv(SA, t, c, ru["w1"], ru["b1"], c, 7, dil, -3 * dil, t, 1, 0, t, snake=S2, alpha=ru["a2"])
                last = u == len(DILATIONS) - 1
                self._conv(S2, t, c, ru["w2"], ru["b2"], c, 1, 0, 0, t, 1, 0, t, skip=H, raw=None if last else H,
                           snake=SA, alpha=blk["alpha"] if last else res[u + 1]["a1"])
            tn = t // s
            nxt = self.eblocks[j + 1]["res"][0]["a1"] if j + 1 < len(self.eblocks) else self.e_final_alpha
            # strided conv on the polyphase view of SA ([t][c] read as [t/s][s c]): 3 taps, in_off -1
            self._conv(SA, tn, s * c, blk["w"], blk["b"], 2 * c, 3, 1, -1, tn, 1, 0, tn,
                       raw=H if j + 1 < len(self.eblocks) else None, snake=S2, alpha=nxt)
            SA, S2 = S2, SA
            t = tn
        self._conv(SA, t, self.e2_cin, self.e2_w, self.e2_b, self.e2_cout, 3, 1, -1, t, 1, 0, t, f32=lat)

    @torch.inference_mode()
    def encode(self, wav: torch.Tensor) -> torch.Tensor:
        """[B, 1, 512 T] fp32 waveform -> [B, 9, T] int64 codes (reference autoencoder.py:22-23)."""
        if not self.has_encoder:
            raise RuntimeError("this DAC state_dict has no encoder weights")
        B, ch, n = wav.shape
        assert ch == 1 and n % DAC_HOP == 0, "preprocess() first: mono, length a multiple of 512"
        T = n // DAC_HOP
        out = torch.empty(B, N_CODEBOOKS, T, dtype=torch.int64, device=self.dev)
        cur = torch.cuda.current_stream(self.dev)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            wav = wav.to(self.dev, torch.float32).contiguous()
            lat = torch.empty(T, 1024, dtype=torch.float32, device=self.dev)
            for b in range(B):
                self.encode_latents(wav[b, 0], lat)
                self.quantize(lat, out[b])
        cur.wait_stream(self.stream)
        return out

    def quantize(self, lat: torch.Tensor, codes: torch.Tensor):
        """lat [T][1024] fp32 -> codes [9][T] int64 (residual VQ, modeling_dac.py:283-345)."""
        T = lat.shape[0]
        _lib.check(self.lib.zmi_dac_vq(lat.data_ptr(), T, self.vq_in_w.data_ptr(), self.vq_in_b.data_ptr(),
                                       self.codebooks.data_ptr(), self.cb_n.data_ptr(), self.cb_n2.data_ptr(),
                                       self.proj_w.data_ptr(), self.proj_b.data_ptr(), codes.data_ptr(), self.sptr),
                   "dac_vq")
