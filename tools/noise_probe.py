"""How often each HIP kernel's bf16 output differs from the correctly rounded value, next to the
reference's CPU ops (F.linear / SDPA on bf16 tensors) — the per-op sources of GPU-vs-reference
logit noise. One JSON line per op.

    python tools/noise_probe.py
"""
import ctypes
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_kernels import _attention, gemv, rnd  # noqa: E402
from zonos_vibes_amd import _lib as L  # noqa: E402


def flips(a, exact):
    return (a.float().cpu() != exact.to(torch.bfloat16).float()).float().mean().item()


def main():
    torch.set_num_threads(8)
    for (M, N, K) in [(2, 2048, 2048), (2, 2048, 8192), (2, 4096, 2048)]:
        W, X = rnd(N, K, scale=0.05, seed=1), rnd(M, K, seed=2)
        out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
        gemv(W, X, L.EPI_STORE, out, N)
        exact = X.double().cpu() @ W.double().cpu().t()
        cpu = F.linear(X.cpu(), W.cpu())
        f32 = torch.zeros(M, N, dtype=torch.float32, device="cuda")
        gemv(W, X, L.EPI_F32, f32, N)
        print(json.dumps(dict(op="gemv", M=M, N=N, K=K, gpu_flip=flips(out, exact), cpu_flip=flips(cpu, exact),
                              gpu_f32_relerr=((f32.double().cpu() - exact).abs() / exact.abs().clamp_min(1e-3)).median().item())))
    from oracle.attention_cpu import attend
    H, Hkv, hd, smax = 16, 4, 128, 1024
    positions = [100, 600, 1000]
    kc, vc = rnd(3, Hkv, smax, hd, seed=20), rnd(3, Hkv, smax, hd, seed=21)
    q = rnd(3, H * hd, scale=2.0, seed=22)
    out = _attention(q, kc, vc, positions)
    g = c = n = 0
    for r, p in enumerate(positions):
        ex = torch.stack([torch.nn.functional.scaled_dot_product_attention(
            q[r].view(H, hd)[h].double().cpu().view(1, 1, hd), kc[r, h // 4, : p + 1].double().cpu().unsqueeze(0),
            vc[r, h // 4, : p + 1].double().cpu().unsqueeze(0)).view(hd) for h in range(H)])
        blk = attend(q[r].view(H, hd).cpu(), kc[r].cpu(), vc[r].cpu(), p)
        sd = F.scaled_dot_product_attention(q[r].view(1, H, 1, hd).cpu(), kc[r, :, : p + 1].cpu().unsqueeze(0),
                                            vc[r, :, : p + 1].cpu().unsqueeze(0), enable_gqa=True).view(H, hd)
        gg = out[r].view(H, hd).cpu()
        g += (gg == sd).sum().item()
        c += (blk == sd).sum().item()
        n += sd.numel()
    print(json.dumps(dict(op="attention", gpu_equal_torch_cpu=g / n, oracle_equal_torch_cpu=c / n)))


if __name__ == "__main__":
    main()
