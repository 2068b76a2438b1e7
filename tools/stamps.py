"""In-kernel timeline of the decode GEMV (diagnostic build, -DZMI_STAMPS): where a launch's time goes.

    python -m zonos_vibes_amd.build --stamps && ZMI_LIB_PATH=zonos_vibes_amd/libzonos_hip_stamps.so \
        python tools/stamps.py

Stamps (s_memrealtime, 10 ns ticks) per block: 0 entry, 1 weights issued, 2 activations landed,
3 LayerNorm done, 4 dot products done, 5 reduction barrier, 6 end. Reports the launch span and, per
segment, median and max over blocks (in us), plus the dispatch skew of block entries.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402

assert "stamps" in _lib.LIB_PATH, "run with ZMI_LIB_PATH=.../libzonos_hip_stamps.so"
L = _lib.lib()
dev = "cuda"
SHAPES = {"qkv": (3072, 2048, _lib.EPI_QKV, True), "out": (2048, 2048, _lib.EPI_RESIDUAL, False),
          "fc1": (16384, 2048, _lib.EPI_SWIGLU, True), "fc2": (2048, 8192, _lib.EPI_RESIDUAL, False),
          "heads": (9248, 2048, _lib.EPI_LOGITS, True)}


def run(name, M=2, G=0):
    N, K, epi, ln = SHAPES[name]
    copies = max(4, (1200 << 20) // (N * K * 2) + 1)
    Ws = [torch.empty(N * K, dtype=torch.bfloat16, device=dev).uniform_(-0.05, 0.05) for _ in range(copies)]
    X = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.zeros(M, 9 * 1026 if epi == _lib.EPI_LOGITS else max(N, K), device=dev)
    outb = torch.zeros(M, max(N, K), device=dev).to(torch.bfloat16)
    lw, lb = torch.ones(K, device=dev).to(torch.bfloat16), torch.zeros(K, device=dev).to(torch.bfloat16)
    nb = N // 8
    st = torch.zeros(nb * 8, dtype=torch.int64, device=dev)
    kc = torch.zeros(M, 4, 64, 128, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    rope = torch.zeros(16384, 64, 2, device=dev)
    rk = torch.arange(M, dtype=torch.int32, device=dev)
    rp = torch.full((M,), 5, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    args = []
    for W in Ws:
        a = _lib.GemvArgs()
        a.W, a.X, a.M, a.N, a.K, a.ldx = W.data_ptr(), X.data_ptr(), M, N, K, K
        a.ksplit = -G if G else 0
        if ln:
            a.ln_w, a.ln_b, a.eps = lw.data_ptr(), lb.data_ptr(), 1e-5
        if epi == _lib.EPI_LOGITS:
            a.out, a.ldo, a.n_valid = out.data_ptr(), 0, 9 * 1026
        else:
            a.out, a.ldo, a.n_valid = outb.data_ptr(), (N // 2 if epi == _lib.EPI_SWIGLU else 2048), N
        if epi == _lib.EPI_QKV:
            a.row_kv, a.row_pos, a.k_cache, a.v_cache = rk.data_ptr(), rp.data_ptr(), kc.data_ptr(), vc.data_ptr()
            a.smax, a.hq, a.hkv, a.hd, a.rope = 64, 16, 4, 128, rope.data_ptr()
        a.slab = st.data_ptr()
        args.append(a)
    sp = s.cuda_stream
    with torch.cuda.stream(s):
        for a in args:
            _lib.check(L.zmi_gemv_launch(ctypes.byref(a), epi, sp))
    s.synchronize()
    _lib.check(L.zmi_graph_begin(sp))
    with torch.cuda.stream(s):
        for a in args:
            _lib.check(L.zmi_gemv_launch(ctypes.byref(a), epi, sp))
    g = ctypes.c_void_p()
    _lib.check(L.zmi_graph_end(sp, ctypes.byref(g)))
    _lib.check(L.zmi_graph_launch(g, 3, sp))
    s.synchronize()
    L.zmi_graph_destroy(g)
    t = st.view(-1, 8).cpu().numpy().astype(np.int64)
    blocks = t.shape[0] if not G else (nb + G - 1) // G
    t = t[:blocks]
    t0 = t[:, 0].min()
    rel = (t - t0) / 100.0  # us
    seg = {f"s{i}-{i + 1}": rel[:, i + 1] - rel[:, i] for i in range(6)}
    res = dict(shape=name, G=G, blocks=blocks, span_us=round(float(rel[:, 6].max()), 2),
               entry_skew_us=round(float(rel[:, 0].max()), 2),
               last_entry_to_end=round(float(rel[:, 6].max() - rel[:, 0].max()), 2))
    for k, v in seg.items():
        res[k] = [round(float(np.median(v)), 2), round(float(v.max()), 2)]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    for n in SHAPES:
        run(n)
        torch.cuda.empty_cache()
    run("fc1", G=2)
    run("qkv", G=2)
