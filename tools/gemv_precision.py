"""Max error of the decode GEMV's fp32 sums against fp64, relative to sum |x||w| (dot2 rounding check)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zonos_vibes_amd import _lib  # noqa: E402

L = _lib.lib()
for M, N, K in ((2, 3072, 2048), (2, 2048, 8192)):
    g = torch.Generator().manual_seed(1)
    W = ((torch.rand(N, K, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16).cuda()
    X = (torch.rand(M, K, generator=g) * 2 - 1).to(torch.bfloat16).cuda()
    Wp = torch.empty(N * K, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    _lib.check(L.zmi_pack_weight(W.data_ptr(), Wp.data_ptr(), N, K, N, 0, s))
    out = torch.zeros(M, N, device="cuda")
    a = _lib.GemvArgs()
    a.W, a.X, a.M, a.N, a.K, a.ldx, a.out, a.ldo, a.n_valid = Wp.data_ptr(), X.data_ptr(), M, N, K, K, out.data_ptr(), N, N
    _lib.check(L.zmi_gemv_launch(ctypes.byref(a), _lib.EPI_F32, s))
    torch.cuda.synchronize()
    ref = X.double() @ W.double().t()
    mag = X.double().abs() @ W.double().abs().t()
    rel = ((out.double() - ref).abs() / mag).max().item()
    print(json.dumps(dict(M=M, N=N, K=K, max_err_over_sum_abs=rel)), flush=True)
