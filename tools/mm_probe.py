"""hipBLASLt (torch.matmul) timing for the hybrid prefill's plain GEMM shapes, bf16: [M x K] x [K x N]."""
import json
import torch

dev = torch.device("cuda", 0)
for M, K, N in ((322, 2048, 8512), (322, 4096, 2048), (322, 2048, 6144), (322, 2048, 2048)):
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(a, w.t())
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(20):
        torch.matmul(a, w.t())
    en.record()
    en.synchronize()
    us = st.elapsed_time(en) * 1000 / 20
    print(json.dumps(dict(M=M, K=K, N=N, us=round(us, 2), tflops=round(2 * M * K * N / us / 1e6, 1))), flush=True)
