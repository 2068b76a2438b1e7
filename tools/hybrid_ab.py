"""A/B of a hybrid (C4) engine switch on one box: utterance wall time and decode step, alternating.

    python tools/hybrid_ab.py attn_block 300
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import LC, cond_tensor  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_hybrid  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    flag, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 300
    dev = torch.device("cuda", 0)
    cfg = zonos_v01_hybrid()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=LC + n + 9, max_prefill=LC + 1)
    cond = cond_tensor(1, cfg.backbone.d_model, dev)
    # "name" toggles a bool; "name=v1,v2" alternates integer values
    vals = [int(v) for v in flag.split("=")[1].split(",")] if "=" in flag else [True, False]
    flag = flag.split("=")[0]
    res = {v: [] for v in vals}
    for rep in range(3):
        for on in vals:
            setattr(m.engine, flag, on)
            m.engine._build_plan()
            m.generate(cond, max_new_tokens=n, sampling_params=dict(temperature=0.0), progress_bar=False, chunk=128)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            codes = m.generate(cond, max_new_tokens=n, sampling_params=dict(temperature=0.0), progress_bar=False,
                               chunk=128)
            torch.cuda.synchronize()
            res[on].append(round((time.perf_counter() - t0) * 1e3, 1))
            assert codes.shape[-1] == n
    print(json.dumps({"flag": flag, "frames": n, "generate_ms": {str(k): v for k, v in res.items()}}))


if __name__ == "__main__":
    main()
