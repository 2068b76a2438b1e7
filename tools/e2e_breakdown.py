"""Where the C2 utterance's wall time goes: prefill, decode loop, codes readback, DAC decode.

    python tools/e2e_breakdown.py [--new-tokens 861] [--chunk 128]

Each phase is bracketed by stream synchronisation and timed on the host clock; the decode loop
is also split into host enqueue time (zmi_graph_launch returning) vs device time. One JSON line.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import LC, cond_tensor  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.engine import SamplingParams  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--new-tokens", type=int, default=861)
    ap.add_argument("--chunk", type=int, default=128)
    args = ap.parse_args()
    n_new = args.new_tokens
    dev = torch.device("cuda", 0)
    cfg = zonos_v01_transformer()
    m = Zonos.synthetic(cfg, dev, seed=0, zero_eos=True, max_seqlen=LC + n_new + 9, max_prefill=LC + 1)
    cond = cond_tensor(1, cfg.backbone.d_model, dev)
    e = m.engine
    params = SamplingParams(temperature=0.0, cfg_scale=2.0)
    res = {}
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e.prefill(0, cond, None, n_new, params)
        e.stream.synchronize()
        t1 = time.perf_counter()
        enq = 0.0
        steps = 0
        while steps < n_new + 8:
            n = min(args.chunk, n_new + 8 - steps)
            a = time.perf_counter()
            e.step(n)
            enq += time.perf_counter() - a
            steps += n
            if not e.slot_state(0)["active"]:
                break
        t2 = time.perf_counter()
        codes = e.read_codes(0)
        e.release(0)
        t3 = time.perf_counter()
        wav = m.autoencoder.decode(codes)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        res = {"prefill_ms": (t1 - t0) * 1e3, "decode_ms": (t2 - t1) * 1e3, "decode_steps": steps,
               "decode_us_per_step": (t2 - t1) * 1e6 / steps, "graph_enqueue_ms": enq * 1e3,
               "readback_ms": (t3 - t2) * 1e3, "dac_ms": (t4 - t3) * 1e3, "total_ms": (t4 - t0) * 1e3,
               "frames": int(codes.shape[-1]), "wav": int(wav.shape[-1]), "rep": rep}
    res["rtf"] = res["frames"] * 512 / 44100 / (res["total_ms"] / 1e3)
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
