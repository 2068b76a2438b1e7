"""DAC decode / encode timing (HIP events on the autoencoder stream) and MFMA roofline fraction.

    python tools/bench_dac.py [frames]
One JSON line per path: ms, frames/s, achieved TFLOP/s (algorithmic FLOP) and the fraction of the
2.5 PFLOP/s dense fp16 MFMA peak."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import MFMA_PEAK_TFLOPS, dac_encode_flop_per_frame  # noqa: E402
from zonos_vibes_amd.autoencoder import DACAutoencoder  # noqa: E402

DEC_FLOP_PER_FRAME = 1_608_302_592  # SURVEY.md §8d (MACs counted by hooks x 2)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    en.synchronize()
    return st.elapsed_time(en) / reps


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 861
    ae = DACAutoencoder("cuda")
    g = torch.Generator().manual_seed(0)
    codes = torch.randint(0, 1024, (1, 9, frames), generator=g).cuda()
    wav = (0.1 * torch.randn(1, 1, frames * 512, generator=g)).cuda()
    for name, fn, fpf in (("dac_decode", lambda: ae.decode(codes), DEC_FLOP_PER_FRAME),
                          ("dac_encode", lambda: ae.encode(wav), dac_encode_flop_per_frame())):
        ms = timed(fn)
        tf = fpf * frames / (ms * 1e-3) / 1e12
        print(json.dumps(dict(path=name, frames=frames, ms=round(ms, 3), frames_per_s=round(frames / ms * 1e3, 1),
                              tflops=round(tf, 1), mfma_frac=round(tf / MFMA_PEAK_TFLOPS, 4))), flush=True)


if __name__ == "__main__":
    main()
