"""Weight placement and the C2 step: the engine's packed weights as separate caching-allocator tensors (as loaded,
or cloned) against one contiguous arena with every tensor at a 2 MiB (or 64 KiB) aligned offset, alternating in
one process (one JSON line per measurement)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from zonos_vibes_amd.config import zonos_v01_transformer  # noqa: E402
from zonos_vibes_amd.model import Zonos  # noqa: E402


def leaves(w, out):
    if isinstance(w, torch.Tensor):
        out.append(w)
    elif isinstance(w, dict):
        for v in w.values():
            leaves(v, out)
    elif isinstance(w, list):
        for v in w:
            leaves(v, out)
    return out


def rebuild(w, f):
    if isinstance(w, torch.Tensor):
        return f(w)
    if isinstance(w, dict):
        return {k: rebuild(v, f) for k, v in w.items()}
    if isinstance(w, list):
        return [rebuild(v, f) for v in w]
    return w


def arena(w, align, stagger=0):
    ts = leaves(w, [])
    off, offs = 0, {}
    for i, t in enumerate(ts):
        offs[id(t)] = off + (i * stagger) % max(align, 1)
        off += (t.numel() * t.element_size() + align - 1) // align * align + (align if stagger else 0)
    buf = torch.empty(off, dtype=torch.uint8, device=ts[0].device)

    def place(t):
        o = offs[id(t)]
        v = buf[o:o + t.numel() * t.element_size()].view(t.dtype).view(t.shape)
        v.copy_(t)
        return v
    return rebuild(w, place), buf


def main():
    dev = torch.device("cuda", 0)
    m = Zonos.synthetic(zonos_v01_transformer(), dev, seed=0, zero_eos=True, max_seqlen=bench.LC + bench.N_NEW + 9,
                        max_prefill=bench.LC + 1)
    e = m.engine
    cond = bench.cond_tensor(0, e.d, dev)
    orig = e.w

    def t(label):
        e._build_plan()
        torch.cuda.synchronize()
        us, _ = bench.time_decode_step(m, cond, steps=128)
        print(json.dumps(dict(case=label, us=round(us, 1))), flush=True)

    t("orig")
    layouts = [("4KiB", 4 << 10, 0), ("64KiB", 64 << 10, 0), ("256KiB", 256 << 10, 0), ("1MiB", 1 << 20, 0),
               ("2MiB", 2 << 20, 0), ("2MiB+64KiB stagger", 2 << 20, 64 << 10), ("2MiB+256KiB stagger", 2 << 20, 256 << 10)]
    for rep in range(2):
        for name, al, st in layouts:
            aw, buf = arena(orig, al, st)
            e.w = aw
            t("arena " + name)
            e.w = orig
            del aw, buf
            torch.cuda.synchronize()
        t("orig")
    codes_equal = None
    print(json.dumps(dict(case="done", codes_equal=codes_equal)), flush=True)


if __name__ == "__main__":
    main()
