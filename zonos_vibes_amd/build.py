"""Build libzonos_hip.so in-tree with hipcc for gfx950 (no JIT cache, travels with the repo).

    python -m zonos_vibes_amd.build [--force]
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(HERE, "libzonos_hip.so")
SOURCES = ["zmi_gemv.hip"] + [f"zmi_gemv_e{i}.hip" for i in range(6)] + ["zmi_attn.hip", "zmi_attnblk.hip", "zmi_sample.hip",
                                                                        "zmi_dac.hip", "zmi_misc.hip", "zmi_cond.hip",
                                                                        "zmi_mamba.hip", "zmi_mambablk.hip",
                                                                        "zmi_gemm_splitk.hip"]
HEADERS = ["zmi_common.h", "zmi_kernels.h", "zmi_gemv_impl.h", "zmi_attn_merge.h", "zmi_attn_ds.h", "zmi_mamba_step.h",
           "zmi_prefetch.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wno-unused-result",
         f"-I{INCLUDE}", f"-I{CSRC}"]


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True, jobs: int = 8) -> str:
    return _build(SOURCES, LIB, [], force, verbose, jobs)


def _build(sources: list[str], lib: str, link: list[str], force: bool, verbose: bool, jobs: int) -> str:
    objdir = os.path.join(HERE, "build")
    flags = FLAGS
    os.makedirs(objdir, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "zonos_hip.h")]
    objs, procs = [], []
    for src in sources:
        sp = os.path.join(CSRC, src)
        obj = os.path.join(objdir, src.replace(".hip", ".o"))
        objs.append(obj)
        if force or _stale(obj, [sp] + hdrs):
            cmd = [HIPCC, *flags, "-c", sp, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
            if len(procs) >= jobs:
                _wait(procs.pop(0))
    for p in procs:
        _wait(p)
    if force or _stale(lib, objs):
        tmp = lib + ".tmp"  # linked aside, then renamed: a reader never sees a half-written library
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, *link, "-o", tmp]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        os.replace(tmp, lib)
    return lib


def _wait(item):
    src, p = item
    out, _ = p.communicate()
    if p.returncode != 0:
        sys.stderr.write(out.decode(errors="replace"))
        raise RuntimeError(f"hipcc failed on {src}")
    if out.strip():
        sys.stderr.write(out.decode(errors="replace"))


if __name__ == "__main__":
    build(force="--force" in sys.argv)
