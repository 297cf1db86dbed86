"""Build the in-tree native library rabia_amd/lib/librabia_gpu.so for gfx950.

Explicit hipcc (no JIT cache): the .so lives in-tree so it travels to the GPU box
with the repo snapshot. `python -m rabia_amd.build [--resource-usage]`.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "librabia_gpu.so")
SOURCES = [os.path.join(CSRC, f) for f in ("rabia_gpu.hip", "rg_shard.hip", "rg_kv.hip", "rg_ingest.hip", "rg_comm.hip")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("rg_common.h", "rg_kernels.h", "rg_ctx.h")] + [
    os.path.join(ROOT, "include", "rabia_gpu.h"), os.path.join(ROOT, "include", "rabia_gpu_debug.h"),
    os.path.join(ROOT, "include", "rabia_kv.h"), os.path.join(ROOT, "include", "rabia_ingest.h")]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, resource_usage: bool = False, verbose: bool = False, out: str = None,
          defines=()) -> str:
    """Compile each translation unit to an object in parallel (hipcc -c), then link.
    out/defines: an experiment build (-D flags) written elsewhere (A/B runs load it
    through RABIA_GPU_LIB)."""
    if out is None and not force and not needs_build() and not resource_usage:
        return LIB
    lib = out or LIB
    obj_dir = os.path.join(LIB_DIR, "obj" if out is None else "obj_" + os.path.basename(out))
    os.makedirs(obj_dir, exist_ok=True)
    base = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result",
            "-I", os.path.join(ROOT, "include")]
    if resource_usage:
        base.insert(1, "-Rpass-analysis=kernel-resource-usage")
    base += [f"-D{d}" for d in defines]
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        cmd = base + ["-c", "-o", obj, src]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
    err_text = ""
    for cmd, proc in procs:
        out, err = proc.communicate()
        err_text += err
        if proc.returncode != 0:
            sys.stderr.write(out + err)
            raise RuntimeError(f"hipcc failed ({proc.returncode}): {' '.join(cmd)}")
    link = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp", *objs]
    proc = subprocess.run(link, capture_output=True, text=True)
    if proc.returncode != 0:
        sys.stderr.write(proc.stdout + proc.stderr)
        raise RuntimeError(f"hipcc link failed ({proc.returncode}): {' '.join(link)}")
    os.replace(lib + ".tmp", lib)
    if verbose and err_text:
        sys.stderr.write(err_text)
    if resource_usage:
        print_resource_usage(err_text)
    return lib


def print_resource_usage(text: str) -> None:
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("sgpr", r"TotalSGPRs: (\d+)"),
                         ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = m.group(1)
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows),
                           capture_output=True, text=True).stdout.split("\n")
    for r, n in zip(rows, names):
        print(f"{n.split('(')[0][:48]:48s} vgpr={r.get('vgpr', '?'):>4} sgpr={r.get('sgpr', '?'):>4} "
              f"scratch={r.get('scratch', '?'):>4} lds={r.get('lds', '?'):>5} occ={r.get('occ', '?')}")


if __name__ == "__main__":
    args = sys.argv[1:]
    out = None
    defs = []
    for a in args:
        if a.startswith("--out="):
            out = a.split("=", 1)[1]
        elif a.startswith("-D"):
            defs.append(a[2:])
    print(build(force=True, resource_usage="--resource-usage" in args, verbose="-v" in args, out=out,
                defines=defs))
