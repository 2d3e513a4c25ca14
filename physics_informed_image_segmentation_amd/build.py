"""Build the gfx950 kernel library in-tree: _lib/libpis.so (hipcc, no JIT cache).

    python -m physics_informed_image_segmentation_amd.build

Staleness is decided by CONTENT, not modification times: a SHA-256 over every source, header,
the compiler flags and the hipcc version is stored next to each object (``*.o.sha``) and the
library (``libpis.so.sha``). A tree copied with fresh or old timestamps (a checkout, a tarball)
rebuilds exactly what changed and never reuses a binary built from other sources.
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ARCH = os.environ.get("PIS_OFFLOAD_ARCH", "gfx950")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC"]


def _digest(paths, extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for p in sorted(paths):
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _fresh(target: str, digest: str) -> bool:
    try:
        with open(target + ".sha") as f:
            return os.path.exists(target) and f.read().strip() == digest
    except OSError:
        return False


def _stamp(target: str, digest: str) -> None:
    with open(target + ".sha", "w") as f:
        f.write(digest + "\n")


def build(verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")))
    headers = sorted(glob.glob(os.path.join(HERE, "csrc", "*.h")) + glob.glob(os.path.join(HERE, "..", "include", "*.h")))
    out_dir = os.path.join(HERE, "_lib")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "libpis.so")
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    try:
        version = subprocess.run([hipcc, "--version"], capture_output=True, text=True).stdout
    except OSError:
        version = ""
    flags = " ".join(FLAGS) + "\n" + version
    objs, obj_digests = [], []
    for s in srcs:
        o = os.path.join(out_dir, os.path.basename(s) + ".o")
        objs.append(o)
        d = _digest([s] + headers, flags)
        obj_digests.append(d)
        if _fresh(o, d):
            continue
        cmd = [hipcc] + FLAGS + ["-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        _stamp(o, d)
    lib_digest = hashlib.sha256("".join(obj_digests).encode() + flags.encode()).hexdigest()
    if _fresh(out, lib_digest):
        return out
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    _stamp(out, lib_digest)
    return out


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
