"""Decomposition / A-B variants of libspectralmc_hip.so without hooks in the product sources.

Copies spectralmc_amd/csrc (+ include/) to a scratch tree, applies literal string replacements to one
source file, and builds tools/micro/libsmc_<name>.so (load it with SMC_LIB_PATH=...).  Build on the
CPU side before a gpurun call.

    python tools/micro/make_variant.py NAME FILE OLD NEW [FILE OLD NEW ...] [--flags "-DX=1"]
    python tools/micro/make_variant.py base            # the unmodified sources
"""

from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRCS = ["capi", "sobol", "gbm", "cvnn", "cvnn_mfma", "basket"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("edits", nargs="*", help="FILE OLD NEW triples (literal, each OLD must occur once)")
    ap.add_argument("--flags", default="")
    a = ap.parse_args()
    if len(a.edits) % 3:
        sys.exit("edits come in FILE OLD NEW triples")
    work = os.path.join("/tmp", f"smc_variant_{a.name}")
    shutil.rmtree(work, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "spectralmc_amd", "csrc"), os.path.join(work, "spectralmc_amd", "csrc"),
                    ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(work, "include"))
    csrc = os.path.join(work, "spectralmc_amd", "csrc")
    for i in range(0, len(a.edits), 3):
        f, old, new = a.edits[i:i + 3]
        p = os.path.join(csrc, f)
        s = open(p).read()
        if s.count(old) != 1:
            sys.exit(f"{f}: {old[:60]!r} occurs {s.count(old)} times")
        open(p, "w").write(s.replace(old, new))

    def build(src: str) -> None:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--offload-compress", "-fvisibility=hidden",
               "-munsafe-fp-atomics", *a.flags.split(), "-c", f"{src}.hip", "-o", f"{src}.o"]
        subprocess.run(cmd, cwd=csrc, check=True)

    with ThreadPoolExecutor(6) as ex:
        list(ex.map(build, SRCS))
    os.makedirs(os.path.join(ROOT, "tools", "micro", "v"), exist_ok=True)  # travels with gpurun: delete after use
    out = os.path.join(ROOT, "tools", "micro", "v", f"libsmc_{a.name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "--offload-arch=gfx950", "-o", out,
                    *[f"{s}.o" for s in SRCS]], cwd=csrc, check=True)
    print("built", out)


if __name__ == "__main__":
    main()
