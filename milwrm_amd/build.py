"""Build the in-tree HIP library ``milwrm_amd/libmilwrm_amd.so`` for gfx950.

One ``hipcc -c`` per source (in parallel), then a shared-library link.  Object
files go to ``build/``; the ``.so`` lands next to this file so it travels with
the repository snapshot to the GPU box.  Re-runs only what changed.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.environ.get("MW_BUILD_DIR") or os.path.join(ROOT, "build")
LIB = os.environ.get("MW_LIB") or os.path.join(HERE, "libmilwrm_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MW_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-but-set-variable"] + os.environ.get("MW_EXTRA_FLAGS", "").split()


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if not _stale(obj, [src] + _headers()):
        return obj, None
    cmd = [HIPCC] + FLAGS + ["-x", "hip", "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")), 16)
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        results = list(ex.map(_compile, srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if _stale(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[milwrm_amd] built {LIB}")
    return LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
