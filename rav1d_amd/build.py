"""Build the gfx950 DSP library in-tree: rav1d_amd/librav1d_amd.so.

hipcc cross-compiles for gfx950 without a GPU. Every translation unit is compiled to an
object in rav1d_amd/build/ (parallel), then linked. No JIT, no torch extension cache: the
.so travels with the repo snapshot to the GPU box.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# MI_BUILD_VARIANT=name builds an experiment variant (librav1d_amd_<name>.so, with
# MI_EXTRA_FLAGS added) next to the product library; load it with MI_LIB=<path>.
_VAR = os.environ.get("MI_BUILD_VARIANT", "")
OUT = os.path.join(HERE, f"librav1d_amd_{_VAR}.so" if _VAR else "librav1d_amd.so")
BUILD = os.path.join(HERE, f"build_{_VAR}" if _VAR else "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-I" + os.path.join(HERE, "..", "include")] + os.environ.get("MI_EXTRA_FLAGS", "").split()


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                  if f.endswith(".hip") or f.endswith(".cpp"))


def _stale(obj, src):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    deps += [os.path.join(HERE, "..", "include", h) for h in ("mi_av1dsp.h", "mi_av1dec.h", "mi_av1out.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if not _stale(obj, src):
        return obj, None
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd.insert(1, "-xhip")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sources()
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        res = list(ex.map(_compile, srcs))
    errs = [e for _, e in res if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in res]
    if not os.path.exists(OUT) or any(os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", OUT]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
