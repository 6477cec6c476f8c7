"""Build libvqx.so (gfx950) in-tree with hipcc; no CMake, no torch linkage.

Usage: python -m vae_npvc_amd.csrc.build [--force] [-j N]
The shared library lands in vae_npvc_amd/lib/libvqx.so and travels with the
repository snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
ROOT = PKG.parent
OUT_DIR = PKG / "lib"
LIB = OUT_DIR / "libvqx.so"
SOURCES = ["vqx_runtime.hip", "vqx_gemm.hip", "vqx_gemm_fwd.hip", "vqx_gemm_dgrad.hip", "vqx_gemm_wgrad.hip",
           "vqx_gemm_dual.hip",
           "vqx_vq.hip", "vqx_misc.hip"]
HEADERS = ["vqx_common.h", "vqx_gemm_kernel.h", "vqx_gemm_inst.h", "vqx_gemm_pp.h", "vqx_gn_math.h",
           str(ROOT / "include" / "vqx.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=fast-honor-pragmas",
         "-Wno-unused-result", "-I", str(ROOT / "include")]


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return False
    t = target.stat().st_mtime
    return all(Path(d).stat().st_mtime <= t for d in deps)


def _compile(src: Path, obj: Path, force: bool, defines=()):
    deps = [src] + [HERE / h if not os.path.isabs(h) else Path(h) for h in HEADERS]
    if not force and _newer(obj, deps):
        return obj, "up-to-date"
    cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in defines], "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj, "built"


def build(force: bool = False, jobs: int = 8, verbose: bool = True, out: Path = None, defines=()) -> Path:
    """Build libvqx.so; `out` + `defines` make an A/B variant elsewhere (its
    own object directory), loaded with env VQX_LIB."""
    lib = Path(out) if out else LIB
    lib.parent.mkdir(parents=True, exist_ok=True)
    objdir = lib.parent / ("obj" if not out else lib.stem + "_obj")
    objdir.mkdir(exist_ok=True)
    srcs = [HERE / s for s in SOURCES]
    objs = [objdir / (s.stem + ".o") for s in srcs]
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for obj, status in ex.map(lambda so: _compile(so[0], so[1], force, defines), zip(srcs, objs)):
            if verbose:
                print(f"[vqx build] {obj.name}: {status}", flush=True)
    if force or not _newer(lib, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[vqx build] linked {lib}", flush=True)
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    ap.add_argument("--out", default=None, help="A/B variant library path (default: the in-tree lib)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra preprocessor define")
    a = ap.parse_args()
    build(force=a.force, jobs=a.j, out=a.out, defines=a.defines)
    sys.exit(0)
