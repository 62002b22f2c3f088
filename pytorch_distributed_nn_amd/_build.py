"""In-tree native build for the framework.

Two shared libraries are produced inside the package (``pytorch_distributed_nn_amd/_lib``) so that
they travel with the repo snapshot to the GPU box and are visibly loaded by the test/smoke processes:

* ``libpdnn_kernels.so`` – every ``csrc/kernels/*.hip`` file, compiled by ``hipcc`` for gfx950 only.
  The kernels expose ``extern "C"`` launchers taking raw device pointers + a ``hipStream_t`` so the
  Python side (``ops/_backend.py``) can call them on torch's current stream (also under graph capture).
* ``libpdnn_runtime.so`` – the host runtime (``csrc/runtime/*.cpp``): TCP control-plane store,
  parameter-server coordinator state machine, IDX reader, native MLP trainer, timeline writer.
  Plain C++17 (g++), no GPU dependency, so it is unit-tested on the CPU-only dev box.

Objects are rebuilt only when their source (or a header) is newer.  ``python -m
pytorch_distributed_nn_amd._build`` builds both.
"""
from __future__ import annotations

import concurrent.futures as cf
import contextlib
import fcntl
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = Path(__file__).resolve().parent
LIBDIR = PKG / "_lib"
BUILD = ROOT / "build"
ARCH = os.environ.get("PDNN_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CXX = shutil.which("g++") or "c++"

HIP_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
    "-munsafe-fp-atomics", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
    "-Wno-unused-but-set-variable", "-Werror=return-type",
    f"-I{ROOT / 'csrc' / 'include'}", f"-I{ROOT / 'csrc' / 'kernels'}",
]
# Per-file extra flags.  MFMA accumulators in plain VGPRs (no AGPR copies): the attention kernels mix
# every MFMA result with VALU work (softmax, masking, bf16 packing), and in AGPR form the compiler spent
# ~400 v_accvgpr_read/write per two key tiles; VGPR form cut the forward's vector instruction count by 30%
# and raised occupancy (fwd 2 -> 3 waves/SIMD, dq 3 -> 4).  In the GEMM engines only the 64-column glds
# tiles held AGPRs; VGPR form there measured +1.9% on the ResNet-50 step (7142/7199 -> 7312/7293 img/s).
VGPR_FORM = ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
KERNEL_FILE_FLAGS = {"attention.hip": VGPR_FORM, "gemm_mfma.hip": VGPR_FORM, "gemm_pp.hip": VGPR_FORM}   # gemm: +1.9% ResNet-50
CXX_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter",
             "-pthread", f"-I{ROOT / 'csrc' / 'include'}", f"-I{ROOT / 'csrc' / 'runtime'}"]


def _newer(src: Path, dst: Path, deps) -> bool:
    if not dst.exists():
        return True
    t = dst.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


@contextlib.contextmanager
def build_lock():
    """Exclusive inter-process lock around a build: torchrun ranks that all find the library missing
    serialise here instead of compiling into the same object files."""
    LIBDIR.mkdir(parents=True, exist_ok=True)
    with open(LIBDIR / ".build.lock", "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)


def stale_sources(kind: str = "kernels"):
    """Sources (or headers) newer than the built library, [] when it is up to date (or missing)."""
    if kind == "kernels":
        d, out, pats = ROOT / "csrc" / "kernels", LIBDIR / "libpdnn_kernels.so", ("*.hip", "*.h")
    else:
        d, out, pats = ROOT / "csrc" / "runtime", LIBDIR / "libpdnn_runtime.so", ("*.cpp", "*.h")
    if not out.exists() or not d.exists():
        return []
    t = out.stat().st_mtime
    return [str(f) for pat in pats for f in d.glob(pat) if f.stat().st_mtime > t + 1.0]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(map(str, cmd)) + "\n" + r.stdout)
    return r.stdout


def _build_lib(srcs, compiler, flags, out: Path, objdir: Path, deps, link_extra=(), jobs=None, file_flags=None):
    objdir.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    objs, todo = [], []
    for s in srcs:
        o = objdir / (s.stem + ".o")
        objs.append(o)
        if _newer(s, o, deps):
            todo.append((s, o))
    jobs = jobs or min(8, os.cpu_count() or 4)
    pid = os.getpid()
    ff = file_flags or {}

    def compile_one(s, o):      # private temp object, renamed into place: readers never see a partial file
        tmp = o.with_name(f"{o.stem}.{pid}.tmp.o")
        _run([compiler, *flags, *ff.get(s.name, []), "-c", str(s), "-o", str(tmp)])
        os.replace(tmp, o)

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(compile_one, s, o) for s, o in todo]
        for f in futs:
            f.result()
    if todo or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        tmp = out.with_name(f"{out.name}.{pid}.tmp")
        _run([compiler, *flags, "-shared", *map(str, objs), "-o", str(tmp), *link_extra])
        os.replace(tmp, out)
    return out


def build_kernels(verbose=False) -> Path:
    with build_lock():
        return _build_kernels()


def _build_kernels() -> Path:
    kdir = ROOT / "csrc" / "kernels"
    srcs = sorted(kdir.glob("*.hip"))
    deps = list(kdir.glob("*.h")) + list((ROOT / "csrc" / "include").glob("*.h"))
    return _build_lib(srcs, HIPCC, HIP_FLAGS, LIBDIR / "libpdnn_kernels.so", BUILD / "kernels", deps,
                      file_flags=KERNEL_FILE_FLAGS)


def build_runtime(verbose=False, sanitize: str | None = None) -> Path:
    with build_lock():
        return _build_runtime(sanitize)


def _build_runtime(sanitize: str | None = None) -> Path:
    rdir = ROOT / "csrc" / "runtime"
    srcs = sorted(rdir.glob("*.cpp"))
    deps = list(rdir.glob("*.h")) + list((ROOT / "csrc" / "include").glob("*.h"))
    flags = list(CXX_FLAGS)
    name = "libpdnn_runtime.so"
    objdir = BUILD / "runtime"
    if sanitize:
        flags += [f"-fsanitize={sanitize}", "-g", "-O1", "-fno-omit-frame-pointer"]
        name = f"libpdnn_runtime_{sanitize}.so"
        objdir = BUILD / f"runtime_{sanitize}"
    return _build_lib(srcs, CXX, flags, LIBDIR / name, objdir, deps, link_extra=["-pthread"])


def build_tools() -> Path:
    """``_lib/pdnn_mlp``: the native MLP command-line driver (csrc/tools), statically linking the runtime
    objects."""
    build_runtime()
    rdir = ROOT / "csrc" / "runtime"
    objs = sorted(o for o in (BUILD / "runtime").glob("*.o") if ".tmp" not in o.name)
    src = ROOT / "csrc" / "tools" / "pdnn_mlp.cpp"
    out = LIBDIR / "pdnn_mlp"
    deps = list(rdir.glob("*.h")) + objs
    if _newer(src, out, deps):
        _run([CXX, *CXX_FLAGS, str(src), *map(str, objs), "-o", str(out), "-pthread"])
    return out


def build_all():
    return build_kernels(), build_runtime(), build_tools()


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "kernels"):
        print(build_kernels())
    if which in ("all", "runtime"):
        print(build_runtime())
    if which in ("all", "tools"):
        print(build_tools())
    if which.startswith("sanitize="):
        print(build_runtime(sanitize=which.split("=", 1)[1]))
